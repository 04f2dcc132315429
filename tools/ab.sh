#!/bin/bash
# A/B timing of fresh-kernel variants (GPU box): GPU tests of the product library first (unless
# AB_TESTS=0), then every lib/exp/libpvac_hip_*.so timed twice in alternating order (tools/exp_fresh.py).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
if [ "${AB_TESTS:-1}" = "1" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/ab_pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
L=(pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_*.so)
timeout -k 10 500 python tools/exp_fresh.py "${L[@]}" "${L[@]}" > gpurun_out/ab_times.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/ab_times.log
