#!/bin/bash
# cfg-4 chain A/B (GPU box): gpu tests of the product library, then bench.py --only chain with the
# product library and with each lib/exp/libpvac_hip_<name>.so given swapped in, alternating
# (new, name1, name2, ..., new, name1, ...).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
[ $# -ge 1 ] || { echo "usage: gpu_chain_ab.sh variant [variant...]"; exit 2; }
L=pvac_hfhe_cppbyv_amd/lib
if [ "${AB_TESTS:-1}" = "1" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/ab_pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
cp $L/libpvac_hip.so gpurun_out/lib_new.so || exit 1
for pass in 1 2; do
  for v in new "$@"; do
    # a variant "env:NAME=VALUE" runs the product library with that environment variable
    envv=""
    if [ $v = new ] || [ "${v#env:}" != "$v" ]; then cp gpurun_out/lib_new.so $L/libpvac_hip.so; else cp $L/exp/libpvac_hip_$v.so $L/libpvac_hip.so; fi
    [ "${v#env:}" != "$v" ] && envv="${v#env:}"
    tag=$(echo "$v" | tr -c 'A-Za-z0-9_\n' '_')
    env $envv timeout -k 10 300 python bench.py --only chain > gpurun_out/chain_$tag$pass.log 2>&1 || { cp gpurun_out/lib_new.so $L/libpvac_hip.so; exit 1; }
    echo -n "$v$pass "
    tail -1 gpurun_out/chain_$tag$pass.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('errors'), round(d['ct_mul_per_s']), round(d['chain_seconds'],3), [round(x) for x in d['stream_ms_by_step']], d.get('oracle_sample_ok'))"
  done
done
cp gpurun_out/lib_new.so $L/libpvac_hip.so
rm -f gpurun_out/lib_new.so
