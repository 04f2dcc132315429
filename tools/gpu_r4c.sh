#!/bin/bash
# round 4: chain API + direct mode validation and measurement, single-call latency, fresh-kernel and
# sigma A/B variants
set -o pipefail
bash tools/gpu_r4b.sh r4b || exit $?
timeout -k 10 120 tests/cpp/build/test_adapter --time-single 100 > gpurun_out/r4b/single.log 2>&1; cat gpurun_out/r4b/single.log
AB_TESTS=0 bash tools/ab.sh
L=(pvac_hfhe_cppbyv_amd/lib/exp_sig/libpvac_hip_*.so)
timeout -k 10 400 python tools/exp_sigma.py "${L[@]}" "${L[@]}" > gpurun_out/r4b/sig_ab.log 2>&1; grep -v amdgpu gpurun_out/r4b/sig_ab.log | tail -6
