#!/bin/bash
# enc_value iteration: enc / PRF parity tests, then the enc_value side measurement
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_enc.py tests/test_gpu_dec.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_e.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_e.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --only enc > gpurun_out/enc.log 2>&1 || exit $?
tail -1 gpurun_out/enc.log
