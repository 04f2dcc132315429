#!/bin/bash
# quick GPU iteration: gpu tests, then the headline bench without CPU baseline / side fields
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_q.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/bench_q.log 2>&1 || exit $?
grep -o '"value": [0-9.e+]*\|"avg_kernel_ms": [0-9.]*\|"frac": [0-9.]*' gpurun_out/bench_q.log
