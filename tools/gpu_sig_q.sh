#!/bin/bash
# sigma iteration: all gpu tests (sigma digests / golden .ct bytes), then the with-sigma side measurement
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --only sigma > gpurun_out/sig.log 2>&1 || exit $?
tail -1 gpurun_out/sig.log
