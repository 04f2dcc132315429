#!/bin/bash
# ct_add iteration: all gpu tests, then the batched ct_add / ct_sub side measurement
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_a.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_a.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --only add > gpurun_out/add.log 2>&1 || exit $?
tail -1 gpurun_out/add.log
