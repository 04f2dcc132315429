#!/bin/bash
# general-path iteration: gpu tests, then the cfg-4 chain side measurement
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_q.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --only chain > gpurun_out/chain.log 2>&1 || exit $?
tail -1 gpurun_out/chain.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ct_mul_per_s'], d['chain_seconds'], [round(x) for x in d['ms_by_step']])"
