#!/bin/bash
# general-path iteration: gpu tests, then the cfg-4 chain side measurement (extra args to bench.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_q.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --only chain "$@" > gpurun_out/chain.log 2>&1 || exit $?
tail -1 gpurun_out/chain.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('errors'), d['streams'], round(d['ct_mul_per_s']), round(d['ct_mul_per_s_incl_enc']), round(d['chain_seconds'],3), round(d['enc_seconds'],3), [round(x) for x in d['stream_ms_by_step']])"
