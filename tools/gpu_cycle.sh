#!/bin/bash
# usage: gpu_cycle.sh TAG  -> tests, bench, diag
TAG=$1
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout=300 -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/bench_$TAG.log 2>&1 || exit $?
grep -o '"value": [0-9.e+]*\|"avg_kernel_ms": [0-9.]*\|"frac": [0-9.]*' gpurun_out/bench_$TAG.log
timeout -k 10 200 python tools/diag_fresh.py > gpurun_out/diag_$TAG.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/diag_$TAG.log | python3 -c "import json,sys; d=json.load(sys.stdin); print(round(d['ticks_per_pair_per_wg'])); [print(' ', k, v['ticks_per_pair']) for k,v in d['phases'].items()]"
