#!/bin/bash
# usage: gpu_ab.sh TAG -> gpu tests, then bench of the fresh kernel at 3 and 2 workgroups per CU, diag
TAG=$1
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout=300 -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
for pc in 3 2; do
  PVAC_FRESH_PER_CU=$pc timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/bench_${TAG}_pc$pc.log 2>&1 || exit $?
  echo "per_cu=$pc"; grep -o '"value": [0-9.e+]*\|"avg_kernel_ms": [0-9.]*\|"frac": [0-9.]*' gpurun_out/bench_${TAG}_pc$pc.log
done
timeout -k 10 200 python tools/diag_fresh.py > gpurun_out/diag_$TAG.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/diag_$TAG.log | python3 -c "import json,sys; d=json.load(sys.stdin); print(round(d['ticks_per_pair_per_wg'])); [print(' ', k, v['ticks_per_pair']) for k,v in d['phases'].items()]"
