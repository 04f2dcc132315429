for k in 1 2 3; do
  PVAC_FRESH_PER_CU=$k timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/percu_$k.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/percu_$k.log').read().strip().splitlines()[-1]); print($k, round(d['roofline']['avg_kernel_ms'],3), round(d['ms_per_step'],3))"
done
