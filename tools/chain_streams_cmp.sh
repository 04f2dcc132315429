#!/bin/bash
# cfg-4 chain throughput for several (host threads / HIP streams, chunk) settings (GPU box)
set -o pipefail
CFGS=${CFGS:-"1:4096 2:2048 4:1024 3:2048 2:2048 4:1024"}
for c in $CFGS; do
  s=${c%%:*}; k=${c##*:}
  timeout -k 10 300 python bench.py --only chain --chain-streams $s --chain-chunk $k > gpurun_out/cc_$s_$k.log 2>&1 || { tail -5 gpurun_out/cc_$s_$k.log; exit 1; }
  echo -n "streams $s chunk $k: "; tail -1 gpurun_out/cc_$s_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('errors'), round(d['ct_mul_per_s']), round(d['chain_seconds'],3), round(sum(d['stream_ms_by_step'])), d.get('peak_hbm_reserved_gb'), d.get('oracle_sample_ok'), d['invariant']['invariant_ok'])"
done
