#!/bin/bash
# cfg-4 chain profile (GPU box): kernel-trace stats of bench.py --only chain (one chunk), plus the
# per-step timing line. Output: gpurun_out/chain_<TAG>/
TAG=${1:-x}
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/chain_$TAG"
mkdir -p "$OUT"
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --only chain --chain-inputs ${CHAIN_INPUTS:-4096} --chain-chunk ${CHAIN_CHUNK:-4096} --chain-check 0 --chain-ref 0 > "$OUT/chain.log" 2>&1) || exit $?
tail -1 "$OUT/chain.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["stream_ms_by_step"], d["ct_mul_per_s"])' 
f=$(find "$OUT" -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:14]: print(r['Name'][:70], r['Calls'], round(float(r['TotalDurationNs'])/1e6,2),'ms total', round(float(r['AverageNs'])/1e3,1),'us avg')"
