#!/bin/bash
# cfg-4 chain timing vs chunk size (GPU box): bench.py --only chain at each --chain-chunk given
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
for c in "$@"; do
  timeout -k 10 300 python bench.py --only chain --chain-chunk $c > gpurun_out/chain_c$c.log 2>&1 || exit $?
  echo -n "chunk $c: "
  tail -1 gpurun_out/chain_c$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('errors'), round(d['ct_mul_per_s']), round(d['chain_seconds'],3), [round(x) for x in d['stream_ms_by_step']])"
done
