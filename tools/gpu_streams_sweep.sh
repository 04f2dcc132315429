#!/bin/bash
# cfg-4 leg at several worker-stream counts and chunk sizes (check-free timed pass only)
set -o pipefail
R="$GRAFT_REPO_ROOT"
D="$R/gpurun_out/sweep"
mkdir -p "$D"
for cfg in "4 1024" "6 1024" "8 1024" "8 512" "4 2048" "6 512"; do
  set -- $cfg
  timeout -k 10 200 python3 "$R/bench.py" --only chain --chain-no-check --chain-streams $1 --chain-chunk $2 > "$D/s$1_c$2.log" 2>&1 || { tail -5 "$D/s$1_c$2.log"; exit 1; }
  echo "streams $1 chunk $2: $(tail -1 "$D/s$1_c$2.log" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d.get("extras",d).get("cfg4_chain",d); print(round(c["ct_mul_per_s"]), round(c["chain_seconds"],3))')"
done
