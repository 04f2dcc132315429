#!/bin/bash
# single-stream kernel trace of the cfg-4 leg (isolated kernel durations of the timed pass) and the
# WRITE_SIZE / FETCH_SIZE passes of the chain, for the library in the tree
set -o pipefail
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
D="$R/gpurun_out/r4q"
mkdir -p "$D"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu "$R/tests/test_gpu_large.py" \
    "$R/tests/test_gpu_chain.py" > "$D/pytest_large_chain.log" 2>&1 || { tail -30 "$D/pytest_large_chain.log"; exit 1; }
tail -3 "$D/pytest_large_chain.log"
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$D/chain1" -o run --output-format csv \
    -- python3 "$R/bench.py" --only chain --chain-no-check --chain-streams 1 --chain-inputs 8192 > "$D/chain1.log" 2>&1) || { tail -20 "$D/chain1.log"; exit 1; }
T=$(find "$D/chain1" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/chain_window.py" "$T" "$D/chain1.log" "$D/chain1_window.json" | head -30
CHAIN_INPUTS=8192 bash "$R/tools/pmc_chain.sh" > "$D/pmc_chain.log" 2>&1; cp "$R/gpurun_out/pmc_chain/summary.json" "$D/pmc_chain_summary.json"
python3 - "$D/pmc_chain_summary.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in sorted(d.items(), key=lambda kv: -(kv[1].get("ms_by_pass", {}).get("p1", 0) if isinstance(kv[1], dict) else 0))[:10]:
    if k == "_total": continue
    print(k[:34], v.get("ms_by_pass", {}).get("p1"), "W GB", round(v.get("hbm_write_bytes", 0) / 1e9, 1), "R GB", round(v.get("hbm_read_bytes_corrected", 0) / 1e9, 1))
print(d["_total"]["hbm_write_bytes"] / 1e9, d["_total"]["hbm_read_bytes_corrected"] / 1e9)
PY
