#!/bin/bash
# full GPU suite, smoke, default bench line, then the chain's PMC passes (timed chain only)
set -o pipefail
R="$GRAFT_REPO_ROOT"
bash "$R/tools/gpu_quick4.sh" r4h || exit 1
CHAIN_INPUTS=4096 timeout -k 10 600 bash "$R/tools/pmc_chain.sh" > "$R/gpurun_out/r4h/pmc_chain.log" 2>&1 || { tail -20 "$R/gpurun_out/r4h/pmc_chain.log"; exit 1; }
cp "$R/gpurun_out/pmc_chain/summary.json" "$R/gpurun_out/r4h/pmc_chain_summary.json"
python3 - "$R/gpurun_out/r4h/pmc_chain_summary.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in sorted(d.items(), key=lambda kv: -(kv[1].get("ms_by_pass", {}).get("p1", 0) if isinstance(kv[1], dict) else 0))[:8]:
    if k == "_total": continue
    print(k[:34], v.get("ms_by_pass", {}).get("p1"), "W GB", round(v.get("hbm_write_bytes", 0) / 1e9, 1), "R GB", round(v.get("hbm_read_bytes_corrected", 0) / 1e9, 1))
print(d["_total"]["hbm_write_bytes"] / 1e9, d["_total"]["hbm_read_bytes_corrected"] / 1e9)
PY
