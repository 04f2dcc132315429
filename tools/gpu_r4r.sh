#!/bin/bash
# record-store cache policy A/B: chain timing, then the chain PMC passes (4096 inputs) on the tree's
# library (streaming stores) and on lib/exp/libpvac_hip_aux0.so (default policy) swapped in
set -o pipefail
R="$GRAFT_REPO_ROOT"
D="$R/gpurun_out/r4r"
L="$R/pvac_hfhe_cppbyv_amd/lib"
mkdir -p "$D"
timeout -k 10 400 python3 "$R/tools/chain_ab.py" --inputs 8192 "$L/libpvac_hip.so" "$L/exp/libpvac_hip_aux0.so" "$L/libpvac_hip.so" "$L/exp/libpvac_hip_aux0.so" 2>&1 | grep -v amdgpu.ids || exit 1
CHAIN_INPUTS=4096 timeout -k 10 600 bash "$R/tools/pmc_chain.sh" > "$D/pmc_aux2.log" 2>&1 || { tail -20 "$D/pmc_aux2.log"; exit 1; }
cp "$R/gpurun_out/pmc_chain/summary.json" "$D/pmc_aux2.json"
cp "$L/exp/libpvac_hip_aux0.so" "$L/libpvac_hip.so"
rm -rf "$R/gpurun_out/pmc_chain"
CHAIN_INPUTS=4096 timeout -k 10 600 bash "$R/tools/pmc_chain.sh" > "$D/pmc_aux0.log" 2>&1 || { tail -20 "$D/pmc_aux0.log"; exit 1; }
cp "$R/gpurun_out/pmc_chain/summary.json" "$D/pmc_aux0.json"
for f in aux2 aux0; do python3 - "$D/pmc_$f.json" $f <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); t = d["_total"]
ks = ["k_large_products_direct", "k_large_count_la", "k_large_lists", "k_large_scan_direct"]
print(sys.argv[2], round(t["hbm_write_bytes"] / 1e9, 1), round(t["hbm_read_bytes_corrected"] / 1e9, 1),
      [(k[8:], d[k]["ms_by_pass"]["p1"], round(d[k]["hbm_write_bytes"] / 1e9, 1), round(d[k]["hbm_read_bytes_corrected"] / 1e9, 1)) for k in ks if k in d])
PY
done
