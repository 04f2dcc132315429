#!/bin/bash
# fresh-kernel phase stamps (diagnostic build) and the sigma kernel's PMC passes on the tree's library
set -o pipefail
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
D="$R/gpurun_out/r4i"
mkdir -p "$D"
timeout -k 10 200 python3 "$R/tools/diag_fresh.py" > "$D/diag_fresh.log" 2>&1 || { tail -20 "$D/diag_fresh.log"; exit 1; }
tail -30 "$D/diag_fresh.log"
timeout -k 10 600 bash "$R/tools/prof_sig_variants.sh" "$R/pvac_hfhe_cppbyv_amd/lib/libpvac_hip.so" > "$D/sig_pmc.log" 2>&1 || { tail -20 "$D/sig_pmc.log"; exit 1; }
tail -30 "$D/sig_pmc.log"
