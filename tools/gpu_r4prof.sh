#!/bin/bash
# round 4: kernel trace of the cfg-4 leg (warm-up + timed pass; tools/chain_window.py keeps the timed
# pass's dispatches), the chain's PMC passes (tools/pmc_chain.sh, timed window only), and the
# headline command's kernel trace
set -o pipefail
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
D="$R/gpurun_out/r4prof"
mkdir -p "$D"
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$D/chain" -o run --output-format csv \
    -- python3 "$R/bench.py" --only chain --chain-no-check > "$D/chain.log" 2>&1) || { tail -20 "$D/chain.log"; exit 1; }
T=$(find "$D/chain" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/chain_window.py" "$T" "$D/chain.log" "$D/chain_window.json" | head -40
cp $(find "$D/chain" -name "*kernel_stats.csv" | head -1) "$D/chain_kernel_stats.csv"
CHAIN_INPUTS=${CHAIN_INPUTS:-8192} bash "$R/tools/pmc_chain.sh" > "$D/pmc_chain.log" 2>&1; tail -30 "$D/pmc_chain.log"
cp "$R/gpurun_out/pmc_chain/summary.json" "$D/pmc_chain_summary.json" 2>/dev/null
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$D/headline" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu --no-extras > "$D/headline.log" 2>&1) || exit $?
cp $(find "$D/headline" -name "*kernel_stats.csv" | head -1) "$D/headline_kernel_stats.csv"
tail -1 "$D/headline.log" | cut -c1-300
