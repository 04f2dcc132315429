#!/bin/bash
# direct-pair writer A/B (GPU box): large + chain GPU tests on the tree's library, the chain A/B against
# lib/exp/libpvac_hip_list1.so, the single-stream kernel trace of the cfg-4 leg and the phase stamps
set -o pipefail
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
D="$R/gpurun_out/r4g"
mkdir -p "$D"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu "$R/tests/test_gpu_large.py" \
    "$R/tests/test_gpu_chain.py" > "$D/pytest_large_chain.log" 2>&1 || { tail -30 "$D/pytest_large_chain.log"; exit 1; }
tail -2 "$D/pytest_large_chain.log"
timeout -k 10 300 python3 "$R/tools/chain_ab.py" --inputs 8192 "$R/pvac_hfhe_cppbyv_amd/lib/libpvac_hip.so" \
    "$R/pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_prev.so" "$R/pvac_hfhe_cppbyv_amd/lib/libpvac_hip.so" "$R/pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_prev.so" > "$D/chain_ab.log" 2>&1 || { tail -20 "$D/chain_ab.log"; exit 1; }
cat "$D/chain_ab.log"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$D/chain1" -o run --output-format csv \
    -- python3 "$R/bench.py" --only chain --chain-no-check --chain-streams 1 --chain-inputs 8192 > "$D/chain1.log" 2>&1) || { tail -20 "$D/chain1.log"; exit 1; }
T=$(find "$D/chain1" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/chain_window.py" "$T" "$D/chain1.log" "$D/chain1_window.json" | head -24
timeout -k 10 200 python3 "$R/tools/diag_direct.py" 8192 > "$D/diag_direct.json" 2>"$D/diag_direct.err" && cat "$D/diag_direct.json"
