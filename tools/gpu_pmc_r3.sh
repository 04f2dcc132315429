#!/bin/bash
# round-3 PMC of the headline kernel: default passes (HBM bytes, VALU, LDS) and the issue/stall set,
# full-batch dispatches only (tools/pmc_summary.py), plus the kernel trace of the same command.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT}"
OUT=${1:-r3pmc}
mkdir -p "$ROOT/gpurun_out/$OUT"
PMC_OUT="$ROOT/gpurun_out/$OUT/pmc" bash "$ROOT/tools/prof_pmc.sh" k_ct_mul_fresh3 > "$ROOT/gpurun_out/$OUT/pmc.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/$OUT/pmc.log"; exit 1; }
tail -5 "$ROOT/gpurun_out/$OUT/pmc.log"
PMC_SET=detail PMC_OUT="$ROOT/gpurun_out/$OUT/detail" bash "$ROOT/tools/prof_pmc.sh" k_ct_mul_fresh3 > "$ROOT/gpurun_out/$OUT/detail.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/$OUT/detail.log"; exit 1; }
tail -3 "$ROOT/gpurun_out/$OUT/detail.log"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/$OUT/trace" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu --no-extras > "$ROOT/gpurun_out/$OUT/trace.log" 2>&1) || exit 1
echo trace ok
