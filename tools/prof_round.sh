#!/bin/bash
# Round profile bundle (GPU box): kernel-trace stats of the default bench run, PMC HBM traffic of the
# dominant kernel (FETCH_SIZE / WRITE_SIZE passes), and the bench line itself. Outputs under
# gpurun_out/round/; copy the summaries into profiles/<round>/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/round"
mkdir -p "$OUT"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras > "$OUT/stats_bench.log" 2>&1) || exit $?
echo "stats ok"
bash "$ROOT/tools/prof_pmc.sh" k_ct_mul_fresh > "$OUT/pmc.log" 2>&1 || exit $?
cp "$ROOT/gpurun_out/pmc/summary.json" "$OUT/pmc_summary.json"
cp "$ROOT/gpurun_out/pmc/pmc_ct_mul_fresh.json" "$OUT/pmc_ct_mul_fresh.json"
echo "pmc ok"
timeout -k 10 600 python3 "$ROOT/bench.py" > "$OUT/bench_default.log" 2>&1 || exit $?
tail -1 "$OUT/bench_default.log"
