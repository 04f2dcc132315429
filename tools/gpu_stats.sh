#!/bin/bash
# usage: gpu_stats.sh TAG -> GPU tests, then kernel-trace stats of a short bench run (gpurun_out/stats_TAG/)
TAG=$1
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout=300 -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/stats_$TAG" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras > "$ROOT/gpurun_out/bench_$TAG.log" 2>&1) || exit $?
grep -o '"value": [0-9.e+]*\|"avg_kernel_ms": [0-9.]*\|"frac": [0-9.]*' gpurun_out/bench_$TAG.log
f=$(find gpurun_out/stats_$TAG -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv,sys
for r in list(csv.DictReader(open('$f')))[:8]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')"
