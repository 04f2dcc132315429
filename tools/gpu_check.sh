#!/bin/bash
# GPU-box check script: pytest -m gpu, then a short bench, then (optionally) rocprofv3 stats.
# Stops at the first GPU fault / abort / timeout (exit >= 2 other than pytest's 1 = failures).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE="${1:-all}"
rc=0
if [ "$STAGE" = "all" ] || [ "$STAGE" = "tests" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout=600 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -5 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
fi
if [ "$STAGE" = "all" ] || [ "$STAGE" = "bench" ]; then
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
  brc=$?
  tail -3 gpurun_out/bench.log
  if [ $brc -ne 0 ]; then echo "bench exit $brc: stopping"; exit $brc; fi
fi
if [ "$STAGE" = "all" ] || [ "$STAGE" = "prof" ]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run \
      --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu \
      > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  prc=$?
  cd "$GRAFT_REPO_ROOT"
  tail -3 gpurun_out/prof.log
  find gpurun_out/prof -name "*stats*" | head
  if [ $prc -ne 0 ]; then echo "rocprof exit $prc"; exit $prc; fi
fi
exit $rc
