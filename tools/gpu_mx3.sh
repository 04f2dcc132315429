#!/bin/bash
# general-path check (GPU box): large-path GPU tests, then cfg-4 kernel stats for the product library
# and the variants given (tools/chain_stats_ab.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/large.log 2>&1; rc=$?; tail -3 gpurun_out/large.log; [ $rc -ne 0 ] && exit $rc
bash tools/chain_stats_ab.sh "$@"
