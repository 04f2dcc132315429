#!/bin/bash
# One round's measurement on the GPU box, in order, every GPU step under its own time limit and the
# script stopping at the first failure:
#   1. the GPU test suite;
#   2. the per-opcode issue probe (tools/issue_probe.py);
#   3. the driver's bench line (bench.py defaults) and a kernel-trace summary of the headline command;
#   4. PMC records stamped with this library's sha256 (tools/pmc_target.sh): headline, sigma, chain.
# Output: gpurun_out/<tag>/ (copy what is judged into profiles/rNN/ and profiles/pmc/).
# Usage: bash tools/gpu_measure.sh <tag> [steps...]   steps: tests probe bench trace pmc (default all)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TMPDIR=/tmp
TAG="${1:-measure}"
shift || true
STEPS="${*:-tests probe bench trace pmc}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
has() { [[ " $STEPS " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
      > "$OUT/pytest.log" 2>&1 || { tail -5 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
if has probe; then
  timeout -k 10 300 python3 tools/issue_probe.py > "$OUT/issue_probe.json" || exit 1
fi
if has bench; then
  timeout -k 10 900 python3 bench.py > "$OUT/bench.log" 2>&1 || { tail -5 "$OUT/bench.log"; exit 1; }
  grep '^{' "$OUT/bench.log" | cut -c1-400
fi
if has trace; then
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/headline_trace" -o run --output-format csv \
      -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu --no-extras > "$OUT/headline_trace.log" 2>&1) || exit 1
fi
if has pmc; then
  bash tools/pmc_target.sh headline k_ct_mul_fresh3 --steps 2 --warmup 1 --no-cpu --no-extras || exit 1
  PVAC_SIGMA_PATH=delta bash tools/pmc_target.sh sigma k_sigma --only sigma || exit 1
  bash tools/pmc_target.sh chain k_ --only chain --chain-inputs 4096 --chain-chunk 1024 --chain-check 0 --chain-ref 0 \
      --chain-no-check || exit 1
  cp gpurun_out/pmc_headline/record.json "$OUT/pmc_headline.json"
  cp gpurun_out/pmc_sigma/record.json "$OUT/pmc_sigma.json"
  cp gpurun_out/pmc_chain/record.json "$OUT/pmc_chain.json"
fi
echo "gpu_measure $TAG: done"
