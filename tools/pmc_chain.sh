#!/bin/bash
# PMC passes over the cfg-4 chain's kernels (GPU box): one counter group per rocprofv3 run
# (FETCH_SIZE and WRITE_SIZE cannot share a pass), then per-kernel TOTALS over the dispatches of the
# TIMED chain only (the bench line's monotonic window; tools/pmc_chain_summary.py). The bench runs
# without its checked second pass (--chain-no-check). Output: gpurun_out/pmc_chain/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/pmc_chain"
mkdir -p "$OUT"
KRE="${KRE:-k_}"
BENCH=(python3 "$ROOT/bench.py" --only chain --chain-inputs "${CHAIN_INPUTS:-4096}" --chain-chunk "${CHAIN_CHUNK:-1024}"
       --chain-check 0 --chain-ref 0 --chain-no-check)
passes=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $p --kernel-include-regex "$KRE" -d "$OUT/p$i" -o run \
      --output-format csv -- "${BENCH[@]}" > "$OUT/p$i.log" 2>&1)
  rc=$?
  echo "pass $i ($p): rc=$rc"
  if [ $rc -ne 0 ]; then
    tail -5 "$OUT/p$i.log"
    if ! grep -qi "counter\|not found\|invalid\|unsupported" "$OUT/p$i.log"; then exit $rc; fi
  fi
done
python3 "$ROOT/tools/pmc_chain_summary.py" "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
