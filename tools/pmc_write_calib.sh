#!/bin/bash
# WRITE_SIZE calibration for 8-byte-per-lane stores (the guide calibrates only 16-B stores): PMC of
# k_ct_add_wave, whose written bytes are known exactly (24 B per output edge + 40 B per layer record).
set -u
ROOT="${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/pmc_add"
mkdir -p "$OUT"
i=0
for p in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 200 rocprofv3 --pmc $p --kernel-include-regex "k_ct_add_wave" -d "$OUT/p$i" -o run --output-format csv -- python3 "$ROOT/bench.py" --only add > "$OUT/p$i.log" 2>&1) || exit $?
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
