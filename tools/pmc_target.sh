#!/bin/bash
# PMC passes over one bench target (GPU box), one counter group per rocprofv3 run (the MI355X guide:
# FETCH_SIZE and WRITE_SIZE cannot share a pass; at most 8 SQ_ and 2 GRBM_ counters per pass), then a
# summary stamped with the sha256 of the libpvac_hip.so that was profiled (tools/pmc_stamp.py).
# bench.py quotes a record's traffic / VALU figures only when that hash equals the library it loaded.
#
# Usage: tools/pmc_target.sh <target> <kernel-regex> <bench args...>
#   target: headline | sigma | chain (the record goes to gpurun_out/pmc_<target>/record.json)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TMPDIR=/tmp
TARGET="$1"
KRE="$2"
shift 2
OUT="$ROOT/gpurun_out/pmc_$TARGET"
rm -rf "$OUT"
mkdir -p "$OUT"
BENCH=(python3 "$ROOT/bench.py" "$@")
passes=(
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
  "FETCH_SIZE GRBM_GUI_ACTIVE"
  "WRITE_SIZE GRBM_GUI_ACTIVE"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  (cd /tmp && timeout -k 10 420 rocprofv3 --pmc $p --kernel-include-regex "$KRE" -d "$OUT/p$i" -o run \
      --output-format csv -- "${BENCH[@]}" > "$OUT/p$i.log" 2>&1)
  rc=$?
  echo "pmc $TARGET pass $i: rc=$rc"
  if [ $rc -ne 0 ]; then
    tail -5 "$OUT/p$i.log"
    exit $rc
  fi
done
python3 "$ROOT/tools/pmc_stamp.py" --target "$TARGET" --dir "$OUT" -- "$@" > "$OUT/record.json" && cat "$OUT/record.json"
