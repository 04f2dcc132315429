#!/bin/bash
# PMC passes over bench.py's dominant kernel (one counter group per rocprofv3 run, as the
# MI355X guide prescribes: FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Usage (GPU box): tools/prof_pmc.sh [kernel-regex] [extra bench args...]
# Output: gpurun_out/pmc/<pass>/... (CSV) + gpurun_out/pmc/summary.json
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TMPDIR=/tmp
KRE="${1:-k_ct_mul}"
shift || true
OUT="${PMC_OUT:-$ROOT/gpurun_out/pmc}"
mkdir -p "$OUT"
BENCH=(python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu --no-extras "$@")
if [ "${PMC_SET:-}" = "cache" ]; then
  # memory-side view: L2 hits / misses, HBM-side fetch, LDS and VALU issue
  passes=(
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD"
    "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM"
    "FETCH_SIZE"
    "TCC_HIT_sum TCC_MISS_sum"
    "GRBM_GUI_ACTIVE GRBM_COUNT"
  )
elif [ "${PMC_SET:-}" = "detail" ]; then
  # issue/stall attribution (no HBM passes)
  passes=(
    "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS"
    "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS_ATOMIC SQ_WAIT_INST_LDS SQ_WAIT_ANY"
    "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_CYCLES SQ_BUSY_CYCLES"
    "GRBM_GUI_ACTIVE GRBM_COUNT"
  )
else
passes=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "GRBM_GUI_ACTIVE GRBM_COUNT"
)
fi
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $p --kernel-include-regex "$KRE" -d "$OUT/p$i" -o run \
      --output-format csv -- "${BENCH[@]}" > "$OUT/p$i.log" 2>&1)
  rc=$?
  echo "pass $i ($p): rc=$rc"
  if [ $rc -ne 0 ]; then
    tail -5 "$OUT/p$i.log"
    # counter-name errors are harmless (nothing ran on the GPU); anything else stops the script
    if ! grep -qi "counter\|not found\|invalid\|unsupported" "$OUT/p$i.log"; then exit $rc; fi
  fi
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
# traffic record for bench.py's roofline.traffic (same pairs / edges-per-layer as the bench run)
python3 - "$OUT/summary.json" "$OUT/pmc_ct_mul_fresh.json" "$@" <<'PY'
import json, sys
summ = json.load(open(sys.argv[1]))
name = next((x for x in ("k_ct_mul_fresh3", "k_ct_mul_fresh") if x in summ), None)
k = summ.get(name) if name else None
args = sys.argv[3:]
pairs = int(args[args.index("--pairs") + 1]) if "--pairs" in args else 1 << 20
epl = int(args[args.index("--epl") + 1]) if "--epl" in args else 20
if k and "hbm_bytes_per_launch" in k:
    json.dump({"kernel": name, "pairs": pairs, "epl": epl, "hbm_bytes_per_launch": k["hbm_bytes_per_launch"],
               "hbm_read_bytes": k["hbm_read_bytes_corrected"], "hbm_write_bytes": k["hbm_write_bytes"],
               "valu_insts_per_launch": k.get("SQ_INSTS_VALU"), "lds_insts_per_launch": k.get("SQ_INSTS_LDS"),
               "lds_bank_conflict_frac": k.get("lds_bank_conflict_frac"), "wait_frac": k.get("wait_frac"),
               "kernel_cycles": k.get("kernel_cycles"),
               "source": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 wide-read correction) / WRITE_SIZE, "
                         "mean per full-batch dispatch (the self-check window launch excluded); tools/prof_pmc.sh",
               "dispatches": k.get("dispatches")}, open(sys.argv[2], "w"), indent=1)
PY
