#!/bin/bash
# PMC counters of k_sigma for each experiment library (GPU box):
#   tools/prof_sig_variants.sh lib1.so lib2.so ...   -> gpurun_out/sigv/ + per-library table
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/sigv"
mkdir -p "$OUT"
passes=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM"
  "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $p --kernel-include-regex "k_sigma" -d "$OUT/p$i" -o run \
      --output-format csv -- python3 "$ROOT/tools/exp_sigma.py" "$@" > "$OUT/p$i.log" 2>&1)
  rc=$?
  echo "pass $i: rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 - "$OUT" "$@" <<'PY'
import csv, sys, glob, collections, os
out, libs = sys.argv[1], [os.path.basename(x) for x in sys.argv[2:]]
per = collections.defaultdict(lambda: collections.defaultdict(float))   # (pass, dispatch) -> counter -> value
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    pas = os.path.relpath(f, out).split("/")[0]
    for r in csv.DictReader(open(f)):
        per[(pas, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
# dispatch order within each pass: 4 per library (1 warm-up + 3 timed)
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for pas in sorted({k[0] for k in per}):
    ds = sorted(k for k in per if k[0] == pas)
    for i, k in enumerate(ds):
        lib = libs[i // 4] if i // 4 < len(libs) else "?"
        if i % 4 == 0: continue
        for c, v in per[k].items(): rows[lib][c].append(v)
for lib in libs:
    d = {c: sum(v) / len(v) for c, v in rows[lib].items()}
    cyc = d.get("GRBM_GUI_ACTIVE", 0) / 8
    print(lib, {k: round(v / 1e6, 1) for k, v in sorted(d.items())}, "kernel_Mcycles", round(cyc / 1e6, 1))
PY
