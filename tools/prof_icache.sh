#!/bin/bash
# instruction-cache and issue counters for one kernel of a bench.py run (GPU box), one pass per
# counter group: tools/prof_icache.sh KERNEL_RE [bench args...]  -> gpurun_out/icache/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TMPDIR=/tmp
KRE="$1"; shift
OUT="$ROOT/gpurun_out/icache"
mkdir -p "$OUT"
(cd /tmp && timeout -k 10 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1) || true
passes=(
  "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
  "SQ_IFETCH SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS"
  "GRBM_GUI_ACTIVE GRBM_COUNT"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $p --kernel-include-regex "$KRE" -d "$OUT/p$i" -o run \
      --output-format csv -- python3 "$ROOT/bench.py" "$@" > "$OUT/p$i.log" 2>&1)
  echo "pass $i ($p): rc=$?"
done
find "$OUT" -name "*counter_collection.csv" | while read f; do
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = (r["Kernel_Name"][:40], r["Counter_Name"]); acc[k] += float(r["Counter_Value"]); n[k] += 1
for k, v in sorted(acc.items()): print(k[0], k[1], v, "dispatches", n[k])
PY
done
