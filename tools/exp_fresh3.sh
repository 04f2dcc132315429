#!/bin/bash
# Phase costs of k_ct_mul_fresh3 (GPU box): kernel time (tools/exp_fresh.py) and VALU instructions
# per pair (rocprofv3 SQ_INSTS_VALU) of the product library and of each experiment library
# (make exp3: a repeated idempotent phase, or no multiply; outputs of the latter are wrong).
set -o pipefail
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/exp3"
mkdir -p "$OUT"
LIBS=("$ROOT/pvac_hfhe_cppbyv_amd/lib/libpvac_hip.so" "$ROOT"/pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_3_*.so)
timeout -k 10 300 python3 "$ROOT/tools/exp_fresh.py" "${LIBS[@]}" > "$OUT/times.log" 2>&1 || exit $?
for L in "${LIBS[@]}"; do
  b=$(basename "$L" .so)
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --kernel-include-regex "k_ct_mul_fresh" \
     -d "$OUT/$b" -o run --output-format csv -- python3 "$ROOT/tools/exp_fresh.py" "$L" > "$OUT/$b.log" 2>&1) || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys
out = sys.argv[1]
times = json.loads(open(os.path.join(out, "times.log")).read().strip().splitlines()[-1])
for d in sorted(glob.glob(os.path.join(out, "libpvac_hip*"))):
    if not os.path.isdir(d): continue
    acc = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for row in csv.DictReader(open(p)):
            acc.setdefault((row["Counter_Name"], row["Dispatch_Id"]), 0.0)
            acc[(row["Counter_Name"], row["Dispatch_Id"])] += float(row["Counter_Value"])
    per = {}
    for (name, _), v in acc.items(): per.setdefault(name, []).append(v)
    m = {k: sum(v) / len(v) for k, v in per.items()}
    b = os.path.basename(d)
    print(b, "ms", times.get(b + ".so"), "VALU/pair %.0f" % (m.get("SQ_INSTS_VALU", 0) / 2**20),
          "LDS/pair %.0f" % (m.get("SQ_INSTS_LDS", 0) / 2**20))
PY
# the issue ceilings of this GPU beside the phase costs (kind 4: 32-bit VALU, kind 0: the mad mix)
python3 -c "
import sys; sys.path.insert(0, '$ROOT')
from pvac_hfhe_cppbyv_amd import Engine
e = Engine(device=0)
print('valu32 ceiling %.4g/s, mad-mix ceiling %.4g/s' % (e.alu_ceiling(4), e.alu_ceiling(0)))
"
