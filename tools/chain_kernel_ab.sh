#!/bin/bash
# Per-kernel times of the cfg-4 chain (one worker stream, 8,192 enc_value inputs, depth 8) through each
# library given (GPU box): rocprofv3 kernel-trace stats per library, the top kernels printed side by side.
# Usage: bash tools/chain_kernel_ab.sh pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_A.so [...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename "$L" .so)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kab_$n -o run --output-format csv -- \
    python3 tools/chain_ab.py --inputs 8192 --streams 1 "$L" > gpurun_out/kab_$n.log 2>&1 || exit $?
done
for L in "$@"; do
  n=$(basename "$L" .so); f=$(find gpurun_out/kab_$n -name '*kernel_stats.csv' | head -1); echo "== $n"
  python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    name = r["Name"].replace("void ", "").replace("pvhip::(anonymous namespace)::", "")[:44]
    print("%-44s %6d %9.1f ms" % (name, int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6))
PY
done
