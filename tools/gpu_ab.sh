#!/bin/bash
# A/B iteration on the fresh ct_mul kernel (GPU box): GPU tests, bench of the default kernel and of
# the previous one (PVAC_FRESH_KERNEL=1), then instruction / LDS counters of the default kernel.
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/ab/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/ab/bench_new.log 2>&1 || exit $?
grep -o '"value": [0-9.e+]*\|"avg_kernel_ms": [0-9.]*' gpurun_out/ab/bench_new.log
if [ "${AB_OLD:-1}" = "1" ]; then
  PVAC_FRESH_KERNEL=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/ab/bench_old.log 2>&1 || exit $?
  grep -o '"value": [0-9.e+]*\|"avg_kernel_ms": [0-9.]*' gpurun_out/ab/bench_old.log
fi
i=0
for p in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM" \
         "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $p --kernel-include-regex "k_ct_mul_fresh" -d "$GRAFT_REPO_ROOT/gpurun_out/ab/p$i" -o run \
      --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu --no-extras > "$GRAFT_REPO_ROOT/gpurun_out/ab/p$i.log" 2>&1) || exit $?
done
python3 tools/pmc_summary.py gpurun_out/ab > gpurun_out/ab/summary.json && python3 - <<'PY'
import json
s = json.load(open("gpurun_out/ab/summary.json"))
for k, m in s.items():
    if "fresh" not in k: continue
    n = 1 << 20
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    print(k, "VALU/pair %.0f LDS/pair %.0f SALU/pair %.0f" % (m["SQ_INSTS_VALU"] / n, m["SQ_INSTS_LDS"] / n, m["SQ_INSTS_SALU"] / n),
          "bank-conflict frac %.3f" % (m.get("SQ_LDS_BANK_CONFLICT", 0) / 256 / max(cyc, 1)),
          "wait frac %.3f" % (m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]), "kernel cycles %.0f" % cyc)
PY
