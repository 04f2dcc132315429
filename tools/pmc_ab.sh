#!/bin/bash
# PMC SQ_INSTS_VALU + time for the product lib and the NOMUL experiment lib
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
L=pvac_hfhe_cppbyv_amd/lib
mkdir -p gpurun_out/pmcab
cp $L/libpvac_hip.so /tmp/base.so
for v in base NOMUL NOWALK; do
  if [ $v = base ]; then cp /tmp/base.so $L/libpvac_hip.so; else cp $L/exp/libpvac_hip_$v.so $L/libpvac_hip.so; fi
  (cd /tmp && timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR --kernel-include-regex k_ct_mul_fresh -d "$GRAFT_REPO_ROOT/gpurun_out/pmcab/$v" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu --no-extras > "$GRAFT_REPO_ROOT/gpurun_out/pmcab/$v.log" 2>&1) || exit $?
  echo "$v done"
done
cp /tmp/base.so $L/libpvac_hip.so
python3 tools/pmc_summary.py gpurun_out/pmcab/base > gpurun_out/pmcab/base.json
python3 tools/pmc_summary.py gpurun_out/pmcab/NOMUL > gpurun_out/pmcab/NOMUL.json
python3 tools/pmc_summary.py gpurun_out/pmcab/NOWALK > gpurun_out/pmcab/NOWALK.json
