#!/bin/bash
# k_large_count_la layers-per-workgroup A/B (PVAC_CNT_LA 2 / 8 against the default) on the cfg-4 chain
set -o pipefail
R="$GRAFT_REPO_ROOT"
L="$R/pvac_hfhe_cppbyv_amd/lib"
timeout -k 10 500 python3 "$R/tools/chain_ab.py" --inputs 8192 "$L/exp/libpvac_hip_base.so" "$L/exp/libpvac_hip_cla2.so" "$L/exp/libpvac_hip_cla8.so" "$L/exp/libpvac_hip_base.so" "$L/exp/libpvac_hip_cla2.so" "$L/exp/libpvac_hip_cla8.so" 2>&1 | grep -v amdgpu.ids
