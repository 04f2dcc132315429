#!/bin/bash
# k_large_count_la register rounds A/B (PVAC_LIST_REG_ROUNDS 16 against 8) on the cfg-4 chain
set -o pipefail
R="$GRAFT_REPO_ROOT"
L="$R/pvac_hfhe_cppbyv_amd/lib"
timeout -k 10 500 python3 "$R/tools/chain_ab.py" --inputs 8192 "$L/exp/libpvac_hip_base.so" "$L/exp/libpvac_hip_reg16.so" "$L/exp/libpvac_hip_base.so" "$L/exp/libpvac_hip_reg16.so" 2>&1 | grep -v amdgpu.ids
