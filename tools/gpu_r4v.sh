#!/bin/bash
# k_large_count_la wave-priority A/B (PVAC_DIR_PRIO 1 / 2 against 0) on the cfg-4 chain
set -o pipefail
R="$GRAFT_REPO_ROOT"
L="$R/pvac_hfhe_cppbyv_amd/lib"
timeout -k 10 500 python3 "$R/tools/chain_ab.py" --inputs 8192 "$L/exp/libpvac_hip_base.so" "$L/exp/libpvac_hip_prio1.so" "$L/exp/libpvac_hip_prio2.so" "$L/exp/libpvac_hip_base.so" "$L/exp/libpvac_hip_prio1.so" "$L/exp/libpvac_hip_prio2.so" 2>&1 | grep -v amdgpu.ids
