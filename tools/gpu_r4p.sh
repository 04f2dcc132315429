#!/bin/bash
# large / chain GPU tests on the library in the tree, then the cfg-4 chain A/B against lib/exp/libpvac_hip_base.so
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/r4p"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu "$R/tests/test_gpu_large.py" "$R/tests/test_gpu_chain.py" > "$R/gpurun_out/r4p/pytest.log" 2>&1 || { tail -30 "$R/gpurun_out/r4p/pytest.log"; exit 1; }
tail -2 "$R/gpurun_out/r4p/pytest.log"
L="$R/pvac_hfhe_cppbyv_amd/lib"
timeout -k 10 400 python3 "$R/tools/chain_ab.py" --inputs 8192 "$L/libpvac_hip.so" "$L/exp/libpvac_hip_base.so" "$L/libpvac_hip.so" "$L/exp/libpvac_hip_base.so" 2>&1 | grep -v amdgpu.ids
