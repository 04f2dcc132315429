set -o pipefail
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu "$GRAFT_REPO_ROOT/tests/test_gpu_large.py" "$GRAFT_REPO_ROOT/tests/test_gpu_chain.py" > "$GRAFT_REPO_ROOT/gpurun_out/r4o_pytest.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/r4o_pytest.log"; exit 1; }
R="$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 "$R/tools/exp_sigma.py" "$R/pvac_hfhe_cppbyv_amd/lib/libpvac_hip.so" "$R/pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_SIG_MINB5.so" "$R/pvac_hfhe_cppbyv_amd/lib/libpvac_hip.so" "$R/pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_SIG_MINB5.so" 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python3 "$R/tools/chain_ab.py" --inputs 8192 "$R/pvac_hfhe_cppbyv_amd/lib/libpvac_hip.so" "$R/pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_prev2.so" "$R/pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_la2.so" "$R/pvac_hfhe_cppbyv_amd/lib/libpvac_hip.so" "$R/pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_prev2.so" 2>&1 | grep -v amdgpu.ids
