set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ab
L=(pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_*.so)
timeout -k 10 400 python3 tools/exp_fresh.py "${L[@]}" "${L[@]}" > gpurun_out/r6ab/ab_times.log 2>&1 || { tail -20 gpurun_out/r6ab/ab_times.log; exit 1; }
grep -v amdgpu gpurun_out/r6ab/ab_times.log | grep -v "^{"
if [ "${AB_STEP:-1}" = "1" ]; then
timeout -k 10 400 python3 tools/step_ab.py "${L[@]}" "${L[@]}" "${L[@]}" > gpurun_out/r6ab/step_ab.log 2>&1 || { tail -20 gpurun_out/r6ab/step_ab.log; exit 1; }
grep -v amdgpu gpurun_out/r6ab/step_ab.log
fi
if [ "${AB_TESTS:-0}" = "1" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6ab/pytest.log 2>&1 || { tail -30 gpurun_out/r6ab/pytest.log; exit 1; }
  tail -2 gpurun_out/r6ab/pytest.log
fi
