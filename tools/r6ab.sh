set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ab
L=(pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_*.so)
timeout -k 10 500 python3 tools/exp_fresh.py "${L[@]}" "${L[@]}" "${L[@]}" > gpurun_out/r6ab/ab_times.log 2>&1 || { tail -20 gpurun_out/r6ab/ab_times.log; exit 1; }
grep -v amdgpu gpurun_out/r6ab/ab_times.log
