# Fresh-kernel residency probe: the kernel capped at 1, 2 and 3 resident workgroups per CU.
# Build the variants on the CPU first (compile-time cap, never in the shipped library):
#   for k in 1 2 3; do make -C pvac_hfhe_cppbyv_amd variant VSRC=csrc/k_mul_fresh.hip VNAME=percu$k VFLAGS=-DPVAC_FRESH_PER_CU=$k; done
# then on the GPU box:
timeout -k 10 300 python tools/exp_fresh.py pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_percu1.so \
  pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_percu2.so pvac_hfhe_cppbyv_amd/lib/exp/libpvac_hip_percu3.so
