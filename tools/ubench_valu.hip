// ubench_valu.hip — VALU throughput of the integer primitives fp_mul is built from (tooling only).
// Every wave runs ITER rounds of 8 independent instruction chains (inline asm, so nothing is folded
// away); the grid fills every SIMD 8 waves deep. Reports SIMD cycles per wave64 instruction.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
constexpr int ITER = 4096;

template <int MODE>
__global__ __launch_bounds__(256) void k_valu(uint32_t* out, uint32_t seed) {
    uint32_t a[8], b[8];
    uint64_t c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { a[k] = seed * (threadIdx.x + k); b[k] = seed ^ (k * 77 + threadIdx.x); c[k] = a[k]; }
    for (int r = 0; r < ITER; ++r) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (MODE == 0) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(c[k]) : "v"(a[k]), "v"(b[k]) : "vcc");
            if (MODE == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
            if (MODE == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
            if (MODE == 3) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[k]) : "v"(b[k]) : "vcc");
            if (MODE == 4) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
            if (MODE == 5) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
            if (MODE == 6) asm volatile("v_fma_f64 %0, %1, %1, %0" : "+v"(c[k]) : "v"(*(uint64_t*)&c[(k + 1) & 7]));
            if (MODE == 7) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[k]) : "v"(b[k]));
            if (MODE == 8) asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(c[k]));
            if (MODE == 9) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[k]) : "v"(b[k]));
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += a[k] + (uint32_t)c[k] + (uint32_t)(c[k] >> 32);
    if (s == 0x12345678u) out[0] = s;
}

template <int MODE>
int run(const char* name, int cus, double clk_ghz) {
    uint32_t* d;
    CK(hipMalloc(&d, 4));
    const int blocks = cus * 8;   // 256-thread blocks: 4 waves each -> 32 waves per CU (8 per SIMD)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_valu<MODE>, dim3(blocks), dim3(256), 0, 0, d, 3u);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_valu<MODE>, dim3(blocks), dim3(256), 0, 0, d, 5u);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double instr_per_simd = (double)blocks * 4 * ITER * 8 / (cus * 4.0);   // wave-instructions per SIMD
    const double cyc = ms * 1e-3 * clk_ghz * 1e9 / instr_per_simd;
    printf("%-22s %8.3f ms  %.2f SIMD cycles per wave64 instruction (at %.1f GHz)\n", name, ms, cyc, clk_ghz);
    CK(hipFree(d));
    return 0;
}

int main() {
    hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const double ghz = p.clockRate / 1e6;
    printf("CUs %d, clock %.2f GHz\n", cus, ghz);
    run<3>("v_add_co_u32", cus, ghz);
    run<9>("v_alignbit_b32", cus, ghz);
    run<0>("v_mad_u64_u32", cus, ghz);
    run<1>("v_mul_lo_u32", cus, ghz);
    run<2>("v_mul_hi_u32", cus, ghz);
    run<4>("v_mul_u32_u24", cus, ghz);
    run<5>("v_mul_hi_u32_u24", cus, ghz);
    run<7>("v_mad_u32_u24", cus, ghz);
    run<8>("v_lshl_add_u64", cus, ghz);
    run<6>("v_fma_f64", cus, ghz);
    return 0;
}
