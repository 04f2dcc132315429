// probe_rates.hip — issue rate of single VALU opcodes on this GPU (diagnostic, never linked into the
// library): 8 independent chains of one opcode per lane, 256-thread blocks at 8 waves per SIMD,
// timed with HIP events. Prints one JSON line: wave-instructions per second per opcode.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_rates.hip -o tools/build/probe_rates
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHAIN8(OP)                                                                                         \
    asm volatile(OP " %0, %0, %8\n\t" OP " %1, %1, %8\n\t" OP " %2, %2, %8\n\t" OP " %3, %3, %8\n\t" OP \
                    " %4, %4, %9\n\t" OP " %5, %5, %9\n\t" OP " %6, %6, %9\n\t" OP " %7, %7, %9"          \
                 : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]),   \
                   "+v"(y[7])                                                                             \
                 : "v"(a), "v"(b))

#define CHAIN8_3(OP)                                                                                       \
    asm volatile(OP " %0, %0, %8, %9\n\t" OP " %1, %1, %8, %9\n\t" OP " %2, %2, %8, %9\n\t" OP            \
                    " %3, %3, %8, %9\n\t" OP " %4, %4, %9, %8\n\t" OP " %5, %5, %9, %8\n\t" OP             \
                    " %6, %6, %9, %8\n\t" OP " %7, %7, %9, %8"                                            \
                 : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]),   \
                   "+v"(y[7])                                                                             \
                 : "v"(a), "v"(b))

template <int K>
__global__ __launch_bounds__(256) void k_rate(uint32_t* out, uint32_t iters) {
    const uint32_t a = threadIdx.x * 2654435761u + 7u, b = a ^ 0x9E3779B9u;
    uint32_t y[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) y[k] = a + k;
    for (uint32_t i = 0; i < iters; ++i) {
        if (K == 0) CHAIN8("v_add_u32");
        if (K == 1) CHAIN8("v_mul_lo_u32");
        if (K == 2) CHAIN8("v_mul_hi_u32");
        if (K == 3) CHAIN8("v_mul_u32_u24");
        if (K == 4) CHAIN8_3("v_mad_u32_u24");
        if (K == 5) CHAIN8_3("v_lshl_add_u32");
        if (K == 6) CHAIN8_3("v_bfe_u32");
        if (K == 7) CHAIN8("v_min_u32");
        if (K == 8) CHAIN8_3("v_add3_u32");
        if (K == 9) CHAIN8_3("v_and_or_b32");
        if (K == 10) CHAIN8("v_mul_hi_u32_u24");
    }
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) r ^= y[k];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int K>
double rate(uint32_t* out, int blocks, uint32_t iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_rate<K><<<blocks, 256>>>(out, 16);
    hipEventRecord(e0);
    k_rate<K><<<blocks, 256>>>(out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double instr = (double)blocks * 4 /* waves */ * iters * 8;
    return instr / (ms * 1e-3);
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    const int blocks = p.multiProcessorCount * 8;   // 8 blocks x 4 waves = 32 waves per CU = 8 per SIMD
    uint32_t* out = nullptr;
    if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    const uint32_t it = 1u << 16;
    std::printf("{\"cus\": %d, \"wave_instr_per_s\": {\"v_add_u32\": %.4g, \"v_mul_lo_u32\": %.4g, \"v_mul_hi_u32\": %.4g, "
                "\"v_mul_u32_u24\": %.4g, \"v_mad_u32_u24\": %.4g, \"v_lshl_add_u32\": %.4g, \"v_bfe_u32\": %.4g, "
                "\"v_min_u32\": %.4g, \"v_add3_u32\": %.4g, \"v_and_or_b32\": %.4g, \"v_mul_hi_u32_u24\": %.4g}}\n",
                p.multiProcessorCount, rate<0>(out, blocks, it), rate<1>(out, blocks, it), rate<2>(out, blocks, it),
                rate<3>(out, blocks, it), rate<4>(out, blocks, it), rate<5>(out, blocks, it), rate<6>(out, blocks, it),
                rate<7>(out, blocks, it), rate<8>(out, blocks, it), rate<9>(out, blocks, it), rate<10>(out, blocks, it));
    hipFree(out);
    return 0;
}
