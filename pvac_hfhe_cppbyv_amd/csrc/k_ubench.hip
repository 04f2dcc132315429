// k_ubench.hip — measured integer-ALU ceilings for the roofline report (bench.py).
//
// The hot kernels are integer-VALU work, so their roofline needs an ALU ceiling next to the HBM
// one. Rather than a cycles-per-instruction constant, the ceiling is measured on the device that
// runs the bench, in the same process:
//   kind 0: wave64 integer VALU instructions per second, chip-wide: 8 independent chains of
//           v_mad_u64_u32 / v_add_co_u32 / v_alignbit_b32 (the fp_mul mix) in inline asm, so the
//           count per iteration is exact; loop control is scalar (SALU)
//   kind 1: lazy products fp_mul_fold1 (the general path's per-product multiply) per second,
//           register resident, 4 independent chains per lane
//   kind 2: full fp_mul (two folds + canonical form) per second, as kind 1
//   kind 3: column-accumulated products (col26_mac: 25 v_mad_u64_u32 into nine u64 columns, the
//           general path's dense loop since round 2) per second, two accumulators per lane
// Grids fill every CU at 8 waves per SIMD. Used by measurement only, never by the ct_* ops.
#include "common.hpp"

namespace pvhip {
namespace {

constexpr int kUB = 256;

__global__ __launch_bounds__(kUB) void k_probe_valu(uint64_t* out, uint32_t iters, uint32_t seed) {
    const uint32_t a = threadIdx.x ^ seed, b = a * 2654435761u + 1u;
    uint64_t x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = ((uint64_t)(a + k) << 32) | (b ^ k);
    uint32_t y[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) y[k] = a * (k + 3);
    for (uint32_t i = 0; i < iters; ++i) {
        // 24 VALU instructions per iteration: 8 x (mad, add_co, alignbit), independent chains
        asm volatile(
            "v_mad_u64_u32 %0, vcc, %16, %17, %0\n\t"
            "v_mad_u64_u32 %1, vcc, %16, %17, %1\n\t"
            "v_mad_u64_u32 %2, vcc, %16, %17, %2\n\t"
            "v_mad_u64_u32 %3, vcc, %16, %17, %3\n\t"
            "v_mad_u64_u32 %4, vcc, %16, %17, %4\n\t"
            "v_mad_u64_u32 %5, vcc, %16, %17, %5\n\t"
            "v_mad_u64_u32 %6, vcc, %16, %17, %6\n\t"
            "v_mad_u64_u32 %7, vcc, %16, %17, %7\n\t"
            "v_add_co_u32 %8, vcc, %8, %16\n\t"
            "v_add_co_u32 %9, vcc, %9, %16\n\t"
            "v_add_co_u32 %10, vcc, %10, %16\n\t"
            "v_add_co_u32 %11, vcc, %11, %16\n\t"
            "v_add_co_u32 %12, vcc, %12, %17\n\t"
            "v_add_co_u32 %13, vcc, %13, %17\n\t"
            "v_add_co_u32 %14, vcc, %14, %17\n\t"
            "v_add_co_u32 %15, vcc, %15, %17\n\t"
            "v_alignbit_b32 %8, %9, %8, 7\n\t"
            "v_alignbit_b32 %9, %10, %9, 7\n\t"
            "v_alignbit_b32 %10, %11, %10, 7\n\t"
            "v_alignbit_b32 %11, %12, %11, 7\n\t"
            "v_alignbit_b32 %12, %13, %12, 7\n\t"
            "v_alignbit_b32 %13, %14, %13, 7\n\t"
            "v_alignbit_b32 %14, %15, %14, 7\n\t"
            "v_alignbit_b32 %15, %8, %15, 7"
            : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
              "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7])
            : "v"(a), "v"(b)
            : "vcc");
    }
    uint64_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) r ^= x[k] ^ y[k];
    out[(uint64_t)blockIdx.x * kUB + threadIdx.x] = r;
}

// single-pass 32-bit VALU issue: 24 independent v_add_u32 / v_xor_b32 / v_alignbit_b32 per iteration
// (kind 4). The bound for a kernel whose VALU stream is mostly 32-bit (the fresh ct_mul kernel):
// the kind-0 mix above carries v_mad_u64_u32, which issues slower than a 32-bit op.
__global__ __launch_bounds__(kUB) void k_probe_valu32(uint64_t* out, uint32_t iters, uint32_t seed) {
    const uint32_t a = threadIdx.x ^ seed, b = a * 2654435761u + 1u;
    uint32_t y[8], z[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        y[k] = a * (k + 3);
        z[k] = b ^ (k * 0x9E3779B9u);
    }
    for (uint32_t i = 0; i < iters; ++i) {
        asm volatile(
            "v_add_u32 %0, %0, %16\n\t"
            "v_add_u32 %1, %1, %16\n\t"
            "v_add_u32 %2, %2, %16\n\t"
            "v_add_u32 %3, %3, %16\n\t"
            "v_add_u32 %4, %4, %17\n\t"
            "v_add_u32 %5, %5, %17\n\t"
            "v_add_u32 %6, %6, %17\n\t"
            "v_add_u32 %7, %7, %17\n\t"
            "v_xor_b32 %8, %8, %0\n\t"
            "v_xor_b32 %9, %9, %1\n\t"
            "v_xor_b32 %10, %10, %2\n\t"
            "v_xor_b32 %11, %11, %3\n\t"
            "v_xor_b32 %12, %12, %4\n\t"
            "v_xor_b32 %13, %13, %5\n\t"
            "v_xor_b32 %14, %14, %6\n\t"
            "v_xor_b32 %15, %15, %7\n\t"
            "v_alignbit_b32 %0, %8, %0, 7\n\t"
            "v_alignbit_b32 %1, %9, %1, 7\n\t"
            "v_alignbit_b32 %2, %10, %2, 7\n\t"
            "v_alignbit_b32 %3, %11, %3, 7\n\t"
            "v_alignbit_b32 %4, %12, %4, 7\n\t"
            "v_alignbit_b32 %5, %13, %5, 7\n\t"
            "v_alignbit_b32 %6, %14, %6, 7\n\t"
            "v_alignbit_b32 %7, %15, %7, 7"
            : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]),
              "+v"(z[0]), "+v"(z[1]), "+v"(z[2]), "+v"(z[3]), "+v"(z[4]), "+v"(z[5]), "+v"(z[6]), "+v"(z[7])
            : "v"(a), "v"(b));
    }
    uint64_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) r ^= (uint64_t)y[k] << 32 | z[k];
    out[(uint64_t)blockIdx.x * kUB + threadIdx.x] = r;
}

template <bool FULL>
__global__ __launch_bounds__(kUB) void k_probe_mul(uint64_t* out, uint32_t iters, uint32_t seed) {
    const uint64_t s = ((uint64_t)(threadIdx.x ^ seed) << 17) | blockIdx.x;
    fp y{s * 0x9E3779B97F4A7C15ull, (s * 0xBF58476D1CE4E5B9ull) & kM63};
    fp x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = fp{s + k, (s >> 3) & kM63};
    for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (FULL) {
                x[k] = fp_mul(x[k], y);
            } else {
                uint64_t l, h;
                fp_mul_fold1(x[k], y, l, h);
                x[k] = fp{l, h & kM63};   // keep the operand below 2^127 (one VALU op)
            }
        }
    }
    uint64_t r = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) r ^= x[k].lo ^ x[k].hi;
    out[(uint64_t)blockIdx.x * kUB + threadIdx.x] = r;
}

// two column accumulators (P and M of the products kernel) fed from limb vectors that change every
// iteration (one VALU op each), so nothing is loop-invariant
__global__ __launch_bounds__(kUB) void k_probe_col26(uint64_t* out, uint32_t iters, uint32_t seed) {
    const uint32_t s = (threadIdx.x ^ seed) * 2654435761u + blockIdx.x;
    uint32_t a[5], b[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        a[k] = (s >> k) & kM26;
        b[k] = (s * (k + 7)) & kM26;
    }
    uint64_t P[9], M[9];
    col26_zero(P);
    col26_zero(M);
    for (uint32_t i = 0; i < iters; ++i) {
        col26_mac(P, a, b);
        col26_mac(M, b, a);
#pragma unroll
        for (int k = 0; k < 5; ++k) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[k]) : "v"(i));
    }
    uint64_t r = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) r ^= P[k] ^ M[k];
    out[(uint64_t)blockIdx.x * kUB + threadIdx.x] = r;
}

// the matrix-core product ceiling of the general path's dense mode (k_mul_large.hip): back-to-back
// v_mfma_i32_32x32x32_i8 on four independent accumulators per wave; one such MFMA is 64 Fp
// products there (32 output rows x 2 sparse edges, 16 x 16 digit pairs each)
typedef int pb_v4 __attribute__((ext_vector_type(4)));
typedef int pb_v16 __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(kUB) void k_probe_mfma8(uint64_t* out, uint32_t iters, uint32_t seed) {
    const int s = (int)((threadIdx.x ^ seed) * 2654435761u + blockIdx.x);
    const pb_v4 a{s, s >> 3, s >> 5, s >> 7}, b{s >> 11, s >> 13, s >> 17, s >> 19};
    pb_v16 c0{}, c1{}, c2{}, c3{};
    for (uint32_t i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, b, c3, 0, 0, 0);
    }
    int r = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) r ^= c0[k] ^ c1[k] ^ c2[k] ^ c3[k];
    out[(uint64_t)blockIdx.x * kUB + threadIdx.x] = (uint32_t)r;
}

}  // namespace

// ops per second of probe `kind` (see above), timed with HIP events on `st` (synchronises)
hipError_t run_alu_probe(int kind, int num_cus, hipStream_t st, double* per_s) {
    const uint32_t blocks = (uint32_t)num_cus * 8u;   // 8 waves per SIMD (4 SIMDs, 4 waves per block)
    uint64_t* buf = nullptr;
    hipError_t e = hipMalloc(&buf, (size_t)blocks * kUB * 8);
    if (e != hipSuccess) return e;
    hipEvent_t t0, t1;
    hipEventCreate(&t0);
    hipEventCreate(&t1);
    const uint32_t iters = kind == 0 || kind == 4 || kind == 5 ? 4096u : 512u;
    double ops = 0;
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {   // the first launch warms clocks and code
        hipEventRecord(t0, st);
        if (kind == 0) {
            hipLaunchKernelGGL(k_probe_valu, dim3(blocks), dim3(kUB), 0, st, buf, iters, 0x5EEDu + rep);
            ops = (double)blocks * (kUB / 64) * iters * 24.0;   // wave64 instructions
        } else if (kind == 4) {
            hipLaunchKernelGGL(k_probe_valu32, dim3(blocks), dim3(kUB), 0, st, buf, iters, 0x5EEDu + rep);
            ops = (double)blocks * (kUB / 64) * iters * 24.0;   // wave64 instructions
        } else if (kind == 1) {
            hipLaunchKernelGGL(k_probe_mul<false>, dim3(blocks), dim3(kUB), 0, st, buf, iters, 0x5EEDu + rep);
            ops = (double)blocks * kUB * iters * 4.0;           // lane products
        } else if (kind == 3) {
            hipLaunchKernelGGL(k_probe_col26, dim3(blocks), dim3(kUB), 0, st, buf, iters, 0x5EEDu + rep);
            ops = (double)blocks * kUB * iters * 2.0;           // lane products
        } else if (kind == 5) {
            hipLaunchKernelGGL(k_probe_mfma8, dim3(blocks), dim3(kUB), 0, st, buf, iters, 0x5EEDu + rep);
            ops = (double)blocks * (kUB / 64) * iters * 4.0 * 64.0;   // dense-mode products (64 per MFMA)
        } else {
            hipLaunchKernelGGL(k_probe_mul<true>, dim3(blocks), dim3(kUB), 0, st, buf, iters, 0x5EEDu + rep);
            ops = (double)blocks * kUB * iters * 4.0;
        }
        hipEventRecord(t1, st);
    }
    e = hipGetLastError();
    if (e == hipSuccess) e = hipEventSynchronize(t1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, t0, t1);
    hipEventDestroy(t0);
    hipEventDestroy(t1);
    hipFree(buf);
    if (e == hipSuccess) *per_s = ms > 0 ? ops / (ms / 1000.0) : 0.0;
    return e;
}

}  // namespace pvhip
