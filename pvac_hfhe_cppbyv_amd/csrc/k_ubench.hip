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
#include <algorithm>
#include <array>
#include <utility>
#include <vector>

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

// ---------------------------------------------------------------- per-opcode issue probe
// One opcode alone, 16 independent accumulators per lane (16 instructions per iteration, each
// depending only on its own previous value), `wps` waves per SIMD on every CU. Thread 0 of every
// workgroup records s_memtime (shader clock) and s_memrealtime (100 MHz) at its start and end, so
// the host gets the clock the SIMDs actually ran at next to the instruction rate: cycles per
// wave64 instruction = (SIMDs x shader clock) / (instructions per second).
#define PVAC_IP16(OPS)                                                                                       \
    asm volatile(OPS                                                                                         \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]),       \
                   "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]),   \
                   "+v"(r[14]), "+v"(r[15])                                                                  \
                 : "v"(a), "v"(b)                                                                            \
                 : "vcc")
// 16 instructions; accumulator k is the destination and the first-listed source: "I %k, PRE%kPOST"
#define PVAC_IPK(I, PRE, POST, k) I " %" #k ", " PRE "%" #k POST "\n\t"
#define PVAC_IPS(I, PRE, POST)                                                                              \
    PVAC_IPK(I, PRE, POST, 0) PVAC_IPK(I, PRE, POST, 1) PVAC_IPK(I, PRE, POST, 2) PVAC_IPK(I, PRE, POST, 3)  \
    PVAC_IPK(I, PRE, POST, 4) PVAC_IPK(I, PRE, POST, 5) PVAC_IPK(I, PRE, POST, 6) PVAC_IPK(I, PRE, POST, 7)  \
    PVAC_IPK(I, PRE, POST, 8) PVAC_IPK(I, PRE, POST, 9) PVAC_IPK(I, PRE, POST, 10)                           \
    PVAC_IPK(I, PRE, POST, 11) PVAC_IPK(I, PRE, POST, 12) PVAC_IPK(I, PRE, POST, 13)                         \
    PVAC_IPK(I, PRE, POST, 14) PVAC_IPK(I, PRE, POST, 15)

template <int OP>
__global__ void k_probe_issue(uint64_t* out, uint64_t* clk, uint32_t iters, uint32_t seed) {
    const uint32_t a = threadIdx.x ^ seed, b = a * 2654435761u + 1u;
    uint32_t r[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) r[k] = a * (k + 3) + b;
    uint64_t t0 = 0, q0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        q0 = __builtin_amdgcn_s_memrealtime();
    }
    for (uint32_t i = 0; i < iters; ++i) {
        // each accumulator's operands: itself and the loop-invariant a / b (16 independent chains)
        if constexpr (OP == 0) PVAC_IP16(PVAC_IPS("v_add_u32", "", ",%16"));
        if constexpr (OP == 1) PVAC_IP16(PVAC_IPS("v_xor_b32", "", ",%16"));
        if constexpr (OP == 2) PVAC_IP16(PVAC_IPS("v_alignbit_b32", "", ",%16,7"));
        if constexpr (OP == 3) PVAC_IP16(PVAC_IPS("v_lshlrev_b32", "%16,", ""));
        if constexpr (OP == 4) PVAC_IP16(PVAC_IPS("v_min_u32", "", ",%16"));
        if constexpr (OP == 5) PVAC_IP16(PVAC_IPS("v_add3_u32", "", ",%16,%17"));
        if constexpr (OP == 6) PVAC_IP16(PVAC_IPS("v_pk_add_u16", "", ",%16"));
        if constexpr (OP == 7) PVAC_IP16(PVAC_IPS("v_fma_f32", "", ",%16,%17"));
        if constexpr (OP == 8) PVAC_IP16(PVAC_IPS("v_mul_lo_u32", "", ",%16"));
        if constexpr (OP == 9) PVAC_IP16(PVAC_IPS("v_mul_hi_u32", "", ",%16"));
        if constexpr (OP == 10) PVAC_IP16(PVAC_IPS("v_cndmask_b32", "%16,", ",vcc"));
        if constexpr (OP == 11) PVAC_IP16(PVAC_IPS("v_bfe_u32", "", ",%16,12"));
        if constexpr (OP == 12) PVAC_IP16(PVAC_IPS("v_add_co_u32", "vcc,", ",%16"));
        if constexpr (OP == 13) PVAC_IP16(PVAC_IPS("v_and_or_b32", "", ",%16,%17"));
        if constexpr (OP == 14) PVAC_IP16(PVAC_IPS("v_pk_min_u16", "", ",%16"));
        if constexpr (OP == 15) PVAC_IP16(PVAC_IPS("v_bitop3_b32", "", ",%16,%17 bitop3:0x96"));
        if constexpr (OP == 16) {
            // v_mad_u64_u32 on 8 64-bit accumulators (register pairs r[2k], r[2k + 1]): 8 per iteration
            uint64_t* x = (uint64_t*)r;
            asm volatile(
                "v_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_mad_u64_u32 %1, vcc, %9, %8, %1\n\t"
                "v_mad_u64_u32 %2, vcc, %8, %8, %2\n\tv_mad_u64_u32 %3, vcc, %9, %9, %3\n\t"
                "v_mad_u64_u32 %4, vcc, %8, %9, %4\n\tv_mad_u64_u32 %5, vcc, %9, %8, %5\n\t"
                "v_mad_u64_u32 %6, vcc, %8, %8, %6\n\tv_mad_u64_u32 %7, vcc, %9, %9, %7"
                : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
                : "v"(a), "v"(b)
                : "vcc");
        }
        if constexpr (OP == 17) PVAC_IP16(PVAC_IPS("v_cndmask_b32_e64", "%16,", ",s[4:5]"));
        if constexpr (OP == 18) PVAC_IP16(PVAC_IPS("v_lshl_add_u32", "", ",3,%16"));
        if constexpr (OP == 19) PVAC_IP16(PVAC_IPS("v_mov_b32_dpp", "", " row_shr:1 row_mask:0xf bank_mask:0xf"));
        if constexpr (OP == 20) PVAC_IP16(PVAC_IPS("v_perm_b32", "", ",%16,%17"));
        if constexpr (OP == 21) PVAC_IP16(PVAC_IPS("v_mul_u32_u24", "", ",%16"));
        if constexpr (OP == 22) PVAC_IP16(PVAC_IPS("v_sub_u32", "%16,", ""));
        if constexpr (OP == 23) PVAC_IP16(PVAC_IPS("v_max3_u32", "", ",%16,%17"));
        // VCC readers (the compiler's v_cmp + v_cndmask_b32_e32 / v_addc_co_u32_e32 pattern)
        if constexpr (OP == 24) {   // 8 x (v_cmp writing vcc, VOP2 v_cndmask reading it): 16 instructions
            asm volatile(
                "v_cmp_gt_u32 vcc, %0, %16\n\tv_cndmask_b32 %1, %16, %1, vcc\n\t"
                "v_cmp_gt_u32 vcc, %2, %16\n\tv_cndmask_b32 %3, %16, %3, vcc\n\t"
                "v_cmp_gt_u32 vcc, %4, %16\n\tv_cndmask_b32 %5, %16, %5, vcc\n\t"
                "v_cmp_gt_u32 vcc, %6, %16\n\tv_cndmask_b32 %7, %16, %7, vcc\n\t"
                "v_cmp_gt_u32 vcc, %8, %16\n\tv_cndmask_b32 %9, %16, %9, vcc\n\t"
                "v_cmp_gt_u32 vcc, %10, %16\n\tv_cndmask_b32 %11, %16, %11, vcc\n\t"
                "v_cmp_gt_u32 vcc, %12, %16\n\tv_cndmask_b32 %13, %16, %13, vcc\n\t"
                "v_cmp_gt_u32 vcc, %14, %16\n\tv_cndmask_b32 %15, %16, %15, vcc"
                : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]),
                  "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15])
                : "v"(a), "v"(b)
                : "vcc");
        }
        if constexpr (OP == 25) PVAC_IP16(PVAC_IPS("v_cndmask_b32_e64", "%16,", ",vcc"));
        if constexpr (OP == 26) PVAC_IP16(PVAC_IPS("v_addc_co_u32", "vcc,", ",%16,vcc"));
        if constexpr (OP == 27) PVAC_IP16(PVAC_IPS("v_addc_co_u32_e64", "s[4:5],", ",%16,s[6:7]"));
        if constexpr (OP == 28) {   // 8 x (v_cmp_e64 writing an SGPR pair, v_cndmask_e64 reading it)
            asm volatile(
                "v_cmp_gt_u32_e64 s[4:5], %0, %16\n\tv_cndmask_b32_e64 %1, %16, %1, s[4:5]\n\t"
                "v_cmp_gt_u32_e64 s[6:7], %2, %16\n\tv_cndmask_b32_e64 %3, %16, %3, s[6:7]\n\t"
                "v_cmp_gt_u32_e64 s[4:5], %4, %16\n\tv_cndmask_b32_e64 %5, %16, %5, s[4:5]\n\t"
                "v_cmp_gt_u32_e64 s[6:7], %6, %16\n\tv_cndmask_b32_e64 %7, %16, %7, s[6:7]\n\t"
                "v_cmp_gt_u32_e64 s[4:5], %8, %16\n\tv_cndmask_b32_e64 %9, %16, %9, s[4:5]\n\t"
                "v_cmp_gt_u32_e64 s[6:7], %10, %16\n\tv_cndmask_b32_e64 %11, %16, %11, s[6:7]\n\t"
                "v_cmp_gt_u32_e64 s[4:5], %12, %16\n\tv_cndmask_b32_e64 %13, %16, %13, s[4:5]\n\t"
                "v_cmp_gt_u32_e64 s[6:7], %14, %16\n\tv_cndmask_b32_e64 %15, %16, %15, s[6:7]"
                : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]),
                  "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15])
                : "v"(a), "v"(b)
                : "s4", "s5", "s6", "s7");
        }
        if constexpr (OP == 29) PVAC_IP16(PVAC_IPS("v_min_u32_e64", "", ",%16"));
        if constexpr (OP == 30) PVAC_IP16(PVAC_IPS("v_add_u32_e64", "", ",%16"));
        if constexpr (OP == 31) PVAC_IP16(PVAC_IPS("v_and_b32", "", ",%16"));
        if constexpr (OP == 32) PVAC_IP16(PVAC_IPS("v_or_b32", "", ",%16"));
        if constexpr (OP == 33) PVAC_IP16(PVAC_IPS("v_lshrrev_b32", "%16,", ""));
        if constexpr (OP == 34) PVAC_IP16(PVAC_IPS("v_mov_b32", "", ""));
        if constexpr (OP == 35) PVAC_IP16(PVAC_IPS("v_max_u32", "", ",%16"));
        // SDWA forms (k_sigma's column flips use them)
        if constexpr (OP == 36)
            PVAC_IP16(PVAC_IPS("v_add_u32_sdwa", "", ",%16 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"));
        if constexpr (OP == 37)
            PVAC_IP16(PVAC_IPS("v_lshlrev_b32_sdwa", "%16,", " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"));
        if constexpr (OP == 38) PVAC_IP16(PVAC_IPS("v_lshlrev_b32_sdwa", "", ",%16 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"));
        if constexpr (OP == 39) PVAC_IP16(PVAC_IPS("v_xor_b32_e64", "", ",%16"));
        if constexpr (OP == 40) PVAC_IP16(PVAC_IPS("v_mad_u32_u24", "", ",%16,%17"));
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc ^= r[k];
    out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), q1 = __builtin_amdgcn_s_memrealtime();
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = q1 - q0;
    }
}
#undef PVAC_IP16
#undef PVAC_IPS
#undef PVAC_IPK

constexpr int kIssueOps = 41;
using probe_fn = void (*)(uint64_t*, uint64_t*, uint32_t, uint32_t);
template <int... I>
constexpr auto issue_table(std::integer_sequence<int, I...>) {
    return std::array<probe_fn, sizeof...(I)>{&k_probe_issue<I>...};
}

}  // namespace

// Per-opcode VALU issue probe (pvac_hip_issue_probe): wave64 instructions per second chip-wide and
// the shader clock measured inside the same launch (median over workgroups of s_memtime ticks per
// s_memrealtime tick x 100 MHz). The launch fills every CU with `wps` waves per SIMD.
hipError_t run_issue_probe(int op, int wps, int num_cus, hipStream_t st, double* per_s, double* clock_hz) {
    static const auto table = issue_table(std::make_integer_sequence<int, kIssueOps>{});
    if (op < 0 || op >= kIssueOps || wps < 1 || wps > 8) return hipErrorInvalidValue;
    const uint32_t threads = 256u;                                      // 4 waves: one per SIMD
    const uint32_t blocks = (uint32_t)num_cus * (uint32_t)wps;          // wps workgroups per CU
    const uint32_t iters = 8192u;
    const double per_iter = op == 16 ? 8.0 : 16.0;
    uint64_t *buf = nullptr, *clk = nullptr;
    hipError_t e = hipMalloc(&buf, (size_t)blocks * threads * 8);
    if (e == hipSuccess) e = hipMalloc(&clk, (size_t)blocks * 16);
    if (e != hipSuccess) {
        hipFree(buf);
        return e;
    }
    hipEvent_t t0, t1;
    hipEventCreate(&t0);
    hipEventCreate(&t1);
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {   // the first launches warm clocks and code
        hipEventRecord(t0, st);
        hipLaunchKernelGGL(table[op], dim3(blocks), dim3(threads), 0, st, buf, clk, iters, 0x5EEDu + rep);
        hipEventRecord(t1, st);
    }
    e = hipGetLastError();
    if (e == hipSuccess) e = hipEventSynchronize(t1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, t0, t1);
    std::vector<uint64_t> h((size_t)blocks * 2);
    if (e == hipSuccess) e = hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
    hipEventDestroy(t0);
    hipEventDestroy(t1);
    hipFree(buf);
    hipFree(clk);
    if (e != hipSuccess) return e;
    std::vector<double> hz;
    hz.reserve(blocks);
    for (uint32_t k = 0; k < blocks; ++k)
        if (h[2 * k + 1]) hz.push_back((double)h[2 * k] / (double)h[2 * k + 1] * 1.0e8);
    std::sort(hz.begin(), hz.end());
    *clock_hz = hz.empty() ? 0.0 : hz[hz.size() / 2];
    const double insts = (double)blocks * (threads / 64) * iters * per_iter;
    *per_s = ms > 0 ? insts / (ms / 1000.0) : 0.0;
    return hipSuccess;
}

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
