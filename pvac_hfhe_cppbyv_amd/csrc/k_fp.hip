// k_fp.hip — element-wise Fp127 kernels (K1) and batch utility kernels.
//
// K1 fp_binop: HBM-bound streaming over SoA limb arrays. Each lane moves 16-byte
// (2-element) vectors of every input array; UNROLL independent vectors per lane keep
// 4*UNROLL 16-byte loads in flight, non-temporal (the data is touched once). 48 algorithmic
// bytes per element (2x16 in, 16 out).
#include "common.hpp"

namespace pvhip {

namespace {

// Streaming (non-temporal) loads and stores, 4 vectors per lane: 6.10-6.25 TB/s against 5.50-5.59
// with cached accesses and 2 vectors (cfg 2's 2^24-element add / mul, profiles/r06/ab/fp_ab.log)
#ifndef PVAC_FP_UNROLL   // A/B builds only
#define PVAC_FP_UNROLL 4
#endif
#ifndef PVAC_FP_NT   // A/B builds only
#define PVAC_FP_NT 1
#endif
constexpr int kFpBlock = 256;
constexpr int kFpUnroll = PVAC_FP_UNROLL;

typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));
#ifndef PVAC_SCALE_NT   // A/B builds only: k_ct_scale's weights read and written non-temporally
#define PVAC_SCALE_NT 1
#endif
__device__ __forceinline__ uint64_t ld_stream64(const uint64_t* p) {
#if PVAC_SCALE_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
__device__ __forceinline__ void st_stream64(uint64_t* p, uint64_t v) {
#if PVAC_SCALE_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
__device__ __forceinline__ ulonglong2 ld_stream(const ulonglong2* p) {
#if PVAC_FP_NT
    const u64x2_t v = __builtin_nontemporal_load((const u64x2_t*)p);
    return make_ulonglong2(v.x, v.y);
#else
    return *p;
#endif
}
__device__ __forceinline__ void st_stream(ulonglong2* p, const ulonglong2& v) {
#if PVAC_FP_NT
    u64x2_t w;
    w.x = v.x;
    w.y = v.y;
    __builtin_nontemporal_store(w, (u64x2_t*)p);
#else
    *p = v;
#endif
}

template <int OP>
__device__ __forceinline__ fp apply(const fp& a, const fp& b) {
    if constexpr (OP == PVAC_FP_ADD) return fp_add(a, b);
    else if constexpr (OP == PVAC_FP_SUB) return fp_sub(a, b);
    else if constexpr (OP == PVAC_FP_NEG) return fp_neg(a);
    else if constexpr (OP == PVAC_FP_INV) return fp_inv(a);
    else return fp_mul(a, b);   // MUL and SCALE
}

template <int OP>
__global__ __launch_bounds__(kFpBlock) void k_fp_binop_vec(const ulonglong2* __restrict__ alo,
                                                           const ulonglong2* __restrict__ ahi,
                                                           const ulonglong2* __restrict__ blo,
                                                           const ulonglong2* __restrict__ bhi,
                                                           ulonglong2* __restrict__ clo, ulonglong2* __restrict__ chi,
                                                           size_t nvec, const uint64_t* __restrict__ sp_lo,
                                                           const uint64_t* __restrict__ sp_hi) {
    uint64_t slo = 0, shi = 0;
    if constexpr (OP == PVAC_FP_SCALE) { slo = sp_lo[0]; shi = sp_hi[0]; }
    const size_t stride = (size_t)gridDim.x * kFpBlock * kFpUnroll;
    for (size_t base = (size_t)blockIdx.x * kFpBlock * kFpUnroll + threadIdx.x; base < nvec; base += stride) {
        ulonglong2 al[kFpUnroll], ah[kFpUnroll], bl[kFpUnroll], bh[kFpUnroll];
#pragma unroll
        for (int u = 0; u < kFpUnroll; ++u) {
            const size_t v = base + (size_t)u * kFpBlock;
            if (v < nvec) {
                al[u] = ld_stream(alo + v);
                ah[u] = ld_stream(ahi + v);
                if constexpr (OP != PVAC_FP_NEG && OP != PVAC_FP_SCALE && OP != PVAC_FP_INV) {
                    bl[u] = ld_stream(blo + v);
                    bh[u] = ld_stream(bhi + v);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kFpUnroll; ++u) {
            const size_t v = base + (size_t)u * kFpBlock;
            if (v < nvec) {
                fp b0, b1;
                if constexpr (OP == PVAC_FP_SCALE) {
                    b0 = fp{slo, shi}; b1 = b0;
                } else if constexpr (OP == PVAC_FP_NEG || OP == PVAC_FP_INV) {
                    b0 = fp{0, 0}; b1 = b0;
                } else {
                    b0 = fp{bl[u].x, bh[u].x}; b1 = fp{bl[u].y, bh[u].y};
                }
                const fp r0 = apply<OP>(fp{al[u].x, ah[u].x}, b0);
                const fp r1 = apply<OP>(fp{al[u].y, ah[u].y}, b1);
                st_stream(clo + v, make_ulonglong2(r0.lo, r1.lo));
                st_stream(chi + v, make_ulonglong2(r0.hi, r1.hi));
            }
        }
    }
}

template <int OP>
__global__ __launch_bounds__(kFpBlock) void k_fp_binop_scalar(const uint64_t* alo, const uint64_t* ahi,
                                                              const uint64_t* blo, const uint64_t* bhi, uint64_t* clo,
                                                              uint64_t* chi, size_t lo_idx, size_t n) {
    for (size_t i = lo_idx + (size_t)blockIdx.x * kFpBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kFpBlock) {
        fp b{0, 0};
        if constexpr (OP == PVAC_FP_SCALE) b = fp{blo[0], bhi[0]};
        else if constexpr (OP != PVAC_FP_NEG && OP != PVAC_FP_INV) b = fp{blo[i], bhi[i]};
        const fp r = apply<OP>(fp{alo[i], ahi[i]}, b);
        clo[i] = r.lo;
        chi[i] = r.hi;
    }
}

template <int OP>
hipError_t run_binop(const uint64_t* alo, const uint64_t* ahi, const uint64_t* blo, const uint64_t* bhi, uint64_t* clo,
                     uint64_t* chi, size_t n, hipStream_t st) {
    auto aligned = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
    bool vec_ok = aligned(alo) && aligned(ahi) && aligned(clo) && aligned(chi);
    if constexpr (OP != PVAC_FP_NEG && OP != PVAC_FP_SCALE && OP != PVAC_FP_INV)
        vec_ok = vec_ok && aligned(blo) && aligned(bhi);
    size_t done = 0;
    if (vec_ok && n >= 2) {
        const size_t nvec = n / 2;
        size_t blocks = (nvec + (size_t)kFpBlock * kFpUnroll - 1) / ((size_t)kFpBlock * kFpUnroll);
        if (blocks > 65536) blocks = 65536;
        hipLaunchKernelGGL(k_fp_binop_vec<OP>, dim3((unsigned)blocks), dim3(kFpBlock), 0, st,
                           (const ulonglong2*)alo, (const ulonglong2*)ahi, (const ulonglong2*)blo,
                           (const ulonglong2*)bhi, (ulonglong2*)clo, (ulonglong2*)chi, nvec, blo, bhi);
        done = nvec * 2;
    }
    if (done < n) {
        size_t rem = n - done;
        size_t blocks = (rem + kFpBlock - 1) / kFpBlock;
        if (blocks > 65536) blocks = 65536;
        hipLaunchKernelGGL(k_fp_binop_scalar<OP>, dim3((unsigned)blocks), dim3(kFpBlock), 0, st, alo, ahi, blo, bhi,
                           clo, chi, done, n);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------- utilities
__global__ void k_fill_random(uint64_t seed, uint64_t* out, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t s = seed + i * 0x9e3779b97f4a7c15ULL;
        out[i] = splitmix64(s);
    }
}

// Fresh-shaped synthetic cipher generator (SURVEY §8(d) cfg 3): one thread per cipher.
// Distinct (idx, ch) per layer drawn by rejection against an LDS bitmap, weights uniform
// nonzero canonical, edges grouped by layer and Fisher-Yates shuffled within each layer.
constexpr int kGenBlock = 64;
__global__ __launch_bounds__(kGenBlock) void k_gen_fresh(uint64_t seed, uint64_t first, uint32_t epl, uint32_t B,
                                                         pvac_ct_batch X) {
    extern __shared__ __attribute__((aligned(16))) uint64_t gen_lds[];
    const uint32_t words = (2 * B + 63) / 64;
    uint64_t* used = gen_lds + (size_t)threadIdx.x * words;
    const uint64_t i = (uint64_t)blockIdx.x * kGenBlock + threadIdx.x;
    if (i >= X.n) return;
    // keyed by the GLOBAL cipher index: a shard [first, first + n) reproduces a 1-GPU batch
    uint64_t s = seed ^ ((first + i) * 0xD1B54A32D192ED03ULL);
    (void)splitmix64(s);
    const uint64_t loff = 2 * i, eoff = 2ull * epl * i;
    X.l_off[i] = loff;
    X.l_cnt[i] = 2;
    X.e_off[i] = eoff;
    X.e_cnt[i] = 2ull * epl;
    for (uint32_t l = 0; l < 2; ++l) {
        pvac_layer L;
        L.rule = 0; L.pa = 0; L.pb = 0; L.pad = 0;
        L.ztag = splitmix64(s);
        L.nonce_lo = splitmix64(s);
        L.nonce_hi = splitmix64(s);
        X.layers[loff + l] = L;
        for (uint32_t w = 0; w < words; ++w) used[w] = 0;
        const uint64_t e0 = eoff + (uint64_t)l * epl;
        for (uint32_t k = 0; k < epl; ++k) {
            uint32_t slot;
            do { slot = (uint32_t)(splitmix64(s) % (2ull * B)); } while ((used[slot >> 6] >> (slot & 63)) & 1ull);
            used[slot >> 6] |= 1ull << (slot & 63);
            fp w;
            do { w = fp_from_words(splitmix64(s), splitmix64(s) & kM63); } while (!fp_nonzero(w));
            X.meta[e0 + k] = make_meta(l, slot >> 1, slot & 1);
            X.w_lo[e0 + k] = w.lo;
            X.w_hi[e0 + k] = w.hi;
        }
        for (uint32_t k = epl - 1; k > 0; --k) {   // Fisher-Yates within the layer
            const uint32_t j = (uint32_t)(splitmix64(s) % (k + 1));
            const uint64_t m = X.meta[e0 + k], a = X.w_lo[e0 + k], b = X.w_hi[e0 + k];
            X.meta[e0 + k] = X.meta[e0 + j]; X.w_lo[e0 + k] = X.w_lo[e0 + j]; X.w_hi[e0 + k] = X.w_hi[e0 + j];
            X.meta[e0 + j] = m; X.w_lo[e0 + j] = a; X.w_hi[e0 + j] = b;
        }
    }
}

// Product-layer nonces keyed by (seed, GLOBAL pair index, product layer): word 2k/2k+1 of the
// product layer (la, lb) of pair i sits at its output layer slot (ABI nonce convention).
__global__ void k_fill_nonces(uint64_t seed, uint64_t first, pvac_ct_batch A, pvac_ct_batch B, const uint64_t* c_l_off,
                              uint64_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.n) return;
    const uint64_t LA = A.l_cnt[i], LB = B.l_cnt[i];
    const uint64_t s0 = c_l_off[i] + LA + LB;
    for (uint64_t k = 0; k < LA * LB; ++k) {
        uint64_t s = seed ^ ((first + i) * 0xD1B54A32D192ED03ULL) ^ (k * 0x8CB92BA72F3D8DD7ULL);
        out[2 * (s0 + k)] = splitmix64(s);
        out[2 * (s0 + k) + 1] = splitmix64(s);
    }
}

__device__ __forceinline__ uint64_t fnv_u64(uint64_t h, uint64_t x) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { h ^= (x >> (8 * i)) & 0xFF; h *= 0x100000001b3ULL; }
    return h;
}

__global__ void k_batch_digest(pvac_ct_batch X, uint64_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= X.n) return;
    uint64_t h = 0xcbf29ce484222325ULL;
    const uint64_t o = X.e_off[i], c = X.e_cnt[i];
    for (uint64_t e = 0; e < c; ++e) {
        h = fnv_u64(h, X.meta[o + e]);
        h = fnv_u64(h, X.w_lo[o + e]);
        h = fnv_u64(h, X.w_hi[o + e]);
    }
    out[i] = h;
}

// Position-keyed digest: sum over a cipher's edges e of mix64(e, meta, w_lo, w_hi) (mod 2^64). Order-
// sensitive through the position e, but a sum, so one workgroup per cipher reduces it in parallel
// (the FNV digest above walks the edges serially: ~12 ms per depth-8 cipher).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_batch_sumdigest(pvac_ct_batch X, uint64_t* out) {
    __shared__ uint64_t part[4];
    const uint64_t i = blockIdx.x;
    const uint64_t o = X.e_off[i], c = X.e_cnt[i];
    uint64_t acc = 0;
    for (uint64_t e = threadIdx.x; e < c; e += 256) {
        const uint64_t m = X.meta[o + e], lo = X.w_lo[o + e], hi = X.w_hi[o + e];
        acc += mix64(mix64(mix64(e * 0x9E3779B97F4A7C15ULL ^ m) ^ lo) ^ hi);
    }
    for (int d = 32; d >= 1; d >>= 1) acc += __shfl_xor(acc, d);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) out[i] = part[0] + part[1] + part[2] + part[3] + c;
}

// ct_scale (arithmetic.hpp:33-37), in place: 32 lanes per cipher, eight ciphers per workgroup
// (fresh ciphers have ~40 edges; a workgroup per cipher left most lanes idle)
__global__ __launch_bounds__(256) void k_ct_scale(pvac_ct_batch X, uint64_t slo, uint64_t shi) {
    const uint64_t c = (uint64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
    if (c >= X.n) return;
    const uint64_t o = X.e_off[c], n = X.e_cnt[c];
    const fp s{slo, shi};
    // the first 64 weights (every fresh cipher: 40) are all loaded before the first store: the
    // update is in place, so loads issued after a store could not be hoisted above it
    constexpr int kPre = 2;
    const uint64_t e0 = threadIdx.x & 31u;
    fp w[kPre];
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
        const uint64_t e = e0 + 32u * u;
        w[u] = fp{0, 0};
        if (e < n) w[u] = fp{ld_stream64(X.w_lo + o + e), ld_stream64(X.w_hi + o + e)};
    }
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
        const uint64_t e = e0 + 32u * u;
        if (e < n) {
            const fp r = fp_mul(w[u], s);
            st_stream64(X.w_lo + o + e, r.lo);
            st_stream64(X.w_hi + o + e, r.hi);
        }
    }
    for (uint64_t e = e0 + 32u * kPre; e < n; e += 32) {
        const fp r = fp_mul(fp{ld_stream64(X.w_lo + o + e), ld_stream64(X.w_hi + o + e)}, s);
        st_stream64(X.w_lo + o + e, r.lo);
        st_stream64(X.w_hi + o + e, r.hi);
    }
}

}  // namespace

hipError_t launch_fp_binop(int op, const uint64_t* alo, const uint64_t* ahi, const uint64_t* blo, const uint64_t* bhi,
                           uint64_t* clo, uint64_t* chi, size_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    switch (op) {
        case PVAC_FP_ADD: return run_binop<PVAC_FP_ADD>(alo, ahi, blo, bhi, clo, chi, n, st);
        case PVAC_FP_SUB: return run_binop<PVAC_FP_SUB>(alo, ahi, blo, bhi, clo, chi, n, st);
        case PVAC_FP_MUL: return run_binop<PVAC_FP_MUL>(alo, ahi, blo, bhi, clo, chi, n, st);
        case PVAC_FP_NEG: return run_binop<PVAC_FP_NEG>(alo, ahi, blo, bhi, clo, chi, n, st);
        case PVAC_FP_SCALE: return run_binop<PVAC_FP_SCALE>(alo, ahi, blo, bhi, clo, chi, n, st);
        case PVAC_FP_INV: return run_binop<PVAC_FP_INV>(alo, ahi, blo, bhi, clo, chi, n, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_fill_random(uint64_t seed, uint64_t* out, size_t n, hipStream_t st) {
    if (!n) return hipSuccess;
    size_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_fill_random, dim3((unsigned)blocks), dim3(256), 0, st, seed, out, n);
    return hipGetLastError();
}

hipError_t launch_fill_nonces(uint64_t seed, uint64_t first, const pvac_ct_batch& A, const pvac_ct_batch& B,
                              const uint64_t* c_l_off, uint64_t* out, hipStream_t st) {
    if (!A.n) return hipSuccess;
    hipLaunchKernelGGL(k_fill_nonces, dim3((unsigned)((A.n + 255) / 256)), dim3(256), 0, st, seed, first, A, B,
                       c_l_off, out);
    return hipGetLastError();
}

hipError_t launch_gen_fresh(uint64_t seed, uint64_t first, uint32_t epl, uint32_t B, const pvac_ct_batch& X,
                            hipStream_t st) {
    if (!X.n) return hipSuccess;
    if (epl == 0 || epl > 2 * B) return hipErrorInvalidValue;
    const size_t words = (2 * B + 63) / 64;
    const size_t lds = words * 8 * kGenBlock;
    const size_t blocks = (X.n + kGenBlock - 1) / kGenBlock;
    hipLaunchKernelGGL(k_gen_fresh, dim3((unsigned)blocks), dim3(kGenBlock), lds, st, seed, first, epl, B, X);
    return hipGetLastError();
}

hipError_t launch_batch_digest(const pvac_ct_batch& X, uint64_t* out, hipStream_t st) {
    if (!X.n) return hipSuccess;
    hipLaunchKernelGGL(k_batch_digest, dim3((unsigned)((X.n + 255) / 256)), dim3(256), 0, st, X, out);
    return hipGetLastError();
}

hipError_t launch_batch_sumdigest(const pvac_ct_batch& X, uint64_t* out, hipStream_t st) {
    if (!X.n) return hipSuccess;
    hipLaunchKernelGGL(k_batch_sumdigest, dim3((unsigned)X.n), dim3(256), 0, st, X, out);
    return hipGetLastError();
}

hipError_t launch_ct_scale(const pvac_ct_batch& X, uint64_t slo, uint64_t shi, hipStream_t st) {
    if (!X.n) return hipSuccess;
    hipLaunchKernelGGL(k_ct_scale, dim3((unsigned)((X.n + 7) / 8)), dim3(256), 0, st, X, slo, shi);
    return hipGetLastError();
}

}  // namespace pvhip
