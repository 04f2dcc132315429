// k_check.hip — batched gsum invariant of ct_mul (reference utils/metrics.hpp:70-113).
//
// The reference's check_mul_gsum_all(pk, A, B, C) asserts, for every layer pair (la, lb),
//     gsum(C, lc) == gsum(A, la) * gsum(B, lb),   gsum(X, l) = sum over X's edges in layer l of
//     +/- w * powg_B[idx]  (+ for SGN_P, - otherwise; agg_layer_gsum, metrics.hpp:70-86),
// with lc = |A.L| + |B.L| + la |B.L| + lb, i.e. on C before compact_layers renumbers it. It holds
// because powg_B[i] = g^i with g^B = 1, so a product edge's g^((ia + ib) mod B) = g^ia g^ib.
// Here C is the compacted output, so the product layer of (la, lb) is found by its nonce: the
// caller's nonce words for that pair's slot (the ct_mul ABI's randomness input) must equal the
// nonce of exactly the C layer that holds its edges. A layer pair whose product layer was dropped
// (no edge emitted) must have gsum(A, la) * gsum(B, lb) == 0; a C layer with edges that is not a
// product layer fails the check.
//
// One 256-thread workgroup per pair (persistent over the batch). The layer tables live in LDS while
// they fit (to depth 8 of the cfg-4 chains); deeper steps (depth 9: |C.L| ~ 3,100 layers of 48-byte
// sums) run the same code over a per-workgroup slab of global scratch. Per-layer sums are exact: each
// canonical term is split into 43/42/42-bit limbs (fp_split3) and summed per (layer, channel) with
// LDS u64 atomics (< 2^21 edges per cipher), then folded and P - M taken once. Equal to the
// reference's fp_add / fp_sub chains, which compute exact residues for canonical terms.
// Status per pair: 0 holds, 1 violated, 2 an edge idx >= B (the reference reads past powg_B),
// 3 too many edges (> 2^21 in one cipher: the limb sums could overflow; not checked).
#include <algorithm>

#include "common.hpp"

namespace pvhip {
namespace {

constexpr int kCB = 256;

__device__ __forceinline__ uint32_t wmax(uint32_t v) {
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d, 64));
    return v;
}

struct check_args {
    pvac_ct_batch A, B, C;
    const uint64_t* nonces;
    const ulonglong2* powg;
    uint32_t Bm;
    uint32_t* status;
    unsigned long long* n_bad;
    uint8_t* gscratch;      // global mode: per-workgroup slabs of gstride bytes (else null: LDS)
    uint64_t gstride;
};

struct check_lds {   // byte offsets into dynamic LDS
    uint32_t powg, accA, accB, accC, cntC, cand, found, total;
};

__host__ __device__ inline uint32_t al16(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ inline check_lds check_layout(uint32_t Bm, uint32_t la, uint32_t lb, uint32_t lc, uint32_t lp) {
    check_lds L;
    uint32_t o = 0;
    L.powg = o;  o = al16(o + Bm * 16u);
    L.accA = o;  o = al16(o + la * 48u);
    L.accB = o;  o = al16(o + lb * 48u);
    L.accC = o;  o = al16(o + lc * 48u);
    L.cntC = o;  o = al16(o + lc * 4u);
    L.cand = o;  o = al16(o + lp * 16u);
    L.found = o; o = al16(o + lp * 4u);
    L.total = o;
    return L;
}

// sums of one cipher's edges into acc[layer][P0 P1 P2 M0 M1 M2]; flags idx >= B
__device__ void gsum_edges(const pvac_ct_batch& X, uint64_t eo, uint64_t ne, uint32_t L, const ulonglong2* pg,
                           uint32_t Bm, unsigned long long* acc, uint32_t* cnt, uint32_t& bad) {
    for (uint64_t e = threadIdx.x; e < ne; e += kCB) {
        const uint64_t m = X.meta[eo + e];
        const uint32_t l = meta_layer(m), idx = meta_idx(m);
        if (idx >= Bm) {
            bad = 2u;
            continue;
        }
        if (l >= L) continue;   // matches no layer id of the reference's loops
        const ulonglong2 g = pg[idx];
        const fp t = fp_mul(fp{X.w_lo[eo + e], X.w_hi[eo + e]}, fp{g.x, g.y});
        uint64_t l0, l1, l2;
        fp_split3(t, l0, l1, l2);
        unsigned long long* a = acc + 6u * l + (meta_ch(m) == 0 ? 0u : 3u);
        atomicAdd(a, (unsigned long long)l0);
        atomicAdd(a + 1, (unsigned long long)l1);
        atomicAdd(a + 2, (unsigned long long)l2);
        if (cnt) atomicAdd(cnt + l, 1u);
    }
}

// acc[l] -> (P - M) mod p into its first two words
__device__ void gsum_fold(unsigned long long* acc, uint32_t L) {
    for (uint32_t l = threadIdx.x; l < L; l += kCB) {
        unsigned long long* a = acc + 6u * l;
        const fp P = fp_fold3(a[0], a[1], a[2]), M = fp_fold3(a[3], a[4], a[5]);
        const fp s = fp_sub(P, M);
        a[0] = s.lo;
        a[1] = s.hi;
    }
}

template <bool kGlobal>
__global__ __launch_bounds__(kCB) void k_check_gsum(check_args g, check_lds Ls) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
    uint8_t* lds = kGlobal ? g.gscratch + (uint64_t)blockIdx.x * g.gstride : lds_dyn;
    ulonglong2* pg = (ulonglong2*)(lds + Ls.powg);
    unsigned long long* accA = (unsigned long long*)(lds + Ls.accA);
    unsigned long long* accB = (unsigned long long*)(lds + Ls.accB);
    unsigned long long* accC = (unsigned long long*)(lds + Ls.accC);
    uint32_t* cntC = (uint32_t*)(lds + Ls.cntC);
    ulonglong2* cand = (ulonglong2*)(lds + Ls.cand);
    uint32_t* found = (uint32_t*)(lds + Ls.found);
    __shared__ uint32_t bad;
    for (uint32_t i = threadIdx.x; i < g.Bm; i += kCB) pg[i] = g.powg[i];
    for (uint64_t p = blockIdx.x; p < g.A.n; p += gridDim.x) {
        const uint32_t LA = (uint32_t)g.A.l_cnt[p], LB = (uint32_t)g.B.l_cnt[p], LC = (uint32_t)g.C.l_cnt[p];
        const uint64_t nA = g.A.e_cnt[p], nB = g.B.e_cnt[p], nC = g.C.e_cnt[p];
        const uint32_t LP = LA * LB;
        const uint64_t cslot = g.C.l_off[p] + LA + LB;   // nonce slot of product layer (0, 0)
        if (threadIdx.x == 0) bad = (nA >> 21) | (nB >> 21) | (nC >> 21) ? 3u : 0u;
        for (uint32_t w = threadIdx.x; w < 6u * (LA + LB + LC); w += kCB) {
            // accA, accB, accC are laid out back to back up to 16-byte alignment: clear each
            const uint32_t l = w / 6u, f = w - 6u * l;
            unsigned long long* a = l < LA ? accA + 6u * l : l < LA + LB ? accB + 6u * (l - LA) : accC + 6u * (l - LA - LB);
            a[f] = 0;
        }
        for (uint32_t l = threadIdx.x; l < LC; l += kCB) cntC[l] = 0;
        for (uint32_t q = threadIdx.x; q < LP; q += kCB) {
            cand[q] = make_ulonglong2(g.nonces[2 * (cslot + q)], g.nonces[2 * (cslot + q) + 1]);
            found[q] = 0;
        }
        if (kGlobal) __threadfence();   // global slab: each phase's writes / atomics visible to the next
        __syncthreads();
        if (bad != 3u) {
            uint32_t b = 0;
            gsum_edges(g.A, g.A.e_off[p], nA, LA, pg, g.Bm, accA, nullptr, b);
            gsum_edges(g.B, g.B.e_off[p], nB, LB, pg, g.Bm, accB, nullptr, b);
            gsum_edges(g.C, g.C.e_off[p], nC, LC, pg, g.Bm, accC, cntC, b);
            if (b) bad = b;
        }
        if (kGlobal) __threadfence();
        __syncthreads();
        gsum_fold(accA, LA);
        gsum_fold(accB, LB);
        gsum_fold(accC, LC);
        if (kGlobal) __threadfence();
        __syncthreads();
        if (bad == 0u) {
            // every C layer with edges is the product layer of the (la, lb) whose nonce it carries
            for (uint32_t l = threadIdx.x; l < LC; l += kCB) {
                if (!cntC[l]) continue;
                const pvac_layer y = g.C.layers[g.C.l_off[p] + l];
                uint32_t q = LP;
                for (uint32_t k = 0; k < LP; ++k)
                    if (cand[k].x == y.nonce_lo && cand[k].y == y.nonce_hi) {
                        q = k;
                        break;
                    }
                if (q == LP || y.rule != 1u) {
                    bad = 1u;
                    continue;
                }
                found[q] = 1u;
                const uint32_t la = q / LB, lb = q - la * LB;
                const fp e = fp_mul(fp{accA[6u * la], accA[6u * la + 1]}, fp{accB[6u * lb], accB[6u * lb + 1]});
                if (e.lo != accC[6u * l] || e.hi != accC[6u * l + 1]) bad = 1u;
            }
        }
        __syncthreads();
        if (bad == 0u) {
            // a dropped product layer: its gsum product must vanish
            for (uint32_t q = threadIdx.x; q < LP; q += kCB) {
                if (found[q]) continue;
                const uint32_t la = q / LB, lb = q - la * LB;
                const fp e = fp_mul(fp{accA[6u * la], accA[6u * la + 1]}, fp{accB[6u * lb], accB[6u * lb + 1]});
                if (fp_nonzero(e)) bad = 1u;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            if (g.status) g.status[p] = bad;
            if (bad) atomicAdd(g.n_bad, 1ull);
        }
        __syncthreads();
    }
}

// launch sizing: max |A.L|, |B.L|, |C.L|, |A.L||B.L| over the batch
__global__ __launch_bounds__(kCB) void k_check_sizes(pvac_ct_batch A, pvac_ct_batch B, pvac_ct_batch C, unsigned int* mx) {
    uint32_t a = 0, b = 0, c = 0, pr = 0;
    for (uint64_t p = (uint64_t)blockIdx.x * kCB + threadIdx.x; p < A.n; p += (uint64_t)gridDim.x * kCB) {
        const uint64_t la = A.l_cnt[p], lb = B.l_cnt[p], lc = C.l_cnt[p];
        const uint64_t lp = la * lb;
        a = max(a, (uint32_t)min(la, 0xFFFFFFFFull));
        b = max(b, (uint32_t)min(lb, 0xFFFFFFFFull));
        c = max(c, (uint32_t)min(lc, 0xFFFFFFFFull));
        pr = max(pr, (uint32_t)min(lp, 0xFFFFFFFFull));
    }
    a = wmax(a); b = wmax(b); c = wmax(c); pr = wmax(pr);
    if ((threadIdx.x & 63) == 0) {
        atomicMax(mx, a);
        atomicMax(mx + 1, b);
        atomicMax(mx + 2, c);
        atomicMax(mx + 3, pr);
    }
}

}  // namespace

hipError_t launch_check_sizes(const pvac_ct_batch& A, const pvac_ct_batch& B, const pvac_ct_batch& C, unsigned int* mx,
                              hipStream_t st) {
    if (!A.n) return hipSuccess;
    uint64_t blocks = (A.n + kCB - 1) / kCB;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(k_check_sizes, dim3((unsigned)blocks), dim3(kCB), 0, st, A, B, C, mx);
    return hipGetLastError();
}

namespace {
constexpr uint32_t kCheckLds = 160u * 1024u;
uint64_t check_blocks(uint64_t n, int num_cus, bool global) {
    const uint64_t b = (uint64_t)num_cus * (global ? 2 : 8);
    return b > n ? n : b;
}
}  // namespace

// global scratch the check needs for the batch's largest tables (0: they fit LDS)
uint64_t check_gsum_scratch_bytes(uint32_t Bm, const unsigned int* mx_host, uint64_t n, int num_cus) {
    const check_lds L = check_layout(Bm, mx_host[0], mx_host[1], mx_host[2], mx_host[3]);
    if (L.total <= kCheckLds) return 0;
    return check_blocks(n, num_cus, true) * (uint64_t)al16(L.total);
}

// tables beyond LDS run over gscratch (check_gsum_scratch_bytes of it; hipErrorInvalidValue if null)
hipError_t launch_check_gsum(const pvac_ct_batch& A, const pvac_ct_batch& B, const pvac_ct_batch& C, const uint64_t* nonces,
                             const uint64_t* powg, uint32_t Bm, const unsigned int* mx_host, uint32_t* status,
                             unsigned long long* n_bad, int num_cus, uint8_t* gscratch, hipStream_t st) {
    if (!A.n) return hipSuccess;
    const check_lds L = check_layout(Bm, mx_host[0], mx_host[1], mx_host[2], mx_host[3]);
    const bool global = L.total > kCheckLds;
    if (global && !gscratch) return hipErrorInvalidValue;
    check_args g{A, B, C, nonces, (const ulonglong2*)powg, Bm, status, n_bad, global ? gscratch : nullptr,
                 al16(L.total)};
    const uint64_t blocks = check_blocks(A.n, num_cus, global);
    if (global)
        hipLaunchKernelGGL(k_check_gsum<true>, dim3((unsigned)blocks), dim3(kCB), 0, st, g, L);
    else
        hipLaunchKernelGGL(k_check_gsum<false>, dim3((unsigned)blocks), dim3(kCB), L.total, st, g, L);
    return hipGetLastError();
}

// Chain statistics (pvac_hip_ct_mul_chain): out[0] += sum of |C.E|, out[1] += sum of |A.E| |X.E| over the
// pairs of one step (the products the step multiplied). One block-reduced atomic per block.
namespace {
__global__ __launch_bounds__(256) void k_chain_stats(const uint64_t* a_cnt, const uint64_t* x_cnt, const uint64_t* c_cnt,
                                                     uint64_t n, unsigned long long* out) {
    __shared__ unsigned long long part[2][4];
    unsigned long long e = 0, p = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        e += c_cnt[i];
        p += a_cnt[i] * x_cnt[i];
    }
    for (int o = 32; o; o >>= 1) {
        e += __shfl_xor(e, o);
        p += __shfl_xor(p, o);
    }
    if ((threadIdx.x & 63) == 0) {
        part[0][threadIdx.x >> 6] = e;
        part[1][threadIdx.x >> 6] = p;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(out, part[0][0] + part[0][1] + part[0][2] + part[0][3]);
        atomicAdd(out + 1, part[1][0] + part[1][1] + part[1][2] + part[1][3]);
    }
}
}  // namespace

// chain worker staging (pvac_hip_ct_mul_chain, a chunk whose inputs live on another device or with
// PVAC_CHAIN_STAGE_INPUTS): cipher i's rows from src (its own offsets) to dst (offsets scanned from
// the counts already copied into dst); one workgroup per cipher, coalesced u64 copies; src pointers
// may be another GPU's memory (peer reads over xGMI)
__global__ __launch_bounds__(256) void k_stage_rows(pvac_ct_batch src, pvac_ct_batch dst) {
    const uint64_t i = blockIdx.x;
    const uint64_t nl = dst.l_cnt[i], ne = dst.e_cnt[i];
    const uint64_t* sL = (const uint64_t*)(src.layers + src.l_off[i]);
    uint64_t* dL = (uint64_t*)(dst.layers + dst.l_off[i]);
    static_assert(sizeof(pvac_layer) == 40, "layer record = 5 u64");
    for (uint64_t w = threadIdx.x; w < 5 * nl; w += 256) dL[w] = sL[w];
    const uint64_t se = src.e_off[i], de = dst.e_off[i];
    for (uint64_t e = threadIdx.x; e < ne; e += 256) {
        dst.meta[de + e] = src.meta[se + e];
        dst.w_lo[de + e] = src.w_lo[se + e];
        dst.w_hi[de + e] = src.w_hi[se + e];
    }
    if (dst.sigma) {   // pvac_hip_batch_pack of a batch with sigma: sigma_words per edge, contiguous
        const uint64_t sw = dst.sigma_words;
        const uint64_t* sS = src.sigma + se * sw;
        uint64_t* dS = dst.sigma + de * sw;
        for (uint64_t w = threadIdx.x; w < ne * sw; w += 256) dS[w] = sS[w];
    }
}

hipError_t launch_stage_rows(const pvac_ct_batch& src, const pvac_ct_batch& dst, hipStream_t st) {
    if (!dst.n) return hipSuccess;
    hipLaunchKernelGGL(k_stage_rows, dim3((unsigned)dst.n), dim3(256), 0, st, src, dst);
    return hipGetLastError();
}

hipError_t launch_chain_stats(const pvac_ct_batch& A, const pvac_ct_batch& X, const pvac_ct_batch& C,
                              unsigned long long* out, hipStream_t st) {
    if (!A.n) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<uint64_t>((A.n + 255) / 256, 1024);
    hipLaunchKernelGGL(k_chain_stats, dim3(blocks), dim3(256), 0, st, A.e_cnt, X.e_cnt, C.e_cnt, A.n, out);
    return hipGetLastError();
}

}  // namespace pvhip
