// k_mul_large.hip — batched ct_mul for general pairs (reference ops/arithmetic.hpp:47-106):
// chains c_k = c_{k-1} * x (test_main.cpp:289-295), squares (test_depth.cpp:46), any pair the
// LDS-resident fresh kernel cannot hold.
//
// The reference aggregates |A.E||B.E| products in one std::unordered_map. Here the product
// space is cut along its natural independence: every product of an A edge in layer la and a
// B edge in layer lb lands in product layer lp = la*LB + lb, a cyclic convolution of length B
// over Fp with +/- channels. One workgroup owns one (la, lb) TASK:
//   dense-owner mode : the side with more edges becomes a dense [2][B] table of 26-bit limbs in
//                      LDS; one lane per output index r loops over the other side's edges and
//                      accumulates P/M sums as nine u64 columns each (25 v_mad_u64_u32 per
//                      product, no carry chain; fp127.hpp col26_*) and the key's first-insert time
//                      in REGISTERS (no atomics). For saturated chain layers (674 edges) every
//                      probe is useful.
//   scatter mode     : sparse x sparse tasks (and inputs with duplicate (layer, idx, ch) edges)
//                      accumulate 43/42/42-bit limbs with LDS atomics, as the fresh kernel.
// Results go to a dense per-pair key-slot array [|A.L||B.L|][B] in global scratch.
//
// The reference's emit order (hash-table list order: bucket first-insert time DESC, key
// first-insert time DESC; see k_mul_fresh.hip) is rebuilt without sorting:
//   link  : key -> libstdc++ bucket (hash * 0x9E37... mod bucket_count), bucket chains through
//           a global open-addressing table keyed by bucket id;
//   rank  : each key walks its (short) chain: bucket first-insert time t_b, edges of its bucket
//           emitted before it; bucket leaders mark bit t_b in a 64-bit mask per 64 first-insert
//           times and add their bucket's edge count to that block;
//   scan  : suffix scan over blocks (n/64 entries, not n);
//   order : position = block offset + edges of leaders later in the same block (mask bits above,
//           each resolved to its key slot from the leader's (i, j) = (t / |B.E|, t % |B.E|)) +
//           rank inside the bucket; slot ids are scattered into an order array (4 B each);
//   write : one coalesced pass writes (meta, w) in order.
// compact_layers (encrypt.hpp:73-104) runs per pair between aggregation and write, so edges
// are written once with their final layer ids; guard_budget (encrypt.hpp:106-111) switches a
// pair to (layer, idx, P<M) order when its edge count exceeds edge_budget.
#include "common.hpp"
#include "sha256.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#ifdef PVAC_DIR_STAMPS   // diagnostic build only: k_large_products_direct's wave 0 s_memtime per phase
__device__ unsigned long long g_dir_stamps[24];
extern "C" int pvac_hip_diag_dir_stamps(unsigned long long* host, int reset) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dir_stamps), sizeof(g_dir_stamps)) != hipSuccess) return -5;
    if (reset) {
        unsigned long long z[24] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_dir_stamps), z, sizeof(z)) != hipSuccess) return -5;
    }
    return 0;
}
__device__ __forceinline__ unsigned long long dir_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define DSTAMP(ph) do { const unsigned long long t_ = dir_stamp(); st_acc[ph] += t_ - t_prev; t_prev = t_; } while (0)
#else
#define DSTAMP(ph) do {} while (0)
#endif

namespace pvhip {

namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kIblkMaxSparse = 20;   // == kMxMaxSparse: B layers the matrix-core mode takes
constexpr int kLB = 256;            // threads per workgroup (task / grid-stride kernels)
constexpr int kLBig = 1024;         // threads per workgroup (per-pair kernels)

__device__ __forceinline__ uint64_t* w64(uint32_t* s, uint64_t o) { return (uint64_t*)(s + o); }

__device__ __forceinline__ uint32_t mod_small(uint32_t x, uint32_t B) { return x >= B ? x - B : x; }

// a bucket leader with first-insert time t and E > 0 edges: its 2-bit edge code lands in the u64
// of its 16-time block (times are unique, so the add is an OR) and E in the block's count
__device__ __forceinline__ void leader_mark(unsigned long long* bpack, uint32_t t, uint32_t E) {
    const uint64_t code = E < 3u ? E : 3u;
    atomicAdd(&bpack[t >> 4], ((unsigned long long)E << 32) | (code << (2u * (t & 15u))));
}

// static bucket groups (large_desc::g_head): 0 = the key is alone in its libstdc++ bucket
__device__ __forceinline__ const uint32_t* group_heads(const mul_large_args& g, const large_desc& d) {
    return d.g_head != kNoGrp ? g.grp + d.g_head : nullptr;
}

// workgroup exclusive scan for any multiple-of-64 block size
template <int BS>
__device__ __forceinline__ uint32_t wg_exclusive_scan(uint32_t v, uint32_t* part, uint32_t& total) {
    return block_exclusive_scan<BS>(v, part, total);
}

// ---------------------------------------------------------------- init
// iblk pairs leave the block marks alone (k_large_layers clears them for a pair that falls back)
// and tkey (iblk_dead): only cnt and the used flags are zeroed (static groups have no bucket table)
__global__ __launch_bounds__(kLB) void k_large_init(mul_large_args g) {
    const large_desc& d = g.desc[blockIdx.y];
    const uint64_t stride = (uint64_t)gridDim.x * kLB;
    const uint64_t nz = d.iblk ? kCntWords + d.Lc : d.zero_words;
    const uint64_t nt = d.iblk ? 0 : d.S;   // iblk: products sets every slot of a live layer pair
    const uint64_t lim = nz > nt ? nz : nt;
    for (uint64_t w = (uint64_t)blockIdx.x * kLB + threadIdx.x; w < lim; w += stride) {
        if (w < nz) g.scratch[d.iblk && w >= kCntWords ? d.o_used + (w - kCntWords) : d.o_zero + w] = 0;
        if (w < nt) g.scratch[d.o_tkey + w] = kInf;
    }
}

// iblk pairs leave tkey unset in the layer pairs (la, lb) with no edges on one side: no products
// there, so no keys; the passes that walk every slot skip them
__device__ __forceinline__ bool iblk_dead(const uint32_t* S, const large_desc& d, uint64_t s, uint32_t Bm) {
    if (!d.iblk) return false;
    const uint32_t lp = (uint32_t)s / Bm, la = lp / d.LB, lb = lp - la * d.LB;
    return S[d.o_lstA + d.LA + la] == 0u || S[d.o_lstB + d.LB + lb] == 0u;
}

// ---------------------------------------------------------------- per-layer edge lists
// One workgroup per pair: validates edges (layer < |L|, idx < B, ch <= 1), buckets edge ids
// by layer (any order inside a layer: first-insert times are minima, not positions) and
// lists the non-empty layers of both sides.
#ifndef PVAC_LIST_REG_ROUNDS   // rounds of 4 x kLBig A edges whose pass 2 reads registers
#define PVAC_LIST_REG_ROUNDS 8
#endif
constexpr uint32_t kListRegRounds = PVAC_LIST_REG_ROUNDS;
static_assert(kLargeLayersMax <= (1u << 15), "k_large_lists packs a layer in 15 bits");
__global__ __launch_bounds__(kLBig) void k_large_lists(mul_large_args g) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];   // [LA + LB] counts, then cursors
    __shared__ uint32_t flag;
    const large_desc& d = g.desc[blockIdx.x];
    const uint64_t pr = d.pair;
    const uint32_t LA = d.LA, LB = d.LB, nA = d.nA, nB = d.nB, Bm = g.Bm;
    const uint64_t aeo = g.A.e_off[pr], beo = g.B.e_off[pr];
    uint32_t* S = g.scratch;
    uint32_t* cnt = S + d.o_cnt;
    const int tid = threadIdx.x;
    for (uint32_t l = tid; l < LA + LB; l += kLBig) hist[l] = 0;
    if (tid == 0) flag = 0;
    __syncthreads();
    // A as a dense chain image (mul_large_args::A_img, written by the previous step's
    // k_large_products_direct): layer l >= first holds the 2B edges [(l - first) 2B, (l - first + 1) 2B)
    // in cell order, and 32-bit word s of the pair's meta region is slot s's direct id (hash-order
    // edge | cell << 21): the lists are the slabs themselves, nothing to validate or bucket
    const bool aimg = g.A_img && g.A_img[pr];
    const uint32_t slab = 2u * Bm;
    const uint32_t nslab = aimg ? nA / slab : 0u;
    const uint32_t first = aimg && nslab <= LA ? LA - nslab : 0u;
    if (aimg) {
        for (uint32_t l = first + tid; l < LA; l += kLBig) hist[l] = slab;
        if (tid == 0 && (nslab > LA || nslab * slab != nA || !d.direct)) flag = 1;
    }
    // four edges per thread and round, loads first; the first kListRegRounds rounds keep each edge's
    // layer and cell in registers for the scatter pass (layer < 2^15, cell < 2^11), later rounds
    // load their metas again
    uint32_t pk[kListRegRounds][4];
    auto hist_round = [&](uint32_t i0, uint32_t (&pr)[4]) {
        uint64_t m[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = i0 + (uint32_t)u * kLBig;
            m[u] = i < nA ? g.A.meta[aeo + i] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            pr[u] = meta_layer(m[u]) | (meta_ch(m[u]) * Bm + meta_idx(m[u])) << 15;
            if (i0 + (uint32_t)u * kLBig >= nA) continue;
            const uint32_t la = meta_layer(m[u]);
            if (la >= LA || meta_idx(m[u]) >= Bm || meta_ch(m[u]) > 1) flag = 1;
            else atomicAdd(&hist[la], 1u);
        }
    };
    if (!aimg) {
#pragma unroll
        for (uint32_t r = 0; r < kListRegRounds; ++r)
            if (tid + r * 4u * kLBig < nA) hist_round(tid + r * 4u * kLBig, pk[r]);
        for (uint32_t i0 = tid + kListRegRounds * 4u * kLBig; i0 < nA; i0 += 4u * kLBig) {
            uint32_t pr[4];
            hist_round(i0, pr);
        }
    }
    for (uint32_t j = tid; j < nB; j += kLBig) {
        const uint64_t m = g.B.meta[beo + j];
        const uint32_t lb = meta_layer(m);
        if (lb >= LB || meta_idx(m) >= Bm || meta_ch(m) > 1) flag = 1;
        else atomicAdd(&hist[LA + lb], 1u);
    }
    __syncthreads();
    if (flag) {   // invalid references: reject the pair (reference behaviour is UB)
        if (tid == 0) {
            cnt[2] = 1;
            g.pair_status[pr] = 2;
            g.C.l_cnt[pr] = 0;
            g.C.e_cnt[pr] = 0;
        }
        return;
    }
    // layer ranges by atomic allocation; non-empty layer lists by atomic append
    for (uint32_t l = tid; l < LA + LB; l += kLBig) {
        const uint32_t c = hist[l];
        if (d.iblk && l >= LA && c > kIblkMaxSparse) cnt[kCntIFail] = 1;   // its tasks would be deferred
        const bool a = l < LA;
        uint32_t* lst = a ? S + d.o_lstA : S + d.o_lstB;
        const uint32_t ll = a ? l : l - LA;
        const uint32_t L = a ? LA : LB;
        uint32_t start = 0;
        if (c) {
            start = atomicAdd(&cnt[a ? 5 : 6], c);
            if (aimg && a) start = (ll - first) * slab;   // the layer's slab
            const uint32_t k = atomicAdd(&cnt[a ? 0 : 1], 1u);
            (S + (a ? d.o_neA : d.o_neB))[k] = ll;
        }
        lst[ll] = start;
        lst[L + ll] = c;
        hist[l] = start;   // cursor
    }
    __syncthreads();
    uint32_t* idsA = S + d.o_lstA + 2 * LA;
    uint32_t* idsB = S + d.o_lstB + 2 * LB;
    if (d.direct) {   // k_large_count_la stores the count bytes of the A edges whose ranges hold keys only
        uint4* z = (uint4*)(S + d.o_icnt);
        for (uint32_t i = tid; i < 2u * ((nA + 31u) >> 5); i += kLBig) z[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    // direct pairs: an A id carries its dense cell, i | (ch B + idx) << 21 (the host checked
    // |A.E| < 2^21, B <= 1024), so their passes need no per-edge meta gather
    const uint32_t dsh = d.direct ? 21u : 32u;
    auto scatter_round = [&](uint32_t i0, const uint32_t (&pr)[4]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = i0 + (uint32_t)u * kLBig;
            if (i >= nA) break;
            const uint64_t cell = pr[u] >> 15;
            idsA[atomicAdd(&hist[pr[u] & 0x7FFFu], 1u)] = i | (uint32_t)((cell << dsh) & 0xFFFFFFFFull);
        }
    };
    if (!aimg) {   // (an image's ids sit in its meta region: the direct kernels read them there)
#pragma unroll
        for (uint32_t r = 0; r < kListRegRounds; ++r)
            if (tid + r * 4u * kLBig < nA) scatter_round(tid + r * 4u * kLBig, pk[r]);
    }
    for (uint32_t i0 = tid + kListRegRounds * 4u * kLBig; i0 < nA && !aimg; i0 += 4u * kLBig) {
        uint64_t m[4];
        uint32_t pr[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = i0 + (uint32_t)u * kLBig;
            m[u] = i < nA ? g.A.meta[aeo + i] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) pr[u] = meta_layer(m[u]) | (meta_ch(m[u]) * Bm + meta_idx(m[u])) << 15;
        scatter_round(i0, pr);
    }
    for (uint32_t j = tid; j < nB; j += kLBig) {
        const uint32_t lb = meta_layer(g.B.meta[beo + j]);
        idsB[atomicAdd(&hist[LA + lb], 1u)] = j;
    }
}

// one edge of a layer: its words and its index in the pair's edge array (first-insert times use it)
struct edge_rec {
    uint64_t meta, lo, hi;
    uint32_t e;
};
// the edges of one layer of one side of a pair, gathered through the layer's id list (layer-grouped
// 32-byte records written by k_large_lists were measured: the scattered record writes cost lists
// more than the products kernel saved)
struct layer_src {
    const pvac_ct_batch* X;
    uint64_t eo;          // the pair's edge offset in X
    const uint32_t* ids;
    uint32_t n;
};
__device__ __forceinline__ edge_rec load_edge(const layer_src& L, uint32_t k) {
    const uint32_t e = L.ids[k];
    return edge_rec{L.X->meta[L.eo + e], L.X->w_lo[L.eo + e], L.X->w_hi[L.eo + e], e};
}
__device__ __forceinline__ layer_src side_layer(const pvac_ct_batch* X, uint64_t eo, const uint32_t* S, uint64_t o_lst, uint32_t L,
                                                uint32_t l) {
    return layer_src{X, eo, S + o_lst + 2u * L + S[o_lst + l], S[o_lst + L + l]};
}

// ---------------------------------------------------------------- products (one task per WG)
constexpr int kLP = 384;                 // products workgroup: one lane per output index r (B = 337)
constexpr int kLPX = 256;                // products workgroup with the matrix-core dense mode (4 waves)
constexpr int kLPRows = 3;               // B <= kLP * kLPRows
constexpr uint32_t kBmax = kLP * kLPRows;
constexpr uint32_t kChunk = 128;         // sparse-side edges staged per round (chain steps: ~20)
// one product per sparse edge goes into each lane's P and M column sets between col26_norm calls
static_assert(kChunk <= kCol26MaxProducts, "col26 columns overflow: normalise more often");

__host__ __device__ inline uint32_t al16(uint32_t x) { return (x + 15u) & ~15u; }
// dense mode: dl4[2][2B] (limbs 0-3, 16 B) | dx[2][2B] (limb 4, first-insert share) | sl4[kChunk]
//             (16 B) | sl1[kChunk] | sinf[kChunk] | sid[kChunk] | dup. Per channel the B dense slots
//             are stored twice (x and x + B), so lane r finds slot (r - sidx) mod B at r + B - sidx:
//             no wrap test, and the sparse edge's part of the address is wave-uniform (SALU)
constexpr uint32_t kDenseFixed = 96u, kDenseChunk = 28u;
// scatter   : acc[2B x 3] (u64) | tk[B]
__host__ __device__ inline uint32_t prod_lds_bytes(uint32_t Bm) {
    const uint32_t dense = al16(kDenseFixed * Bm) + kDenseChunk * kChunk + 16u;
    const uint32_t scat = 48u * Bm + 4u * Bm;
    return dense > scat ? dense : scat;
}

// ---- dense mode on the matrix cores (gfx950 v_mfma_i32_32x32x32_i8) --------------------------
// An Fp value v (canonical) is taken as the signed integer V = v (v < 2^126) or v - p, written
// with 16 balanced base-256 digits d_i in [-128, 127] (int8). For output index r of a task,
//     sum_e D[r - idx_e] * w_e  =  sum_m 256^m  sum_e sum_j W_e[m][j] D[r - idx_e][j],
// W_e[m][j] = digit (m - j) of w_e (zero outside 0..15): a 32 x 32 (digit position m) x (row r)
// tile over K = 2 sparse edges x 16 digits is ONE v_mfma_i32_32x32x32_i8. Column sums stay
// below 2^23 (<= 20 edges x 16 digit pairs x 2^14), so nothing overflows before the epilogue
// turns the 31 digit positions of a row into Fp (mx_fold). Operand maps (tools/mfma_i8_probe.hip):
// A lane l = (m = l & 31, half h = l >> 5) byte j  x  B lane (r = l & 31, h) byte j, for the same
// (h, j); D lane l register i = position (i & 3) + 8 (i >> 2) + 4 h of row l & 31.
typedef int mx_v4 __attribute__((ext_vector_type(4)));
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef int mx_v16 __attribute__((ext_vector_type(16)));
constexpr int kMxKS = 10;                          // k-steps held in registers: 2 sparse edges each
constexpr uint32_t kMxMaxSparse = 2u * kMxKS;      // sparse sides up to this size take the MFMA path
static_assert(kMxMaxSparse == kIblkMaxSparse, "iblk pairs need every B layer on the matrix cores");
constexpr uint64_t kDigC = 0x8080808080808080ull;  // 128 in every byte
#ifdef PVAC_ASM_MARKS   // ISA census builds only (tools/asm_phases.py)
#define MXMARK(ph) asm volatile("; PVAC_MARK " #ph ::: "memory")
#else
#define MXMARK(ph) do {} while (0)
#endif
#ifndef PVAC_EXP_IBREP   // experiment builds only: the per-A-edge passes run this many times (same result)
#define PVAC_EXP_IBREP 1
#endif
#ifndef PVAC_EXP_MXREP   // experiment builds only: the MFMA loop run this many times (same result)
#define PVAC_EXP_MXREP 1
#endif

// a loaded value kept in a VGPR until here: a uniform load is otherwise moved to an SGPR right
// after it is issued, and that readfirstlane waits for every load in flight
__device__ __forceinline__ uint32_t late(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}

// t = i D + j for D <= 63: m = floor(2^32 / D), i = (t m) >> 32 is i or i - 1
__device__ __forceinline__ uint32_t div_small(uint32_t t, uint32_t D, uint64_t m, uint32_t& j) {
    uint32_t i = (uint32_t)(((uint64_t)t * m) >> 32);
    uint32_t r = t - i * D;
    if (r >= D) {
        ++i;
        r -= D;
    }
    j = r;
    return i;
}

// balanced digits of a canonical value: U = V + C (C = 128 in each of the 16 bytes), d = U ^ C
__device__ __forceinline__ void fp_digits8(const fp& v, uint64_t& dl, uint64_t& dh) {
    const bool neg = (v.hi >> 62) != 0;            // v >= 2^126: V = v - p = v + 2^127 + 1 (mod 2^128)
    const uint64_t l = v.lo + (neg ? 1ull : 0ull);
    const uint64_t h = v.hi + (neg ? 0x8000000000000000ull + (l < v.lo ? 1ull : 0ull) : 0ull);
    const uint64_t ul = l + kDigC;
    const uint64_t uh = h + kDigC + (ul < l ? 1ull : 0ull);
    dl = ul ^ kDigC;
    dh = uh ^ kDigC;
}

// A lane's 16 column sums c[i] sit at digit positions k(i) = (i & 3) + 8 (i >> 2) + 4 h, and
// k(i + 8) = k(i) + 16: 256^16 = 2^128 == 2 (mod p), so d[i] = c[i] + 2 c[i + 8] (32-bit, |d| < 2^24
// for <= 20 sparse edges) leaves positions 4h..4h+3 (d[0..3]) and 8+4h..11+4h (d[4..7]), i.e. the
// 32-bit words h and 2 + h of the row's value: ga, gb (|g| < 2^48.1).
// acc + (int64) x * m in one v_mad_i64_i32 (sign extension, shift and 64-bit add: the compiler's
// form of a power-of-two multiple is a sign-extending shift plus a 64-bit shift-add per term)
#ifndef PVAC_MX_MAD
#define PVAC_MX_MAD 1
#endif
__device__ __forceinline__ int64_t mad_i64_i32(int32_t x, uint32_t m, int64_t acc) {
#if PVAC_MX_MAD
    int64_t r;
    asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"(x), "s"(m), "v"(acc) : "vcc");
    return r;
#else
    return acc + (int64_t)x * (int64_t)m;
#endif
}
__device__ __forceinline__ void mx_groups(const mx_v16& c, int64_t& ga, int64_t& gb) {
    int32_t d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = c[i] + 2 * c[i + 8];
    ga = mad_i64_i32(d[3], 16777216u, mad_i64_i32(d[2], 65536u, mad_i64_i32(d[1], 256u, (int64_t)d[0])));
    gb = mad_i64_i32(d[7], 16777216u, mad_i64_i32(d[6], 65536u, mad_i64_i32(d[5], 256u, (int64_t)d[4])));
}

// Z = H0 + H1 2^32 + H2 2^64 + H3 2^96 mod p (|H| < 2^56), canonical. 2^128 == 2, 2^127 == 1 (mod p).
__device__ __forceinline__ fp mx_fold(int64_t a0, int64_t a1, int64_t b0, int64_t b1) {
    // 32-bit words W0..W4 of Z; W4 2^128 == 2 W4 goes into W0
    int64_t t = (int64_t)(uint32_t)a0 + 2 * (b1 >> 32);
    const uint32_t x0 = (uint32_t)t;
    t = (t >> 32) + (a0 >> 32) + (int64_t)(uint32_t)a1;
    const uint32_t x1 = (uint32_t)t;
    t = (t >> 32) + (a1 >> 32) + (int64_t)(uint32_t)b0;
    const uint32_t x2 = (uint32_t)t;
    t = (t >> 32) + (b0 >> 32) + (int64_t)(uint32_t)b1;
    const uint32_t x3 = (uint32_t)t;
    const int64_t k = t >> 32;                     // Z == X + 2 k, X = x3..x0 in [0, 2^128), |k| <= 1
    uint64_t lo = (uint64_t)x0 | (uint64_t)x1 << 32, hi = (uint64_t)x2 | (uint64_t)x3 << 32;
    const int64_t s = (int64_t)(hi >> 63) + 2 * k; // X = Xl + 2^127 Xh
    hi &= kM63;
    // Xl + s, or Xl + (p + s) when s < 0: stays in [0, 2^128)
    const uint64_t alo = s < 0 ? kAll - (uint64_t)(-s) : (uint64_t)s;
    const uint64_t ahi = s < 0 ? kM63 : 0ull;
    lo += alo;
    hi += ahi + (lo < alo ? 1ull : 0ull);
    return fp_from_words(lo, hi);
}

__device__ __forceinline__ int64_t shfl_xor64(int64_t v, int mask) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, mask);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)((uint64_t)v >> 32), mask);
    return (int64_t)((uint64_t)hi << 32 | lo);
}

// LDS of the MFMA dense mode: dig[2][2B] (16 B of digits per dense slot, stored twice per channel
// like the column mode's tables) | tt[2][2B] (the dense side's share of the first-insert time) |
// dup; then, per sparse side, prec[kMxMaxSparse][3] (48 B per sparse edge: 16 zero bytes, its
// digits reversed, 16 zero bytes: W_e's row m is the 16-byte window at 31 - m) and
// pinf[kMxMaxSparse] (uint4: P and M slot offsets relative to row r, the sparse side's share of t)
__host__ __device__ inline uint32_t mx_lds_bytes(uint32_t Bm) { return al16(80u * Bm + 4u); }
// k_large_count_la (no digit tables): M1 / M2 [0, 32 B) | tt [32 B, 48 B) | dup | list length, then
// the B layers' staging at cnt_lds_bytes (6 workgroups per CU where mx_lds_bytes allowed 4)
constexpr uint32_t kCntTtOff = 32u;
__host__ __device__ inline uint32_t cnt_lds_bytes(uint32_t Bm) { return al16((kCntTtOff + 16u) * Bm + 8u); }
constexpr uint32_t kMxSparseBytes = 64u * kMxMaxSparse;
constexpr uint32_t kIblkBjtBytes = 4u * 64u;       // k_large_products_la: B edge table of iblk pairs

// the dense side of a task into dig / tt. Every thread calls it; barriers inside; false
// (workgroup-uniform) when the layer holds duplicate (idx, ch) edges
template <int BS>
__device__ bool mx_stage_dense(uint8_t* lds, uint32_t Bm, const layer_src& D, uint32_t tmul) {
    uint4* dig = (uint4*)lds;
    uint32_t* tt = (uint32_t*)(lds + 64u * Bm);
    uint32_t* dup = (uint32_t*)(lds + 80u * Bm);
    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < 4 * Bm; k += BS) {
        dig[k] = make_uint4(0, 0, 0, 0);
        tt[k] = kInf;
    }
    if (tid == 0) *dup = 0;
    __syncthreads();
    for (uint32_t k0 = tid; k0 < D.n; k0 += 2u * BS) {   // two edges per round, loads first
        edge_rec x[2];
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const uint32_t k = k0 + (uint32_t)v * BS;
            x[v] = load_edge(D, k < D.n ? k : 0u);
        }
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            if (k0 + (uint32_t)v * BS >= D.n) break;
            const uint32_t sl = meta_ch(x[v].meta) * 2u * Bm + meta_idx(x[v].meta);
            const uint32_t te = x[v].e * tmul;   // the dense side's share of t = i |B.E| + j
            if (atomicCAS(&tt[sl], kInf, te) != kInf) {
                *dup = 1;
            } else {
                uint64_t dl, dh;
                fp_digits8(fp_canon(x[v].lo, x[v].hi), dl, dh);
                dig[sl] = dig[sl + Bm] = make_uint4((uint32_t)dl, (uint32_t)(dl >> 32), (uint32_t)dh, (uint32_t)(dh >> 32));
                tt[sl + Bm] = te;
            }
        }
    }
    __syncthreads();
    return *dup == 0;
}

// the sparse side of a task (n <= kMxMaxSparse edges) into prec / pinf; thread k writes edge k
// (an odd count gets a zero padding edge). No barrier.
__device__ __forceinline__ void mx_stage_sparse(uint4* prec, uint4* pinf, uint32_t Bm, const layer_src& Sd, uint32_t smul,
                                                uint32_t k) {
    const uint32_t nks = (Sd.n + 1u) >> 1;
    if (k >= 2u * nks) return;
    uint4 mid = make_uint4(0, 0, 0, 0);
    uint4 inf = make_uint4(Bm, Bm, kInf, 0);   // padding edge: zero digits, time never smaller, w = 0
    if (k < Sd.n) {
        const edge_rec x = load_edge(Sd, k);
        uint64_t dl, dh;
        fp_digits8(fp_canon(x.lo, x.hi), dl, dh);
        const uint64_t rl = __builtin_bswap64(dh), rh = __builtin_bswap64(dl);   // digit 15 - x at byte x
        mid = make_uint4((uint32_t)rl, (uint32_t)(rl >> 32), (uint32_t)rh, (uint32_t)(rh >> 32));
        const uint32_t sidx = meta_idx(x.meta), sch = meta_ch(x.meta);
        // dense slot of output row r: P (dense channel == sparse channel), M (the other)
        inf = make_uint4(sch * 2u * Bm + Bm - sidx, (sch ^ 1u) * 2u * Bm + Bm - sidx, x.e * smul, 0);
    }
    prec[3u * k] = make_uint4(0, 0, 0, 0);
    prec[3u * k + 1u] = mid;
    prec[3u * k + 2u] = make_uint4(0, 0, 0, 0);
    pinf[k] = inf;
}

// where a task's results go: dense key-slot arrays of the pair
struct task_out {
    uint32_t* tkey;
    uint32_t* info;
    ulonglong2* sums;
    const uint32_t* ghead;              // static bucket groups (nullptr: dynamic chains)
    unsigned long long* bpack;          // bucket-leader block marks
    // iblk (k_large_products_la): per output row of this B layer, the key's record for iblk_layer:
    // dense slot of its A edge | j << 12 | edge bits << 18 | shared << 20 | 1 << 21 (0: no key)
    uint32_t* recs = nullptr;
    const uint32_t* bjt = nullptr;      // B edge j: idx | ch << 16
    uint32_t nB = 0;
    uint64_t nb_m = 0;
};
constexpr uint32_t kRecKey = 1u << 21, kRecShared = 1u << 20;

// the products of one staged task on the matrix cores: each wave takes blocks of 32 output rows
// (both channels), writes tkey / info / sums and marks lone bucket leaders. No barrier; returns
// whether any of this thread's keys emits.
// NKS = k-steps of two sparse edges, a compile-time count: the k-step loop is straight-line code,
// so every k-step's LDS reads can be issued ahead of the MFMAs (a runtime guard per k-step made
// each one a basic block of its own: two dependent LDS round trips per k-step)
template <int BS, int NKS>
__device__ bool mx_blocks_n(const uint8_t* lds, const uint4* prec, const uint4* pinf, uint32_t Bm, uint64_t slot0,
                            const task_out& o) {
    const uint4* dig = (const uint4*)lds;
    const uint32_t* tt = (const uint32_t*)(lds + 64u * Bm);
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t h = lane >> 5, n = lane & 31u;
    bool any = false;
    // A operand of k-step s: row m = n of W_e, e = 2 s + h: 16 bytes at 31 - n of prec[e]
    mx_v4 frag[NKS];
    {
        const uint32_t y0 = 31u - n, sh = y0 & 3u;
        const uint32_t* pw = (const uint32_t*)prec + (y0 >> 2) + 12u * h;
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
            const uint32_t* q = pw + 24u * (uint32_t)s;
            const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
            frag[s] = mx_v4{(int)__builtin_amdgcn_alignbyte(w1, w0, sh), (int)__builtin_amdgcn_alignbyte(w2, w1, sh),
                            (int)__builtin_amdgcn_alignbyte(w3, w2, sh), (int)__builtin_amdgcn_alignbyte(w4, w3, sh)};
        }
    }
    const uint32_t nblk = (Bm + 31u) >> 5;
    MXMARK(1);
    for (uint32_t blk = wave; blk < nblk; blk += BS / 64) {
        MXMARK(2);
        const uint32_t r = blk * 32u + n;
        const bool live = r < Bm;
        const uint32_t rr = live ? r : 0u;
        mx_v16 aP{}, aM{};
        uint32_t tmin = kInf;
        for (int rep_ = 0; rep_ < PVAC_EXP_MXREP; ++rep_) {   // experiment builds repeat the loop
            uint32_t rq = rr;
            asm volatile("" : "+v"(rq));
            if (rep_) {   // keep the previous repetition live: add x - y where x == y at run time
                int zp = aP[0], zm = aM[0];
                asm volatile("" : "+v"(zp), "+v"(zm));
                tmin += (uint32_t)(zp - aP[0]) + (uint32_t)(zm - aM[0]);
            }
            aP = mx_v16{};
            aM = mx_v16{};
            tmin = min(tmin, kInf);
#pragma unroll
            for (int s = 0; s < NKS; ++s) {
                const uint4 in = pinf[2u * (uint32_t)s + h];
                const uint4 dp = dig[in.x + rq], dm = dig[in.y + rq];
                const uint32_t tp = tt[in.x + rq], tm = tt[in.y + rq];
                aP = __builtin_amdgcn_mfma_i32_32x32x32_i8(frag[s], mx_v4{(int)dp.x, (int)dp.y, (int)dp.z, (int)dp.w}, aP, 0, 0, 0);
                aM = __builtin_amdgcn_mfma_i32_32x32x32_i8(frag[s], mx_v4{(int)dm.x, (int)dm.y, (int)dm.z, (int)dm.w}, aM, 0, 0, 0);
                tmin = min(tmin, min(__builtin_elementwise_add_sat(tp, in.z), __builtin_elementwise_add_sat(tm, in.z)));
            }
        }
        MXMARK(3);
        // half 0 folds row r's P sum, half 1 its M sum; each needs the other half's two words
        int64_t paw, pbw, maw, mbw;
        mx_groups(aP, paw, pbw);
        mx_groups(aM, maw, mbw);
        const int64_t ra = shfl_xor64(h ? paw : maw, 32), rb = shfl_xor64(h ? pbw : mbw, 32);
        MXMARK(4);
        const fp v = mx_fold(h ? ra : paw, h ? maw : ra, h ? rb : pbw, h ? mbw : rb);
        MXMARK(5);
        const uint32_t nz = fp_nonzero(v) ? 1u : 0u;
        const uint32_t nzo = (uint32_t)__shfl_xor((int)nz, 32);
        const uint32_t eb = h ? (nzo | nz << 1) : (nz | nzo << 1);
        tmin = min(tmin, (uint32_t)__shfl_xor((int)tmin, 32));
        if (live) {
            const uint64_t s = slot0 + r;
            if (h == 0) o.tkey[s] = tmin;
            if (tmin != kInf) {
                o.sums[2 * s + h] = make_ulonglong2(v.lo, v.hi);
                if (h == 0) {
                    o.info[s] = eb;
                    if (eb && o.bpack && o.ghead && o.ghead[s] == 0u) leader_mark(o.bpack, tmin, __popc(eb));
                }
                any |= eb != 0;
            }
            if (o.recs && h == 0) {   // iblk: the key's A edge (dense slot) and B edge j
                uint32_t rv = 0;
                const bool shared = tmin != kInf && o.ghead && o.ghead[s] != 0u;
                if (tmin != kInf && (eb || shared)) {
                    uint32_t j;
                    const uint32_t i = div_small(tmin, o.nB, o.nb_m, j);
                    const uint32_t ij = o.bjt[j] & 0xFFFFu;
                    const uint32_t x = r >= ij ? r - ij : r + Bm - ij;
                    const uint32_t dd = tt[x] == i * o.nB ? x : Bm + x;
                    rv = dd | j << 12 | eb << 18 | (shared ? kRecShared : 0u) | kRecKey;
                }
                o.recs[r] = rv;
            }
        }
    }
    return any;
}

template <int BS>
__device__ bool mx_blocks(const uint8_t* lds, const uint4* prec, const uint4* pinf, uint32_t ns, uint32_t Bm, uint64_t slot0,
                          const task_out& o) {
    static_assert(kMxKS == 10, "one instantiation per k-step count");
    switch ((ns + 1u) >> 1) {   // workgroup-uniform
    case 0: return false;       // no products: the slots keep their initial time
    case 1: return mx_blocks_n<BS, 1>(lds, prec, pinf, Bm, slot0, o);
    case 2: return mx_blocks_n<BS, 2>(lds, prec, pinf, Bm, slot0, o);
    case 3: return mx_blocks_n<BS, 3>(lds, prec, pinf, Bm, slot0, o);
    case 4: return mx_blocks_n<BS, 4>(lds, prec, pinf, Bm, slot0, o);
    case 5: return mx_blocks_n<BS, 5>(lds, prec, pinf, Bm, slot0, o);
    case 6: return mx_blocks_n<BS, 6>(lds, prec, pinf, Bm, slot0, o);
    case 7: return mx_blocks_n<BS, 7>(lds, prec, pinf, Bm, slot0, o);
    case 8: return mx_blocks_n<BS, 8>(lds, prec, pinf, Bm, slot0, o);
    case 9: return mx_blocks_n<BS, 9>(lds, prec, pinf, Bm, slot0, o);
    default: return mx_blocks_n<BS, 10>(lds, prec, pinf, Bm, slot0, o);
    }
}

// One (la, lb) task: the matrix-core dense mode when MX and the sparse side is small, else the
// column-accumulator dense mode (when col26_ok), else (sparse x sparse, duplicate edges) the
// scatter mode. Every thread of the workgroup calls it (barriers inside); LDS from plds,
// prod_lds_bytes(B) (col26 / scatter) or al16(mx_lds_bytes(B)) + kMxSparseBytes (MX), 52 B (scatter).
template <int BS, bool MX>
__device__ void run_task(const mul_large_args& g, const large_desc& d, uint32_t la, uint32_t lb, uint8_t* plds,
                         bool col26_ok = true) {
    uint32_t* S = g.scratch;
    const uint32_t LA = d.LA, LB = d.LB, Bm = g.Bm, nB = d.nB;
    const layer_src srcA = side_layer(&g.A, g.A.e_off[d.pair], S, d.o_lstA, LA, la);
    const layer_src srcB = side_layer(&g.B, g.B.e_off[d.pair], S, d.o_lstB, LB, lb);
    const uint32_t na = srcA.n, nb = srcB.n;
    const uint32_t lp = la * LB + lb;
    const uint64_t slot0 = (uint64_t)lp * Bm;
    const int tid = threadIdx.x;
    const bool denseA = na >= nb;
    const uint32_t nd = denseA ? na : nb, ns = denseA ? nb : na;
    const layer_src& Dn = denseA ? srcA : srcB;
    const layer_src& Sp = denseA ? srcB : srcA;
    const uint32_t tmulD = denseA ? nB : 1u, tmulS = denseA ? 1u : nB;   // shares of t = i |B.E| + j
    uint32_t* tkey = S + d.o_tkey;
    uint32_t* info = S + d.o_info;
    ulonglong2* sums = (ulonglong2*)(S + d.o_sums);
    // keys alone in their bucket are their own bucket leaders: mark them here, where the atomic
    // overlaps the multiply-bound loop of other waves, and `rank` skips them
    const uint32_t* ghead = group_heads(g, d);
    // iblk pairs: no block marks here (k_large_products_la counts per A edge; a pair that falls back
    // has its lone leaders marked by k_large_rank)
    unsigned long long* bpack = d.iblk ? nullptr : (unsigned long long*)w64(S, d.o_bmask);
    bool any = false;

    bool dense = col26_ok && nd >= kLargeDenseMin;
    if (MX && dense && ns <= kMxMaxSparse) {
        uint4* prec = (uint4*)(plds + mx_lds_bytes(Bm));
        uint4* pinf = prec + 3u * kMxMaxSparse;
        mx_stage_sparse(prec, pinf, Bm, Sp, tmulS, (uint32_t)tid);   // made visible by the dense staging's barriers
        dense = mx_stage_dense<BS>(plds, Bm, Dn, tmulD);
        if (dense) any = mx_blocks<BS>(plds, prec, pinf, ns, Bm, slot0, task_out{tkey, info, sums, ghead, bpack});
        __syncthreads();
    } else if (dense) {
        // Dense-owner mode with column accumulators (fp127.hpp col26_*): both sides are staged as
        // 26-bit limbs, each probe is 25 v_mad_u64_u32 into the lane's P or M columns and a
        // saturating add + min for the first-insert time. Empty dense slots hold zero limbs and
        // time kInf, so the loop has no branch: a miss adds 0 and leaves the time alone.
        uint4* dl4 = (uint4*)plds;
        uint2* dx = (uint2*)(plds + 64u * Bm);
        uint4* sl4 = (uint4*)(plds + al16(kDenseFixed * Bm));
        uint32_t* sl1 = (uint32_t*)(sl4 + kChunk);
        uint32_t* sinf = sl1 + kChunk;
        uint32_t* sidv = sinf + kChunk;
        uint32_t* dup = sidv + kChunk;
        // the first sparse chunk's loads go out before the dense staging, so the two sides' global
        // round trips overlap (thread k < kChunk < BS stages sparse edge k)
        edge_rec pr0{0, 0, 0, 0};
        if ((uint32_t)tid < min(ns, kChunk)) pr0 = load_edge(Sp, tid);
        for (uint32_t k = tid; k < 4 * Bm; k += BS) {
            dl4[k] = make_uint4(0, 0, 0, 0);
            dx[k] = make_uint2(0, kInf);
        }
        if (tid == 0) *dup = 0;
        __syncthreads();
        for (uint32_t k0 = tid; k0 < nd; k0 += 2u * BS) {   // two edges per round, loads first
            edge_rec x[2];
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                const uint32_t k = k0 + (uint32_t)v * BS;
                x[v] = load_edge(Dn, k < nd ? k : 0u);
            }
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                if (k0 + (uint32_t)v * BS >= nd) break;
                const uint32_t sl = meta_ch(x[v].meta) * 2u * Bm + meta_idx(x[v].meta);
                // dx.y holds the dense side's share of the first-insert time t = i |B.E| + j
                const uint32_t te = x[v].e * tmulD;
                if (atomicCAS(&dx[sl].y, kInf, te) != kInf) {
                    *dup = 1;
                } else {   // canonical operands: the limb split needs a, b < 2^127
                    uint32_t l[5];
                    fp_split26(fp_canon(x[v].lo, x[v].hi), l);
                    dl4[sl] = dl4[sl + Bm] = make_uint4(l[0], l[1], l[2], l[3]);
                    dx[sl].x = l[4];
                    dx[sl + Bm] = make_uint2(l[4], te);
                }
            }
        }
        __syncthreads();
        dense = *dup == 0;   // duplicate (layer, idx, ch) edges: use the scatter mode instead
        if (dense) {
            const uint32_t rows = (Bm + BS - 1) / BS;   // workgroup-uniform (1 for B <= BS)
            for (uint32_t u = 0; u < rows; ++u) {
                const uint32_t r = tid + u * BS;
                const bool live = r < Bm;
                const uint4* dl4r = dl4 + (live ? r : 0u);
                const uint2* dxr = dx + (live ? r : 0u);
                uint64_t P[9], M[9];
                col26_zero(P);
                col26_zero(M);
                uint32_t tmin = kInf;
                for (uint32_t c0 = 0; c0 < ns; c0 += kChunk) {
                    const uint32_t cn = min(kChunk, ns - c0);
                    __syncthreads();
                    if ((uint32_t)tid < cn) {
                        const uint32_t k = (uint32_t)tid;
                        const bool first = u == 0 && c0 == 0;   // prefetched above
                        const edge_rec x = first ? pr0 : load_edge(Sp, c0 + k);
                        uint32_t l[5];
                        fp_split26(fp_canon(x.lo, x.hi), l);
                        sl4[k] = make_uint4(l[0], l[1], l[2], l[3]);
                        sl1[k] = l[4];
                        // wave-uniform offsets of the P and M slots relative to lane r: the dense
                        // channel equal to the sparse one gives P, the other M
                        const uint32_t sidx = meta_idx(x.meta), sch = meta_ch(x.meta);
                        sinf[k] = (sch * 2u * Bm + Bm - sidx) | (((sch ^ 1u) * 2u * Bm + Bm - sidx) << 16);
                        sidv[k] = x.e * tmulS;   // the sparse side's share of t
                    }
                    __syncthreads();
                    if (live) {
                        for (uint32_t q = 0; q < cn; ++q) {
                            const uint32_t so = __builtin_amdgcn_readfirstlane(sinf[q]);
                            const uint32_t oP = so & 0xFFFFu, oM = so >> 16;
                            const uint4 b4 = sl4[q];
                            const uint32_t b[5] = {b4.x, b4.y, b4.z, b4.w, sl1[q]};
                            const uint32_t se = sidv[q];
                            const uint4 p4 = dl4r[oP], m4 = dl4r[oM];
                            const uint2 px = dxr[oP], mx = dxr[oM];
                            const uint32_t ap[5] = {p4.x, p4.y, p4.z, p4.w, px.x};
                            const uint32_t am[5] = {m4.x, m4.y, m4.z, m4.w, mx.x};
                            col26_mac(P, ap, b);
                            col26_mac(M, am, b);
                            tmin = min(tmin, min(__builtin_elementwise_add_sat(px.y, se),
                                                 __builtin_elementwise_add_sat(mx.y, se)));
                        }
                        col26_norm(P);
                        col26_norm(M);
                    }
                }
                if (live) {
                    const uint64_t s = slot0 + r;
                    tkey[s] = tmin;
                    if (tmin != kInf) {
                        const fp ps = col26_fold(P), ms = col26_fold(M);
                        const uint32_t eb = (fp_nonzero(ps) ? 1u : 0u) | (fp_nonzero(ms) ? 2u : 0u);
                        info[s] = eb;
                        sums[2 * s] = make_ulonglong2(ps.lo, ps.hi);
                        sums[2 * s + 1] = make_ulonglong2(ms.lo, ms.hi);
                        any |= eb != 0;
                        if (eb && bpack && ghead && ghead[s] == 0u) leader_mark(bpack, tmin, __popc(eb));
                    }
                }
            }
        }
        __syncthreads();
    }
    if (!dense) {
        unsigned long long* acc = (unsigned long long*)plds;
        uint32_t* tk = (uint32_t*)(plds + 48u * Bm);
        for (uint32_t k = tid; k < 6 * Bm; k += BS) acc[k] = 0ull;
        for (uint32_t k = tid; k < Bm; k += BS) tk[k] = kInf;
        __syncthreads();
        const uint64_t np = (uint64_t)na * nb;
        for (uint64_t t = tid; t < np; t += BS) {
            const uint32_t ai = (uint32_t)(t / nb), bj = (uint32_t)(t - (uint64_t)ai * nb);
            const edge_rec xa = load_edge(srcA, ai), xb = load_edge(srcB, bj);
            const uint32_t r = mod_small(meta_idx(xa.meta) + meta_idx(xb.meta), Bm);
            const uint32_t chn = meta_ch(xa.meta) ^ meta_ch(xb.meta);
            const fp pv = fp_mul(fp{xa.lo, xa.hi}, fp{xb.lo, xb.hi});
            uint64_t l0, l1, l2;
            fp_split3(pv, l0, l1, l2);
            unsigned long long* q = acc + (size_t)(r * 2 + chn) * 3;
            atomicAdd(q + 0, (unsigned long long)l0);
            atomicAdd(q + 1, (unsigned long long)l1);
            atomicAdd(q + 2, (unsigned long long)l2);
            atomicMin(&tk[r], xa.e * nB + xb.e);
        }
        __syncthreads();
        for (uint32_t r = tid; r < Bm; r += BS) {
            const uint64_t s = slot0 + r;
            const uint32_t tkr = tk[r];
            tkey[s] = tkr;
            if (tkr != kInf) {
                const unsigned long long* q = acc + (size_t)r * 6;
                const fp p = fp_fold3(q[0], q[1], q[2]);
                const fp m = fp_fold3(q[3], q[4], q[5]);
                const uint32_t eb = (fp_nonzero(p) ? 1u : 0u) | (fp_nonzero(m) ? 2u : 0u);
                info[s] = eb;
                sums[2 * s] = make_ulonglong2(p.lo, p.hi);
                sums[2 * s + 1] = make_ulonglong2(m.lo, m.hi);
                any |= eb != 0;
                if (eb && bpack && ghead && ghead[s] == 0u) leader_mark(bpack, tkr, __popc(eb));
            }
        }
        __syncthreads();   // the caller may reuse the LDS
    }
    if (any) S[d.o_used + (LA + LB) + lp] = 1;   // benign race: every writer stores 1
}

// one workgroup per task (la, lb): pairs with many B layers (squares)
template <int BS, bool MX>
__global__ __launch_bounds__(BS) void k_large_products(mul_large_args g) {
    extern __shared__ __attribute__((aligned(16))) uint8_t plds[];
    const large_desc& d = g.desc[g.sel[g.n_la + blockIdx.y]];
    uint32_t* S = g.scratch;
    const uint32_t* cnt = S + d.o_cnt;
    if (cnt[2]) return;
    const uint32_t LB = d.LB;
    const uint32_t tl = blockIdx.x;
    const uint32_t la_i = tl / LB, lb_i = tl - la_i * LB;
    if (la_i >= cnt[0] || lb_i >= cnt[1]) return;
    run_task<BS, MX>(g, d, S[d.o_neA + la_i], S[d.o_neB + lb_i], plds);
}

// ---- per-A-edge emit order (iblk pairs) ---------------------------------------------------
// The reference emits keys in hash-list order: bucket first-insert time DESC, then key time DESC
// (see k_mul_fresh.hip). A first-insert time t = i |B.E| + j names A edge i and B edge j, and the
// key lies in product layer (layer(i), layer(j)): every key whose time falls in A edge i's range
// [i |B.E|, (i + 1) |B.E|) belongs to ONE A layer, which one k_large_products_la workgroup
// multiplies against every B layer. So that workgroup can count the edges of A edge i's keys and
// rank each key among them (by j DESC) in LDS; a suffix scan over the |A.E| counts then gives
// every key's position: offset(i) + rank. This replaces the n/16-word block marks (zeroed, marked
// with random 64-bit atomics, scanned and read back at random: k_large_init / products / scan /
// order) with |A.E| plain counts. Keys that share a libstdc++ bucket with another slot of the
// static group (a few percent) are emitted at their bucket leader's time: k_large_rank moves their
// edges from their own A edge's count to the leader's, and every A edge range holding such a key
// is flagged so that `order` ranks its keys by probing the range's |B.E| times instead.

// After the tasks of A layer la (all B layers) have left one record per key in recs (the MFMA
// epilogue: the dense slot d of the key's A edge, its B edge j, its edge bits): M1[d] / M2[d] = bit j
// for the keys whose first-insert time is (A edge at d, B edge j) and that emit a P / an M edge,
// bit 63 of M1 = a key of a shared bucket lies in the range (`order` probes it); then icnt[i] and,
// for ranges with keys, imask[i] = (M1, M2). M1 / M2 use the dense digit table's LDS (dead now), tt
// maps dense slot d back to its A edge. Barriers inside; every thread calls it.
template <int BS>
__device__ void iblk_layer(uint8_t* plds, const mul_large_args& g, const large_desc& d, uint32_t la, uint4 lbq,
                           uint32_t neB, const uint32_t* recs, uint32_t* icnt, ulonglong2* imask) {
    const uint32_t Bm = g.Bm, nB = d.nB;
    uint32_t* S = g.scratch;
    unsigned long long* M1 = (unsigned long long*)plds;
    unsigned long long* M2 = M1 + 2u * Bm;
    const uint32_t* tt = (const uint32_t*)(plds + 64u * Bm);
    const uint64_t m = d.nb_m;
    const uint32_t tid = threadIdx.x, nk = neB * Bm;
    for (uint32_t k = tid; k < 4u * Bm; k += BS) M1[k] = 0ull;
    __syncthreads();
    bool shared = false;
    for (uint32_t q = tid; q < nk; q += BS) {
        const uint32_t v = recs[q];
        if (!v) continue;
        const uint32_t dd = v & 0xFFFu, j = (v >> 12) & 63u, e = (v >> 18) & 3u;
        if (e & 1u) atomicOr(&M1[dd], 1ull << j);
        if (e & 2u) atomicOr(&M2[dd], 1ull << j);
        if (v & kRecShared) {   // with or without edges: it may lead its bucket
            atomicOr(&M1[dd], 1ull << 63);
            shared = true;
        }
    }
    if (shared) S[d.o_cnt + kCntIShared] = 1u;
    __syncthreads();
    for (uint32_t dd = tid; dd < 2u * Bm; dd += BS) {
        const uint32_t ch = dd >= Bm ? 1u : 0u;
        const uint32_t te = tt[dd + ch * Bm];   // tt slot ch 2B + idx
        if (te == kInf) continue;
        uint32_t j;
        const uint32_t i = div_small(te, nB, m, j);
        const unsigned long long x1 = M1[dd], x2 = M2[dd];
        icnt[i] = (uint32_t)__popcll(x1 & ~(1ull << 63)) + (uint32_t)__popcll(x2);
        // only ranges that hold keys are read back (write_ranges, order): most A edges of a deep
        // chain step hold none (their keys were all inserted by earlier A edges)
        if (x1 | x2) imask[i] = make_ulonglong2(x1, x2);
    }
    __syncthreads();   // the next A layer's staging overwrites M1 / M2, tt and recs
}

// ---- direct mode (large_desc::direct) ------------------------------------------------------
// k_large_count_la's per-A-layer output, held in registers so that its global stores can be issued
// after the next layer's staging has consumed its loads (a wave's vmcnt counts stores and loads in
// one FIFO: stores issued between a load and its use made that use wait for them)
constexpr uint32_t kPendCells = 3;   // dense cells per thread held (2 B <= 3 x 256 for B <= 384)
struct cnt_pend {
    uint32_t i[kPendCells], w[kPendCells], k[kPendCells];   // A edge, list word, list slot + 1 (0: none)
    ulonglong2 m[kPendCells];
    uint32_t n;        // the layer's list length
    uint32_t used;     // product layers (bit k: B layer k) with a key, from this thread's keys
};

// iblk_layer's counts and masks for a direct pair, as the A layer's writer list: the A edges whose
// ranges hold keys, wl[k] = A edge i | its idx << 21 and imask[k] = (P mask, M mask) in any order
// (slots from an LDS counter), so that k_large_products_direct reads one contiguous list per A layer.
// k_large_lists zeroed the count bytes; only ranges with keys store theirs. Cells beyond kPendCells per
// thread store at once. Barriers inside; every thread calls it.
template <int BS>
__device__ void cnt_layer_list(uint8_t* plds, uint32_t Bm, uint32_t nB, uint64_t nb_m, uint32_t nk, const uint32_t* recs,
                               cnt_pend& p, uint8_t* icnt, uint32_t* wl, ulonglong2* imask) {
    unsigned long long* M1 = (unsigned long long*)plds;
    unsigned long long* M2 = M1 + 2u * Bm;
    const uint32_t* tt = (const uint32_t*)(plds + kCntTtOff * Bm);
    uint32_t* wn = (uint32_t*)(plds + (kCntTtOff + 16u) * Bm) + 1;   // after stage_tt's dup word
    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < 4u * Bm; k += BS) M1[k] = 0ull;
    if (tid == 0) *wn = 0;
    __syncthreads();
    for (uint32_t q = tid; q < nk; q += BS) {   // (no shared buckets in a direct pair)
        const uint32_t v = recs[q];
        if (!v) continue;
        const uint32_t dd = v & 0xFFFu, j = (v >> 12) & 63u, e = (v >> 18) & 3u;
        if (e & 1u) atomicOr(&M1[dd], 1ull << j);
        if (e & 2u) atomicOr(&M2[dd], 1ull << j);
    }
    __syncthreads();
    // cell dd: its list word and slot + 1 (0: no range with keys), its masks
    auto cell = [&](uint32_t dd, uint32_t& i, uint32_t& w, ulonglong2& mk) -> uint32_t {
        if (dd >= 2u * Bm) return 0u;
        const uint32_t ch = dd >= Bm ? 1u : 0u;
        const uint32_t te = tt[dd + ch * Bm];   // tt slot ch 2B + idx
        if (te == kInf) return 0u;
        const unsigned long long x1 = M1[dd], x2 = M2[dd];
        if (!(x1 | x2)) return 0u;
        uint32_t j;
        i = div_small(te, nB, nb_m, j);
        w = i | (dd - ch * Bm) << 21;
        mk = make_ulonglong2(x1, x2);
        return atomicAdd(wn, 1u) + 1u;
    };
#pragma unroll
    for (uint32_t v = 0; v < kPendCells; ++v) p.k[v] = cell(tid + v * BS, p.i[v], p.w[v], p.m[v]);
    for (uint32_t dd = tid + kPendCells * BS; dd < 2u * Bm; dd += BS) {   // B > 384 only
        uint32_t i, w;
        ulonglong2 mk;
        const uint32_t k = cell(dd, i, w, mk);
        if (!k) continue;
        icnt[i] = (uint8_t)(__popcll(mk.x) + __popcll(mk.y));   // <= 128
        wl[k - 1u] = w;
        imask[k - 1u] = mk;
    }
    __syncthreads();   // the next A layer's staging overwrites M1 / M2, tt and recs
    p.n = *wn;
}

__device__ __forceinline__ void cnt_flush(const cnt_pend& p, uint8_t* icnt, uint32_t* wl, ulonglong2* imask,
                                          uint32_t* wln) {
#pragma unroll
    for (uint32_t u = 0; u < kPendCells; ++u) {
        if (!p.k[u]) continue;
        icnt[p.i[u]] = (uint8_t)(__popcll(p.m[u].x) + __popcll(p.m[u].y));
        wl[p.k[u] - 1u] = p.w[u];
        imask[p.k[u] - 1u] = p.m[u];
    }
    if (threadIdx.x == 0) *wln = p.n;
}
// Which keys emit, and in which order, follows from key PRESENCE alone when no key's products cancel:
// a P (M) cell emits iff some product lands in it (arithmetic.hpp:96-101 with sums assumed != 0).
// So the per-A-edge counts and masks of iblk_layer can be built before any multiply, the counts
// scanned into offsets, and the products kernel can write C's edge records at their positions from
// its epilogue: no per-key sums, first-insert times or key records go through HBM, and the range
// writer that gathered them is not needed. A key whose sum turns out to be 0 sends the pair to the
// host's redo (exact path), as the fresh kernel does.

// the dense side's first-insert shares only (no digits): tt[2][2B] as mx_stage_dense lays them out,
// at kCntTtOff (iblk_layer<LIST> reads them there), from the cells in the direct pair's A ids; false
// when the layer has duplicate (idx, ch) edges
template <int BS>
__device__ bool stage_tt(uint8_t* lds, uint32_t Bm, const layer_src& D, uint32_t tmul, const uint32_t (&pre)[4]) {
    uint32_t* tt = (uint32_t*)(lds + kCntTtOff * Bm);
    uint32_t* dup = (uint32_t*)(lds + (kCntTtOff + 16u) * Bm);
    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < 4 * Bm; k += BS) tt[k] = kInf;
    if (tid == 0) *dup = 0;
    __syncthreads();
    for (uint32_t k0 = tid; k0 < D.n; k0 += 4u * BS) {   // four edges per round (the first: loaded ahead)
        uint32_t e[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const uint32_t k = k0 + (uint32_t)v * BS;
            e[v] = k0 == tid ? pre[v] : D.ids[k < D.n ? k : 0u];   // A edge | dense cell << 21 (k_large_lists)
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            if (k0 + (uint32_t)v * BS >= D.n) break;
            const uint32_t cell = e[v] >> 21, ch = cell >= Bm ? 1u : 0u;
            const uint32_t sl = cell + ch * Bm;   // slot ch 2B + idx
            const uint32_t te = (e[v] & 0x1FFFFFu) * tmul;
            if (atomicCAS(&tt[sl], kInf, te) != kInf) *dup = 1;
            else tt[sl + Bm] = te;
        }
    }
    __syncthreads();
    return *dup == 0;
}

// Pass 1 of a direct pair, one workgroup per (pair, la_per_wg A layers) like k_large_products_la:
// per A layer, every key (r, B layer) gets its first-insert time and its P / M presence from the
// dense shares and the B layers' edges, one record per key (the products kernel's iblk record),
// then iblk_layer's counts and masks; product-layer used flags for compact_layers. A layer the
// matrix-core mode cannot take (duplicate edges, fewer than kLargeDenseMin edges) fails the pair
// (cnt[kCntIFail]): k_large_scan_direct sends it to the host's redo.
template <int BS>
// resident workgroups per CU k_large_count_la is compiled for: 6 (<= 80 VGPRs, no spills) against
// 5 (81 VGPRs unconstrained): cfg-4 chain 195 K against 188-190 K ct_mul/s on one stream; 7 spills
#ifndef PVAC_CNT_MINB
#define PVAC_CNT_MINB 6
#endif
__global__ __launch_bounds__(BS, PVAC_CNT_MINB) void k_large_count_la(mul_large_args g) {
    extern __shared__ __attribute__((aligned(16))) uint8_t plds[];
    const large_desc d = g.desc[g.sel[blockIdx.y]];   // registers (the kernel's stores could alias it)
    if (!d.direct) return;
    uint32_t* S = g.scratch;
    uint32_t* cnt = S + d.o_cnt;
    const uint32_t LA = d.LA, LB = d.LB, Bm = g.Bm, nB = d.nB;
    const uint32_t tid = threadIdx.x;
    const uint32_t i0 = blockIdx.x * g.la_per_wg;
    // The prologue's loads in dependency levels, each level's loads issued together (the A and B
    // chains are independent): 1 the pair's counters, its B layer ids, the first A layer id, B's
    // edge offset; 2 the layers' list ranges; 3 the id lists; 4 B's edge metas. (Issued in program
    // order the chains took seven dependent round trips per workgroup.) Reads past a short list
    // stay inside the pair's scratch and are not used.
    const uint32_t c2 = cnt[2], cf = cnt[kCntIFail], c0 = cnt[0], c1 = cnt[1];
    uint32_t lbv[kLaMaxLB];
#pragma unroll
    for (uint32_t k = 0; k < kLaMaxLB; ++k) lbv[k] = S[d.o_neB + k];
    uint32_t la_c = S[d.o_neA + min(i0, LA - 1u)];
    const uint64_t beo = g.B.e_off[d.pair];
    if (c2 || cf) return;
    const uint32_t neA = c0, neB = min(c1, kLaMaxLB);
    if (i0 >= neA) return;
    const uint32_t i1 = min(neA, i0 + g.la_per_wg);
    // level 2
    uint32_t nbv[kLaMaxLB], bst[kLaMaxLB];
#pragma unroll
    for (uint32_t k = 0; k < kLaMaxLB; ++k) {
        const uint32_t lb = k < neB ? lbv[k] : 0u;
        lbv[k] = lb;
        bst[k] = S[d.o_lstB + lb];
        nbv[k] = k < neB ? S[d.o_lstB + LB + lb] : 0u;   // <= kIblkMaxSparse (k_large_lists failed the pair otherwise)
    }
    uint32_t st_c = S[d.o_lstA + la_c], n_c = S[d.o_lstA + LA + la_c];
    const uint64_t mbj = tid < nB ? g.B.meta[beo + tid] : 0ull;   // bjt below
    // level 3 (A as a dense chain image: its ids are the 32-bit words of its meta region, k_large_lists)
    const bool aimg = g.A_img && g.A_img[d.pair];
    const uint32_t* idsA = aimg ? (const uint32_t*)(g.A.meta + g.A.e_off[d.pair]) : S + d.o_lstA + 2u * LA;
    const uint32_t* idsB = S + d.o_lstB + 2u * LB;
    uint32_t pre[4];
    auto load_ids = [&](uint32_t st, uint32_t n) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const uint32_t k = tid + (uint32_t)v * BS;
            pre[v] = idsA[st + (k < n ? k : 0u)];
        }
    };
    load_ids(st_c, n_c);
    uint32_t eb[kLaMaxLB];
#pragma unroll
    for (uint32_t k = 0; k < kLaMaxLB; ++k) eb[k] = k < neB ? idsB[bst[k] + (tid < nbv[k] ? tid : 0u)] : 0u;
    uint32_t la_n = i0 + 1u < i1 ? S[d.o_neA + i0 + 1u] : 0u;
    // level 4: B layers as per-edge (P slot offset, M slot offset, j, 1), padded to a multiple of 4
    // with (0, 0, INF, 0), as mx_stage_sparse computes them
    uint4* sp = (uint4*)(plds + g.lds_task);                          // [kLaMaxLB][kMxMaxSparse]
    uint32_t* bjt = (uint32_t*)(sp + kLaMaxLB * kMxMaxSparse);        // [64] B edge j: idx | ch << 16
    uint32_t* recs = bjt + 64;                                        // [kLaMaxLB][B]
    uint64_t mbk[kLaMaxLB];
#pragma unroll
    for (uint32_t k = 0; k < kLaMaxLB; ++k) mbk[k] = k < neB ? g.B.meta[beo + eb[k]] : 0ull;
#pragma unroll
    for (uint32_t k = 0; k < kLaMaxLB; ++k) {
        if (k < neB && tid < ((nbv[k] + 3u) & ~3u) && nbv[k] <= kMxMaxSparse) {
            uint4 v = make_uint4(0, 0, kInf, 0);
            if (tid < nbv[k]) {
                const uint32_t sidx = meta_idx(mbk[k]), sch = meta_ch(mbk[k]);
                v = make_uint4(sch * 2u * Bm + Bm - sidx, (sch ^ 1u) * 2u * Bm + Bm - sidx, eb[k], 1);
            }
            sp[k * kMxMaxSparse + tid] = v;
        }
    }
    if (tid < nB) bjt[tid] = meta_idx(mbj) | meta_ch(mbj) << 16;   // published by stage_tt's barriers
    const uint32_t* tt = (const uint32_t*)(plds + kCntTtOff * Bm);
#ifdef PVAC_DIR_STAMPS
    unsigned long long st_acc[4] = {0, 0, 0, 0}, t_prev = dir_stamp();
#endif
    // the previous layer's outputs, stored after this layer's staging (cnt_pend)
    cnt_pend pend;
    uint32_t pend_la = kInf, pend_base = 0;
    auto flush = [&]() {
        if (pend_la == kInf) return;   // workgroup-uniform
        cnt_flush(pend, (uint8_t*)(S + d.o_icnt), S + d.o_wle + pend_base, (ulonglong2*)(S + d.o_imask) + pend_base,
                  S + d.o_wln + pend_la);
        // product layers with a key: compact_layers keeps them (benign race: every writer stores 1)
#pragma unroll
        for (uint32_t k = 0; k < kLaMaxLB; ++k)
            if ((pend.used >> k) & 1u) S[d.o_used + (LA + LB) + pend_la * LB + lbv[k]] = 1;
        pend_la = kInf;
    };
    for (uint32_t i = i0; i < i1; ++i) {
        DSTAMP(0);
        const uint32_t la = late(la_c);
        const layer_src srcA{&g.A, 0, idsA + late(st_c), late(n_c)};
        bool ok = srcA.n >= kLargeDenseMin;
#pragma unroll
        for (uint32_t k = 0; k < kLaMaxLB; ++k) ok &= k >= neB || (nbv[k] <= kMxMaxSparse && nbv[k] <= srcA.n);
        if (!ok) {   // workgroup-uniform: this A layer's tasks would not all run on the matrix cores
            if (tid == 0) atomicExch(&cnt[kCntIFail], 1u);
            return;
        }
        if (!stage_tt<BS>(plds, Bm, srcA, nB, pre)) {
            if (tid == 0) atomicExch(&cnt[kCntIFail], 1u);
            return;
        }
        DSTAMP(1);
        const uint32_t lx = late(la_n);
        uint32_t st_n = 0, n_n = 0;
        if (i + 1u < i1) {   // workgroup-uniform
            st_n = S[d.o_lstA + lx];
            n_n = S[d.o_lstA + LA + lx];
        }
        flush();   // the previous layer's stores, behind this layer's loads
        uint32_t usedm = 0;
        for (uint32_t q = tid; q < neB * Bm; q += BS) {
            const uint32_t k = q / Bm, r = q - k * Bm;
            const uint4* e = sp + k * kMxMaxSparse;
            uint32_t tmin = kInf, pp = 0, pm = 0;
            // four sparse edges per step (padded lists): their LDS reads in flight together
            for (uint32_t x = 0; x < nbv[k]; x += 4) {
                uint4 in[4];
                uint32_t tp[4], tm[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) in[u] = e[x + u];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    tp[u] = tt[in[u].x + r];
                    tm[u] = tt[in[u].y + r];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    pp |= tp[u] != kInf ? in[u].w : 0u;
                    pm |= tm[u] != kInf ? in[u].w : 0u;
                    tmin = min(tmin, min(__builtin_elementwise_add_sat(tp[u], in[u].z),
                                         __builtin_elementwise_add_sat(tm[u], in[u].z)));
                }
            }
            uint32_t rv = 0;
            if (tmin != kInf) {
                const uint32_t eb = pp | pm << 1;
                // no shared buckets in a direct pair (the host's slots_share_bucket check)
                uint32_t j;
                const uint32_t ia = div_small(tmin, nB, d.nb_m, j);
                const uint32_t ij = bjt[j] & 0xFFFFu;
                const uint32_t xx = r >= ij ? r - ij : r + Bm - ij;
                const uint32_t dd = tt[xx] == ia * nB ? xx : Bm + xx;
                rv = dd | j << 12 | eb << 18 | kRecKey;
                usedm |= 1u << k;
            }
            recs[k * Bm + r] = rv;
        }
        __syncthreads();
        DSTAMP(2);
        uint32_t la_n2 = 0;
        if (i + 1u < i1) {
            load_ids(late(st_n), late(n_n));
            if (i + 2u < i1) la_n2 = S[d.o_neA + i + 2u];
        }
        const uint32_t lbase = late(st_c);   // the layer's list slice: as its edge ids
        cnt_layer_list<BS>(plds, Bm, nB, d.nb_m, neB * Bm, recs, pend, (uint8_t*)(S + d.o_icnt), S + d.o_wle + lbase,
                           (ulonglong2*)(S + d.o_imask) + lbase);
        pend.used = usedm;
        pend_la = la;
        pend_base = lbase;
        DSTAMP(3);
#ifdef PVAC_DIR_STAMPS
        if (tid == 0) atomicAdd(&g_dir_stamps[13], (unsigned long long)pend.n);
#endif
        la_c = lx;
        st_c = st_n;
        n_c = n_n;
        la_n = la_n2;
    }
    flush();
#ifdef PVAC_DIR_STAMPS
    if (tid == 0) {
        for (int p = 0; p < 4; ++p) atomicAdd(&g_dir_stamps[8 + p], st_acc[p]);
        atomicAdd(&g_dir_stamps[12], (unsigned long long)(i1 - i0));
    }
#endif
}

// count bytes of a direct pair's A edges (4 per word): their sum, and the sum over the bytes of a
// 32-edge group at positions above b (the word holding positions lo .. lo + 3)
__device__ __forceinline__ uint32_t byte_sum(uint32_t x) { return __builtin_amdgcn_sad_u8(x, 0u, 0u); }
__device__ __forceinline__ uint32_t byte_sum(const uint4& x) {
    return __builtin_amdgcn_sad_u8(x.x, 0u, __builtin_amdgcn_sad_u8(x.y, 0u, __builtin_amdgcn_sad_u8(x.z, 0u, byte_sum(x.w))));
}
__device__ __forceinline__ uint32_t bytes_above(uint32_t x, uint32_t lo, uint32_t b) {
    const uint32_t m = b < lo ? 0xFFFFFFFFu : b >= lo + 3u ? 0u : 0xFFFFFFFFu << (8u * (b - lo + 1u));
    return byte_sum(x & m);
}
// an A edge's exclusive suffix offset: its group's offset plus the counts of the group's later edges
__device__ __forceinline__ uint32_t dir_edge_off(const uint4* c8, const uint32_t* wo, uint32_t e) {
    const uint32_t gi = e >> 5, b = e & 31u;
    const uint4 a = c8[2u * gi], c = c8[2u * gi + 1u];
    return wo[gi] + bytes_above(a.x, 0u, b) + bytes_above(a.y, 4u, b) + bytes_above(a.z, 8u, b) +
           bytes_above(a.w, 12u, b) + bytes_above(c.x, 16u, b) + bytes_above(c.y, 20u, b) + bytes_above(c.z, 24u, b) +
           bytes_above(c.w, 28u, b);
}

// Pass 2 of a direct pair, one workgroup per pair: the total, the guard_budget decision, and the
// per-A-edge count bytes turned into exclusive suffix offsets per 32-edge group (an edge's own
// offset adds its group's later bytes: dir_edge_off). A pair with shared buckets, a fallback or
// the canonical order is not direct after all: it goes to the host's redo.
__global__ __launch_bounds__(kLBig) void k_large_scan_direct(mul_large_args g) {
    __shared__ uint32_t part[kLBig / 64];
    const large_desc& d = g.desc[blockIdx.x];
    if (!d.direct) return;
    uint32_t* S = g.scratch;
    uint32_t* cnt = S + d.o_cnt;
    if (cnt[2]) return;
    const int tid = threadIdx.x;
    const uint4* c8 = (const uint4*)(S + d.o_icnt);   // count bytes, two uint4 per group of 32 A edges
    uint32_t* wo = S + d.o_iwo;
    const uint32_t ng = (d.nA + 31u) >> 5;
    // one pass: the groups' suffix offsets are written while the total accumulates; a pair that is
    // not direct after all (checked after the pass) is redone, so offsets written for it are never read
    if (cnt[kCntIFail] || cnt[kCntIShared] || (g.flags & PVAC_MUL_ORDER_CANONICAL) != 0) {
        if (tid == 0) {
            cnt[kCntRedo] = 1;
            g.pair_status[d.pair] = kPairRedo;
        }
        return;
    }
    uint32_t run0 = 0;
    for (uint32_t base = 0; base < ng; base += 4u * kLBig) {
        const uint32_t r0 = base + 4u * (uint32_t)tid;
        uint4 x[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {   // loads first
            const uint32_t r = r0 + (uint32_t)k, w = ng - 1u - r;
            x[2 * k] = r < ng ? c8[2u * w] : make_uint4(0u, 0u, 0u, 0u);
            x[2 * k + 1] = r < ng ? c8[2u * w + 1u] : make_uint4(0u, 0u, 0u, 0u);
        }
        uint32_t v[4];
        uint32_t local = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[k] = byte_sum(x[2 * k]) + byte_sum(x[2 * k + 1]);
            local += v[k];
        }
        uint32_t tot;
        uint32_t run = run0 + wg_exclusive_scan<kLBig>(local, part, tot);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t r = r0 + (uint32_t)k;
            if (r < ng) wo[ng - 1u - r] = run;
            run += v[k];
        }
        run0 += tot;
    }
    const uint32_t total = run0;
    if (total > g.edge_budget) {   // guard_budget's canonical order: the general path (redo)
        if (tid == 0) {
            cnt[kCntRedo] = 1;
            g.pair_status[d.pair] = kPairRedo;
        }
        return;
    }
    if (tid == 0) {
        cnt[3] = total;
        cnt[4] = 0;
        cnt[kCntDirect] = 1;
        // a chain step writes C as a dense image when every cell of every product layer (la, lb) with
        // edges on both sides holds a key (and the hash positions fit the 21-bit ids the next step's
        // lists carry)
        cnt[kCntImg] = g.C_img && !g.salt_pos && (uint64_t)total == (uint64_t)cnt[0] * cnt[1] * 2u * g.Bm &&
                               total < (1u << 21)
                           ? 1u
                           : 0u;
        g.C.e_cnt[d.pair] = total;
        g.pair_status[d.pair] = 0;
    }
}

// direct pairs handed to the redo (not direct after all, or a key whose products cancel): onto the
// redo list the host re-runs on the full layout (ct_mul_exec's redo step)
__global__ __launch_bounds__(64) void k_large_direct_redo(mul_large_args g) {
    const uint32_t q = blockIdx.x * 64u + threadIdx.x;
    if (q >= g.nl) return;
    const large_desc& d = g.desc[q];
    if (!d.direct) return;
    const uint32_t* cnt = g.scratch + d.o_cnt;
    if (cnt[2]) return;
    if (!cnt[kCntRedo]) {   // finished here: its C is a dense image when the image writer ran
        if (g.C_img && cnt[kCntDirect] && cnt[kCntImg]) {
            g.C_img[d.pair] = 1u;
            if (g.img_count) atomicAdd(g.img_count, 1ull);
        }
        return;
    }
    g.pair_status[d.pair] = kPairRedo;
    g.redo_ids[atomicAdd(g.redo_cnt, 1u)] = d.pair;
}

// One workgroup per (pair, kLaPerWG A layers) for pairs with at most kLaMaxLB B layers (chain
// steps): the B layers' sparse sides are staged once per workgroup and each A layer's dense table
// once for all B layers, so a chain step reads every A edge once (a task per workgroup read it
// |B.L| times) and pays the dependent header loads once per kLaPerWG x |B.L| tasks. The kernel is
// latency-bound: 4 workgroups per CU (<= 128 VGPRs, 32 KB of LDS) against 3: -10%; forced to 96
// VGPRs for 5 per CU it was 28% slower.
// Tasks the matrix-core mode does not take: sparse x sparse (and layers with duplicate edges) run
// the scatter mode in place; dense tasks with a large sparse side (column mode, 33 KB of LDS) go to
// a per-pair list for k_large_products_defer.
#ifndef PVAC_LA_MINB   // resident workgroups per CU the A-layer-major kernel is compiled for
#define PVAC_LA_MINB 4
#endif
template <int BS>
__global__ __launch_bounds__(BS, PVAC_LA_MINB) void k_large_products_la(mul_large_args g) {
    extern __shared__ __attribute__((aligned(16))) uint8_t plds[];
    uint32_t py = blockIdx.y, px = blockIdx.x;
    if (g.la_xcd) {   // workgroups go to XCDs round-robin by linear id: XCD x takes pairs x, x + 8, ...
        const uint32_t lin = blockIdx.x + blockIdx.y * gridDim.x, k = lin >> 3;
        py = (k / gridDim.x) * 8u + (lin & 7u);
        px = k % gridDim.x;
        if (py >= g.n_la) return;
    }
    const large_desc& d = g.desc[g.sel[py]];
    if (d.direct) return;   // k_large_products_direct
    uint32_t* S = g.scratch;
    const uint32_t* cnt = S + d.o_cnt;
    if (cnt[2]) return;
    const uint32_t neA = cnt[0], neB = min(cnt[1], kLaMaxLB);   // the host sends pairs with |B.L| <= kLaMaxLB
    const uint32_t i0 = px * g.la_per_wg;
    if (i0 >= neA) return;
    const uint32_t LA = d.LA, LB = d.LB, Bm = g.Bm, nB = d.nB;
    uint8_t* sreg = plds + g.lds_task;   // per B layer: prec | pinf
    uint32_t lbv[kLaMaxLB], nbv[kLaMaxLB];
    uint32_t okm = 0;   // B layers staged as MX sparse sides
#pragma unroll
    for (uint32_t k = 0; k < kLaMaxLB; ++k) {
        lbv[k] = 0;
        nbv[k] = 0;
        if (k < neB) {
            const uint32_t lb = S[d.o_neB + k];
            const layer_src srcB = side_layer(&g.B, g.B.e_off[d.pair], S, d.o_lstB, LB, lb);
            lbv[k] = lb;
            nbv[k] = srcB.n;
            if (srcB.n <= kMxMaxSparse) {
                okm |= 1u << k;
                uint4* prec = (uint4*)(sreg + k * kMxSparseBytes);
                mx_stage_sparse(prec, prec + 3u * kMxMaxSparse, Bm, srcB, 1u, threadIdx.x);
            }
        }
    }
    // iblk: per-A-edge counts and ranks (iblk_layer) instead of block marks, unless the pair has
    // fallen back (cnt[kCntIFail], set by k_large_lists or by a workgroup below)
    bool ib = d.iblk && !S[d.o_cnt + kCntIFail];
    uint32_t* bjt = (uint32_t*)(sreg + kLaMaxLB * kMxSparseBytes);   // B edge j: idx | ch << 16
    uint32_t* recs = bjt + 64;                                           // [kLaMaxLB][B] key records
    if (ib && threadIdx.x < nB) {   // published by the dense staging's barriers
        const uint64_t mb = g.B.meta[g.B.e_off[d.pair] + threadIdx.x];
        bjt[threadIdx.x] = meta_idx(mb) | meta_ch(mb) << 16;
    }
    const task_out o{S + d.o_tkey, S + d.o_info, (ulonglong2*)(S + d.o_sums), group_heads(g, d),
                     d.iblk ? nullptr : (unsigned long long*)w64(S, d.o_bmask)};
    const uint32_t i1 = min(neA, i0 + g.la_per_wg);
    for (uint32_t i = i0; i < i1; ++i) {
        const uint32_t la = S[d.o_neA + i];
        const layer_src srcA = side_layer(&g.A, g.A.e_off[d.pair], S, d.o_lstA, LA, la);
        const uint32_t na = srcA.n;
        uint32_t mxm = 0;   // B layers whose task with this A layer runs on the matrix cores
        bool dupA = false;
        if (na >= kLargeDenseMin)
#pragma unroll
            for (uint32_t k = 0; k < kLaMaxLB; ++k)
                if (((okm >> k) & 1u) && na >= nbv[k]) mxm |= 1u << k;
        if (mxm) {
#ifdef PVAC_EXP_STAGE2   // experiment builds only: the dense staging twice (same result)
            mx_stage_dense<BS>(plds, Bm, srcA, nB);
#endif
            if (mx_stage_dense<BS>(plds, Bm, srcA, nB)) {   // barriers inside (they also publish the B staging)
#pragma unroll
                for (uint32_t k = 0; k < kLaMaxLB; ++k) {
                    if (!((mxm >> k) & 1u)) continue;
                    const uint4* prec = (const uint4*)(sreg + k * kMxSparseBytes);
                    const uint32_t lp = la * LB + lbv[k];
                    task_out ok = o;
                    if (ib) {
                        ok.recs = recs + k * Bm;
                        ok.bjt = bjt;
                        ok.nB = nB;
                        ok.nb_m = d.nb_m;
                    }
                    if (mx_blocks<BS>(plds, prec, prec + 3u * kMxMaxSparse, nbv[k], Bm, (uint64_t)lp * Bm, ok))
                        S[d.o_used + (LA + LB) + lp] = 1;
                }
            } else {
                mxm = 0;   // duplicate edges in this A layer: its tasks take run_task's scatter mode
                dupA = true;
            }
            __syncthreads();
        }
        for (uint32_t k = 0; k < neB; ++k) {
            if ((mxm >> k) & 1u) continue;
            if (!dupA && max(na, nbv[k]) >= kLargeDenseMin) {
                if (threadIdx.x == 0) S[d.o_defer + atomicAdd((uint32_t*)cnt + 7, 1u)] = i << 16 | k;
            } else {
                run_task<BS, false>(g, d, la, lbv[k], plds, false);   // scatter mode
            }
        }
        if (ib) {
            // every task of this A layer ran on the matrix cores (its dense table staged, no duplicate
            // (idx, ch) edges): count and rank per A edge; otherwise the pair falls back
            if (mxm == (1u << neB) - 1u) {
                static_assert(kLaMaxLB == 4, "iblk_layer takes the B layers as a uint4");
                for (int rep_ = 0; rep_ < PVAC_EXP_IBREP; ++rep_)   // experiment builds repeat it (idempotent)
                    iblk_layer<BS>(plds, g, d, la, make_uint4(lbv[0], lbv[1], lbv[2], lbv[3]), neB, recs, S + d.o_icnt,
                                   (ulonglong2*)(S + d.o_imask));
            } else {
                if (threadIdx.x == 0) atomicExch(&S[d.o_cnt + kCntIFail], 1u);
                ib = false;
            }
        }
    }
}

// Pass 3 of a direct pair (after k_large_scan_direct and the layers pass), one workgroup per
// (pair, la_per_wg A layers) like k_large_products_la. Per A layer: the matrix-core products of every
// B layer with each row's folded P / M sums staged in LDS by key slot (no first-insert times: the
// order is already in the counts and masks of k_large_count_la), then a range writer: the A layer's
// ranges (its A edges with keys, positions [off(i), off(i) + cnt(i)) of the output) are walked like
// k_large_write_ranges walks all of them, each position resolved to its key (j DESC, P before M) and
// its value read from LDS, so C's records are stored range by range, coalesced, with no per-key
// scratch in HBM. A staged value of 0 at a present cell (products that cancel) flags the pair for
// the host's redo.
//
// LDS: dig1 [2][B] uint4 (one copy per channel: slot (r - idx) mod B with a wrap, 32 B per index) |
// per B layer: prec | pinf (kMxSparseBytes) | bjt [64] | stg [neB][B][2] (16 B per cell)
__host__ __device__ inline uint32_t dir_lds_base(uint32_t Bm) {   // the digit table, reused by the writer
    // okey [8 B] u16 | obase, oidx, oexc [256] u32 | omk [256] 16 B | part
    return al16(max(32u * Bm, 16u * Bm + 28u * 256u + 64u));
}
__host__ __device__ inline uint32_t dir_lds_bytes(uint32_t Bm, uint32_t nbl) {
    return dir_lds_base(Bm) + nbl * kMxSparseBytes + kIblkBjtBytes + nbl * 32u * Bm;
}

// the dense side (an A layer) as digits, one copy per channel (k_large_count_la checked for
// duplicate cells). Barriers inside; every thread calls it.
// slab: kInf, or (A held as a dense chain image) the layer's first edge slot: list entry k's weight
// sits at slab + k instead of at its hash-order edge (a contiguous read instead of a gather)
template <int BS>
__device__ void dir_stage_dense(uint4* dig, uint32_t Bm, const layer_src& D, uint32_t slab) {
    constexpr uint32_t kV = 3;   // a dense A layer (<= 2 B = 674 edges) in one round of loads
    const uint32_t tid = threadIdx.x;
    uint32_t c[kV];
    uint64_t lo[kV], hi[kV];
    auto load = [&](uint32_t k0) {   // direct pairs' A ids: A edge | dense cell << 21 (k_large_lists)
#pragma unroll
        for (uint32_t v = 0; v < kV; ++v) {
            const uint32_t k = k0 + v * BS;
            const uint32_t kc = k < D.n ? k : 0u;   // D.n >= kLargeDenseMin
            const uint32_t id = D.ids[kc];
            c[v] = id >> 21;
            const uint32_t e = slab != kInf ? slab + kc : (id & 0x1FFFFFu);
            lo[v] = D.X->w_lo[D.eo + e];
            hi[v] = D.X->w_hi[D.eo + e];
        }
    };
    auto put = [&](uint32_t k0) {
#pragma unroll
        for (uint32_t v = 0; v < kV; ++v) {
            if (k0 + v * BS >= D.n) break;
            uint64_t dl, dh;
            // an image's weights are the previous step's folded sums, canonical already
            fp_digits8(slab != kInf ? fp{lo[v], hi[v]} : fp_canon(lo[v], hi[v]), dl, dh);
            dig[c[v]] = make_uint4((uint32_t)dl, (uint32_t)(dl >> 32), (uint32_t)dh, (uint32_t)(dh >> 32));
        }
    };
    load(tid);   // in flight across the zero fill and its barrier
    for (uint32_t k = tid; k < 2 * Bm; k += BS) dig[k] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    put(tid);
    for (uint32_t k0 = tid + kV * BS; k0 < D.n; k0 += kV * BS) {
        load(k0);
        put(k0);
    }
    __syncthreads();
}

// a B layer as the MFMA sparse side (prec as mx_stage_sparse) with pinf = (B - idx, P table base,
// M table base) for the one-copy dense table; no first-insert shares. Thread k writes edge k.
__device__ __forceinline__ void dir_stage_sparse(uint4* prec, uint4* pinf, uint32_t Bm, const layer_src& Sd, uint32_t k) {
    const uint32_t nks = (Sd.n + 1u) >> 1;
    if (k >= 2u * nks) return;
    uint4 mid = make_uint4(0, 0, 0, 0);
    uint4 inf = make_uint4(0, 0, Bm, 0);   // padding edge: zero digits
    if (k < Sd.n) {
        const edge_rec x = load_edge(Sd, k);
        uint64_t dl, dh;
        fp_digits8(fp_canon(x.lo, x.hi), dl, dh);
        const uint64_t rl = __builtin_bswap64(dh), rh = __builtin_bswap64(dl);   // digit 15 - x at byte x
        mid = make_uint4((uint32_t)rl, (uint32_t)(rl >> 32), (uint32_t)rh, (uint32_t)(rh >> 32));
        const uint32_t sidx = meta_idx(x.meta), sch = meta_ch(x.meta);
        inf = make_uint4(Bm - sidx, sch * Bm, (sch ^ 1u) * Bm, 0);
    }
    prec[3u * k] = make_uint4(0, 0, 0, 0);
    prec[3u * k + 1u] = mid;
    prec[3u * k + 2u] = make_uint4(0, 0, 0, 0);
    pinf[k] = inf;
}

// one task's products, each row's P (half 0) / M (half 1) sum into stg[(r) 2 + h]
#ifndef PVAC_DIR_PINF_REG   // A/B builds: 1 = the k-steps' sparse-edge offsets held in registers for every block
#define PVAC_DIR_PINF_REG 0   // (177 instead of 187 VALU per block, but 21 spill ops: 428-429 K against 430-431 K)
#endif
template <int BS, int NKS>
__device__ void dir_rows_n(const uint4* dig, const uint4* prec, const uint4* pinf, uint32_t Bm, ulonglong2* stg) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t h = lane >> 5, n = lane & 31u;
    mx_v4 frag[NKS];
    {
        const uint32_t y0 = 31u - n, sh = y0 & 3u;
        const uint32_t* pw = (const uint32_t*)prec + (y0 >> 2) + 12u * h;
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
            const uint32_t* q = pw + 24u * (uint32_t)s;
            const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
            frag[s] = mx_v4{(int)__builtin_amdgcn_alignbyte(w1, w0, sh), (int)__builtin_amdgcn_alignbyte(w2, w1, sh),
                            (int)__builtin_amdgcn_alignbyte(w3, w2, sh), (int)__builtin_amdgcn_alignbyte(w4, w3, sh)};
        }
    }
#if PVAC_DIR_PINF_REG
    // the k-steps' sparse-edge words, byte offsets into the digit table packed as
    // (B - idx) 16 | (P table base) 16 << 16, held in registers for every block: the digit reads of a
    // block depend on no LDS read of their own (the M table base is B 16 minus the P one)
    uint32_t pk[NKS];
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        const uint4 in = pinf[2u * (uint32_t)s + h];
        pk[s] = (in.x << 4) | (in.y << 20);
    }
    const uint32_t B16 = Bm << 4;
#endif
    const uint32_t nblk = (Bm + 31u) >> 5;
    for (uint32_t blk = wave; blk < nblk; blk += BS / 64) {
        const uint32_t r = blk * 32u + n;
        const bool live = r < Bm;
        const uint32_t rr = live ? r : 0u;
        mx_v16 aP{}, aM{};
#if PVAC_DIR_PINF_REG
        const uint32_t rr16 = rr << 4;
        const uint8_t* dg = (const uint8_t*)dig;
#pragma unroll
        for (int s = 0; s < NKS; ++s) asm volatile("" : "+v"(pk[s]));   // unpacked per block: 10 registers, not 20
#endif
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
#if PVAC_DIR_PINF_REG
            uint32_t x = rr16 + (pk[s] & 0xFFFFu);   // 16 ((r - idx) mod B)
            x = min(x, x - B16);
            const uint4 dp = *(const uint4*)(dg + x + (pk[s] >> 16));
            const uint4 dm = *(const uint4*)(dg + (x + B16) - (pk[s] >> 16));
#else
            const uint4 in = pinf[2u * (uint32_t)s + h];
            uint32_t x = rr + in.x;   // (r - idx) mod B
            x = min(x, x - Bm);
            const uint4 dp = dig[in.y + x], dm = dig[in.z + x];
#endif
            aP = __builtin_amdgcn_mfma_i32_32x32x32_i8(frag[s], mx_v4{(int)dp.x, (int)dp.y, (int)dp.z, (int)dp.w}, aP, 0, 0, 0);
            aM = __builtin_amdgcn_mfma_i32_32x32x32_i8(frag[s], mx_v4{(int)dm.x, (int)dm.y, (int)dm.z, (int)dm.w}, aM, 0, 0, 0);
        }
        int64_t paw, pbw, maw, mbw;
        mx_groups(aP, paw, pbw);
        mx_groups(aM, maw, mbw);
        const int64_t ra = shfl_xor64(h ? paw : maw, 32), rb = shfl_xor64(h ? pbw : mbw, 32);
        const fp v = mx_fold(h ? ra : paw, h ? maw : ra, h ? rb : pbw, h ? mbw : rb);
        if (live) stg[2u * r + h] = make_ulonglong2(v.lo, v.hi);
    }
}

template <int BS>
__device__ void dir_rows(const uint4* dig, const uint4* prec, const uint4* pinf, uint32_t ns, uint32_t Bm, ulonglong2* stg) {
    static_assert(kMxKS == 10, "one instantiation per k-step count");
    switch ((ns + 1u) >> 1) {   // workgroup-uniform
    case 0: return;
    case 1: dir_rows_n<BS, 1>(dig, prec, pinf, Bm, stg); return;
    case 2: dir_rows_n<BS, 2>(dig, prec, pinf, Bm, stg); return;
    case 3: dir_rows_n<BS, 3>(dig, prec, pinf, Bm, stg); return;
    case 4: dir_rows_n<BS, 4>(dig, prec, pinf, Bm, stg); return;
    case 5: dir_rows_n<BS, 5>(dig, prec, pinf, Bm, stg); return;
    case 6: dir_rows_n<BS, 6>(dig, prec, pinf, Bm, stg); return;
    case 7: dir_rows_n<BS, 7>(dig, prec, pinf, Bm, stg); return;
    case 8: dir_rows_n<BS, 8>(dig, prec, pinf, Bm, stg); return;
    case 9: dir_rows_n<BS, 9>(dig, prec, pinf, Bm, stg); return;
    default: dir_rows_n<BS, 10>(dig, prec, pinf, Bm, stg); return;
    }
}

// cache policy bits of the products kernel's record stores. Streaming (2) was measured against the
// default (0) on the cfg-4 chain: HBM writes 84.4 against 70.8 GB per 4096 inputs (lines leave L2
// before their neighbours' records fill them, then go out again), reads 47.2 against 58.5, time equal
#ifndef PVAC_DIR_STORE_AUX
#define PVAC_DIR_STORE_AUX 0
#endif
template <int BS>
__global__ __launch_bounds__(BS, PVAC_LA_MINB) void k_large_products_direct(mul_large_args g) {
    extern __shared__ __attribute__((aligned(16))) uint8_t plds[];
    // a register copy of the descriptor: C's stores could alias it, so field reads through the
    // reference were reloaded from memory (a dependent round trip each) after every store
    const large_desc d = g.desc[g.sel[blockIdx.y]];
    if (!d.direct) return;
    uint32_t* S = g.scratch;
    uint32_t* cnt = S + d.o_cnt;
    if (cnt[2] || !cnt[kCntDirect]) return;
    const uint32_t neA = cnt[0], neB = min(cnt[1], g.dir_lb);   // the host sized the LDS for dir_lb B layers
    const uint32_t i0 = blockIdx.x * g.la_per_wg;
    if (i0 >= neA) return;
    const uint32_t LA = d.LA, LB = d.LB, Bm = g.Bm, nB = d.nB;
    static_assert(BS <= 256, "dir_lds_base holds the writer's per-entry words for 256 entries");
    const uint32_t tid = threadIdx.x;
#ifdef PVAC_DIR_STAMPS
    unsigned long long st_acc[9] = {}, t_prev = dir_stamp();
#endif
    uint4* dig = (uint4*)plds;
    uint8_t* sreg = plds + dir_lds_base(Bm);                           // per B layer: prec | pinf
    uint32_t* bjt = (uint32_t*)(sreg + g.dir_lb * kMxSparseBytes);     // B edge j: idx | k << 12 | lb << 16
    ulonglong2* stg = (ulonglong2*)(bjt + 64);                         // [k][B][2]
    uint32_t lbv[kLaMaxLB], nbv[kLaMaxLB];
#pragma unroll
    for (uint32_t k = 0; k < kLaMaxLB; ++k) {
        lbv[k] = 0;
        nbv[k] = 0;
        if (k < neB) {
            const uint32_t lb = S[d.o_neB + k];
            const layer_src srcB = side_layer(&g.B, g.B.e_off[d.pair], S, d.o_lstB, LB, lb);
            lbv[k] = lb;
            nbv[k] = srcB.n;   // <= kMxMaxSparse: k_large_count_la checked
            uint4* prec = (uint4*)(sreg + k * kMxSparseBytes);
            dir_stage_sparse(prec, prec + 3u * kMxMaxSparse, Bm, srcB, tid);
        }
    }
    const uint64_t beo = g.B.e_off[d.pair], aeo = g.A.e_off[d.pair], ceo = g.C.e_off[d.pair];
    if (tid < nB) {   // published by the dense staging's barriers
        const uint32_t lb = meta_layer(g.B.meta[beo + tid]);
        uint32_t kk = 0;
#pragma unroll
        for (uint32_t k = 0; k < kLaMaxLB; ++k)
            if (k < neB && lbv[k] == lb) kk = k;
        bjt[tid] = meta_idx(g.B.meta[beo + tid]) | kk << 12 | lb << 16;
    }
    const uint4* c8 = (const uint4*)(S + d.o_icnt);   // count bytes (k_large_count_la)
    const uint32_t* wo = S + d.o_iwo;                 // group offsets (k_large_scan_direct)
    const ulonglong2* wlm = (const ulonglong2*)(S + d.o_imask);   // writer lists (k_large_count_la)
    const uint32_t* wle = S + d.o_wle;
    const uint32_t* remap = S + d.o_used;  // k_large_layers left the remap here (k_large_layers ran before)
    // C's records by buffer stores: one 32-bit offset for the three arrays
    const __amdgpu_buffer_rsrc_t rmeta = __builtin_amdgcn_make_buffer_rsrc(g.C.meta + ceo, 0, 0x7FFFFFF8, 0x00020000);
    const __amdgpu_buffer_rsrc_t rlo = __builtin_amdgcn_make_buffer_rsrc(g.C.w_lo + ceo, 0, 0x7FFFFFF8, 0x00020000);
    const __amdgpu_buffer_rsrc_t rhi = __builtin_amdgcn_make_buffer_rsrc(g.C.w_hi + ceo, 0, 0x7FFFFFF8, 0x00020000);
    const uint32_t i1 = min(neA, i0 + g.la_per_wg);
    const bool aimg = g.A_img && g.A_img[d.pair];   // A as dense images (k_large_lists made its lists the slabs)
    const bool cimg = cnt[kCntImg] != 0;             // C as dense images (k_large_scan_direct)
    // image slabs: C's kept product layers are exactly those with keys, last in C's layer order and in
    // (la, lb) order, one slab of 2B cells each: C layer lid's slab starts at (lid - nbase) 2B
    const uint32_t nbase = cimg ? (uint32_t)g.C.l_cnt[d.pair] - cnt[0] * cnt[1] : 0u;   // k_large_layers set l_cnt
    // layer headers one layer ahead: the next layer's id loads during this layer's staging, its
    // list range and writer-list length during this layer's writer
    uint32_t la = S[d.o_neA + i0];
    uint32_t a_start = S[d.o_lstA + la], a_n = S[d.o_lstA + LA + la], a_nw = S[d.o_wln + la];
    for (uint32_t ia = i0; ia < i1; ++ia) {
        const layer_src srcA{&g.A, aeo, (aimg ? (const uint32_t*)(g.A.meta + aeo) : S + d.o_lstA + 2u * LA) + a_start, a_n};
        uint32_t lid[kLaMaxLB];
#pragma unroll
        for (uint32_t k = 0; k < kLaMaxLB; ++k) lid[k] = k < neB ? remap[LA + LB + la * LB + lbv[k]] : 0u;
        const uint32_t la_nx = ia + 1u < i1 ? S[d.o_neA + ia + 1u] : 0u;
        DSTAMP(0);
        dir_stage_dense<BS>(dig, Bm, srcA, aimg ? a_start : kInf);   // barriers inside (they also publish the B staging)
        DSTAMP(1);
        for (uint32_t k = 0; k < neB; ++k) {
            const uint4* prec = (const uint4*)(sreg + k * kMxSparseBytes);
            dir_rows<BS>(dig, prec, prec + 3u * kMxMaxSparse, nbv[k], Bm, stg + 2u * Bm * k);
        }
        __syncthreads();
        DSTAMP(2);
        // writer: the A layer's list (its A edges with keys, contiguous; one offset gather each), a
        // round of up to BS list entries at a time. Each entry's thread expands its range's keys in
        // emit order (j DESC, P before M at one j) into okey[excl + kk] (the dead digit table), then
        // every thread takes output slots q = tid, tid + BS, ... of the round: balanced across the
        // waves, stores coalesced within each range, no search.
        const uint32_t lx = late(la_nx);
        uint32_t st_nx = 0, n_nx = 0, nw_nx = 0;
        if (ia + 1u < i1) {   // workgroup-uniform
            st_nx = S[d.o_lstA + lx];
            n_nx = S[d.o_lstA + LA + lx];
            nw_nx = S[d.o_wln + lx];
        }
        const uint32_t lbase = a_start, nw = a_nw;
        uint16_t* okey = (uint16_t*)dig;                       // [<= 8 B] j | ch << 6 | entry << 7
        uint32_t* obase = (uint32_t*)(plds + 16u * Bm);        // [BS] position base: off(i) - excl
        uint32_t* oidx = obase + BS;                           // [BS] the entry's A idx
        uint32_t* oexc = oidx + BS;                            // [BS] the entry's first slot in okey
        ulonglong2* omk = (ulonglong2*)(oexc + BS);            // [BS] the entry's P / M masks
        uint32_t* part = (uint32_t*)(omk + BS);                // [BS / 64] scan partials
        const uint32_t lane = tid & 63u, wave = tid >> 6;
        if (cimg) {
            // dense image writer (a chain step whose C the next step reads): C layer lid (a product
            // layer with keys) owns the 2B slots from (lid - nbase) 2B, cell c = ch B + r at slot + c:
            // 32-bit word s of C's meta region = hash-order position | c << 21 (the next step's list id),
            // the weights in cell order. One wave per writer-list entry, one lane per B edge j: key (j, P) sits after
            // the entry's keys of larger j, (j, M) right after (j, P). With at most two B layers (chain
            // steps) the positions go to an LDS table by cell (the dead okey region, 8 B x 2B) and every
            // store is coalesced; otherwise each key's meta is stored where it is found.
            const bool ptab_ok = neB <= 2u;   // workgroup-uniform
            uint32_t* ptab = (uint32_t*)plds;   // [k][2B] position of cell c of staged B layer k
            // lane j's B edge (the same for every entry): its idx, staged layer and position row
            const uint32_t bjl = bjt[lane];
            const uint32_t kbl = (bjl >> 12) & 15u, idxl = bjl & 0xFFFu;
            uint32_t* const ptl = ptab + kbl * 2u * Bm;
            for (uint32_t b0 = 0; b0 < nw; b0 += BS) {   // workgroup-uniform
                const uint32_t kq = b0 + tid;
                const bool lv = kq < nw;
                const uint32_t we = lv ? wle[lbase + kq] : 0u;
                const ulonglong2 mk = lv ? wlm[lbase + kq] : make_ulonglong2(0ull, 0ull);
                obase[tid] = lv ? dir_edge_off(c8, wo, we & 0x1FFFFFu) : 0u;
                oidx[tid] = we >> 21;
                omk[tid] = make_ulonglong2(mk.x & ~(1ull << 63), mk.y);
                __syncthreads();
                DSTAMP(4);
                const uint32_t ne = min(nw - b0, (uint32_t)BS);
                for (uint32_t l = wave; l < ne; l += BS / 64) {   // wave-uniform
                    const ulonglong2 m2 = omk[l];
                    const uint32_t hp = (uint32_t)(m2.x >> lane) & 1u, hm = (uint32_t)(m2.y >> lane) & 1u;
                    if (!(hp | hm)) continue;
                    const uint32_t above =
                        lane == 63u ? 0u : (uint32_t)__popcll(m2.x >> (lane + 1u)) + (uint32_t)__popcll(m2.y >> (lane + 1u));
                    const uint32_t pos = obase[l] + above;
                    const uint32_t r = mod_small(oidx[l] + idxl, Bm);
                    if (ptab_ok) {
                        if (hp) ptl[r] = pos;
                        if (hm) ptl[Bm + r] = pos + hp;
                        continue;
                    }
                    const uint32_t kb = kbl;
                    const uint32_t lidk = kb == 0 ? lid[0] : kb == 1 ? lid[1] : kb == 2 ? lid[2] : lid[3];
                    const uint32_t sbase = (lidk - nbase) * 2u * Bm;   // < 2^21 (k_large_scan_direct)
                    if (hp) {
                        const ulonglong2 w = stg[(kb * Bm + r) * 2u];
                        if ((w.x | w.y) == 0ull) cnt[kCntRedo] = 1u;   // a present cell whose products cancel
                        __builtin_amdgcn_raw_buffer_store_b32(pos | r << 21, rmeta, (sbase + r) * 4u, 0, PVAC_DIR_STORE_AUX);
                    }
                    if (hm) {
                        const ulonglong2 w = stg[(kb * Bm + r) * 2u + 1u];
                        if ((w.x | w.y) == 0ull) cnt[kCntRedo] = 1u;
                        __builtin_amdgcn_raw_buffer_store_b32((pos + hp) | (Bm + r) << 21, rmeta, (sbase + Bm + r) * 4u, 0,
                                                              PVAC_DIR_STORE_AUX);
                    }
                }
                if (b0 + BS < nw) __syncthreads();   // the next round rewrites obase / oidx / omk
            }
            if (ptab_ok) __syncthreads();   // every position in the table
            DSTAMP(5);
#pragma unroll
            for (uint32_t k = 0; k < kLaMaxLB; ++k) {   // the weights of every cell, coalesced
                if (k >= neB) break;
                const uint32_t sbase = (lid[k] - nbase) * 2u * Bm;
                for (uint32_t c = tid; c < 2u * Bm; c += BS) {
                    const uint32_t ch = c >= Bm ? 1u : 0u, r = c - ch * Bm;
                    const ulonglong2 w = stg[(k * Bm + r) * 2u + ch];
                    const uint32_t bo = (sbase + c) * 8u;
                    if (ptab_ok) {   // every cell is a key (the image is dense)
                        if ((w.x | w.y) == 0ull) cnt[kCntRedo] = 1u;   // a present cell whose products cancel
                        __builtin_amdgcn_raw_buffer_store_b32(ptab[k * 2u * Bm + c] | c << 21, rmeta, (sbase + c) * 4u, 0,
                                                              PVAC_DIR_STORE_AUX);
                    }
                    __builtin_amdgcn_raw_buffer_store_b64(u2v{(uint32_t)w.x, (uint32_t)(w.x >> 32)}, rlo, bo, 0, PVAC_DIR_STORE_AUX);
                    __builtin_amdgcn_raw_buffer_store_b64(u2v{(uint32_t)w.y, (uint32_t)(w.y >> 32)}, rhi, bo, 0, PVAC_DIR_STORE_AUX);
                }
            }
            DSTAMP(8);
        }
        for (uint32_t b0 = 0; b0 < nw && !cimg; b0 += BS) {   // workgroup-uniform
            const uint32_t kq = b0 + tid;
            const bool lv = kq < nw;
            const uint32_t we = lv ? wle[lbase + kq] : 0u;
            const ulonglong2 mk = lv ? wlm[lbase + kq] : make_ulonglong2(0ull, 0ull);
            const uint32_t e = we & 0x1FFFFFu;
            const uint32_t oi = lv ? dir_edge_off(c8, wo, e) : 0u;
            const uint64_t mp = mk.x & ~(1ull << 63), mm = mk.y;   // bit 63: a shared bucket (such pairs are redone)
            uint32_t T;
            const uint32_t excl = wg_exclusive_scan<BS>((uint32_t)__popcll(mp) + (uint32_t)__popcll(mm), part, T);
            obase[tid] = oi - excl;
            oidx[tid] = we >> 21;
            oexc[tid] = excl;
            omk[tid] = make_ulonglong2(mp, mm);
            __syncthreads();
            DSTAMP(6);
            // key expansion, one wave per entry and one lane per B edge j: the range's keys in emit
            // order (j DESC, P before M at one j), so key (j, P) sits at the keys above j
            const uint32_t ne = min(nw - b0, (uint32_t)BS);
            for (uint32_t l = wave; l < ne; l += BS / 64) {   // wave-uniform
                const ulonglong2 m2 = omk[l];
                const uint32_t x0 = oexc[l];
                const uint32_t hp = (uint32_t)(m2.x >> lane) & 1u, hm = (uint32_t)(m2.y >> lane) & 1u;
                const uint32_t above = lane == 63u ? 0u
                                                   : (uint32_t)__popcll(m2.x >> (lane + 1u)) + (uint32_t)__popcll(m2.y >> (lane + 1u));
                if (hp) okey[x0 + above] = (uint16_t)(lane | l << 7);
                if (hm) okey[x0 + above + hp] = (uint16_t)(lane | 64u | l << 7);
            }
            __syncthreads();
            DSTAMP(7);
            for (uint32_t q = tid; q < T; q += BS) {
                const uint32_t v = okey[q];
                const uint32_t l = v >> 7, jj = v & 63u, ch = (v >> 6) & 1u;
                const uint32_t bj = bjt[jj];
                const uint32_t kb = (bj >> 12) & 15u;
                const uint32_t r = mod_small(oidx[l] + (bj & 0xFFFu), Bm);
                const ulonglong2 w = stg[(kb * Bm + r) * 2u + ch];
                if ((w.x | w.y) == 0ull) cnt[kCntRedo] = 1u;   // a present cell whose products cancel
                const uint32_t lidk = kb == 0 ? lid[0] : kb == 1 ? lid[1] : kb == 2 ? lid[2] : lid[3];
                const uint32_t pos = obase[l] + q;
                const uint64_t mv = make_meta(lidk, r, ch);
                const uint32_t bo = pos * 8u;   // < 2^31: the host caps a direct pair at 2^21 A edges
                __builtin_amdgcn_raw_buffer_store_b64(u2v{(uint32_t)mv, (uint32_t)(mv >> 32)}, rmeta, bo, 0, PVAC_DIR_STORE_AUX);
                __builtin_amdgcn_raw_buffer_store_b64(u2v{(uint32_t)w.x, (uint32_t)(w.x >> 32)}, rlo, bo, 0, PVAC_DIR_STORE_AUX);
                __builtin_amdgcn_raw_buffer_store_b64(u2v{(uint32_t)w.y, (uint32_t)(w.y >> 32)}, rhi, bo, 0, PVAC_DIR_STORE_AUX);
                if (g.salt_pos) g.salt_pos[ceo + pos] = pos;
            }
            if (b0 + BS < nw) __syncthreads();   // the next round rewrites okey / obase
        }
        __syncthreads();   // the next A layer's staging overwrites dig and stg
        DSTAMP(3);
        la = lx;
        a_start = late(st_nx);
        a_n = late(n_nx);
        a_nw = late(nw_nx);
    }
#ifdef PVAC_DIR_STAMPS
    if (tid == 0) {
        for (int p = 0; p < 4; ++p) atomicAdd(&g_dir_stamps[p], st_acc[p]);
        for (int p = 4; p < 9; ++p) atomicAdd(&g_dir_stamps[12 + p], st_acc[p]);   // writer parts: [16, 21)
        atomicAdd(&g_dir_stamps[4], (unsigned long long)(i1 - i0));
        atomicAdd(&g_dir_stamps[5], 1ull);
    }
#endif
}

// the column-mode tasks k_large_products_la deferred: kDeferWG workgroups per pair walk its list
constexpr uint32_t kDeferWG = 4;
template <int BS>
__global__ __launch_bounds__(BS) void k_large_products_defer(mul_large_args g) {
    extern __shared__ __attribute__((aligned(16))) uint8_t plds[];
    const large_desc& d = g.desc[g.sel[blockIdx.y]];
    if (d.direct) return;
    uint32_t* S = g.scratch;
    const uint32_t* cnt = S + d.o_cnt;
    if (cnt[2]) return;
    const uint32_t nq = cnt[7];
    for (uint32_t q = blockIdx.x; q < nq; q += kDeferWG) {
        const uint32_t v = S[d.o_defer + q];
        run_task<BS, false>(g, d, S[d.o_neA + (v >> 16)], S[d.o_neB + (v & 0xFFFFu)], plds);
    }
}

// ---------------------------------------------------------------- compact_layers + layer records
// One workgroup per pair (encrypt.hpp:73-104): keep = product layers with emitted edges, plus
// transitive PROD parents; remap by exclusive count; write the kept records (product-layer
// ztags computed here, only for kept layers) and leave the remap in scratch for the writer.
__device__ __forceinline__ void layer_parents(const mul_large_args& g, uint64_t alo, uint64_t blo, uint32_t LA,
                                              uint32_t LB, uint32_t l, uint32_t& rule, uint32_t& pa, uint32_t& pb) {
    const uint32_t base = LA + LB;
    if (l < LA) {
        const pvac_layer& x = g.A.layers[alo + l];
        rule = x.rule; pa = x.pa; pb = x.pb;
    } else if (l < base) {
        const pvac_layer& x = g.B.layers[blo + (l - LA)];
        rule = x.rule; pa = x.pa + LA; pb = x.pb + LA;
    } else {
        rule = 1; pa = (l - base) / LB; pb = LA + (l - base) % LB;
    }
}

__global__ __launch_bounds__(kLBig) void k_large_layers(mul_large_args g) {
    extern __shared__ __attribute__((aligned(16))) uint32_t keep[];   // [Lc]
    __shared__ uint32_t changed;
    __shared__ uint32_t part[kLBig / 64];
    const large_desc& d = g.desc[blockIdx.x];
    uint32_t* S = g.scratch;
    if (S[d.o_cnt + 2]) return;
    // direct pairs: their own pass before their products (redone pairs: none); the others after
    if (g.layers_direct ? !(d.direct && S[d.o_cnt + kCntDirect]) : d.direct != 0) return;
    const uint64_t pr = d.pair;
    const uint32_t LA = d.LA, LB = d.LB, Lc = (uint32_t)d.Lc, base = LA + LB;
    const uint64_t alo = g.A.l_off[pr], blo = g.B.l_off[pr], clo = g.C.l_off[pr];
    uint32_t* used = S + d.o_used;
    const int tid = threadIdx.x;
    if (d.iblk && S[d.o_cnt + kCntIFail])   // k_large_rank marks this pair's leaders next
        for (uint64_t w = tid; w < 2 * d.nblk; w += kLBig) S[d.o_bmask + w] = 0;
    for (uint32_t l = tid; l < Lc; l += kLBig) keep[l] = l >= base ? (used[l] != 0) : 0u;
    for (;;) {
        __syncthreads();
        if (tid == 0) changed = 0;
        __syncthreads();
        for (uint32_t l = tid; l < Lc; l += kLBig) {
            if (!keep[l]) continue;
            uint32_t rule, pa, pb;
            layer_parents(g, alo, blo, LA, LB, l, rule, pa, pb);
            if (rule != 1) continue;
            if (pa < Lc && !keep[pa]) { keep[pa] = 1; changed = 1; }
            if (pb < Lc && !keep[pb]) { keep[pb] = 1; changed = 1; }
        }
        __syncthreads();
        if (!changed) break;
    }
    // remap = exclusive count of kept layers (chunked block scan)
    const uint32_t per = (Lc + kLBig - 1) / kLBig;
    uint32_t local = 0;
    for (uint32_t l = tid * per; l < (tid + 1) * per && l < Lc; ++l) local += keep[l];
    uint32_t kept;
    uint32_t run = wg_exclusive_scan<kLBig>(local, part, kept);
    for (uint32_t l = tid * per; l < (tid + 1) * per && l < Lc; ++l) {
        const uint32_t k = keep[l];
        keep[l] = k ? run : kInf;
        run += k;
    }
    __syncthreads();
    const bool identity = kept == Lc;
    for (uint32_t l = tid; l < Lc; l += kLBig) {
        const uint32_t to = keep[l];
        used[l] = to;   // remap for the edge writer
        if (to == kInf) continue;
        pvac_layer y;
        if (l < LA) {
            y = g.A.layers[alo + l];
        } else if (l < base) {
            y = g.B.layers[blo + (l - LA)];
            if (y.rule == 1) { y.pa += LA; y.pb += LA; }
        } else {
            const uint32_t lp = l - base;
            const uint64_t slot = clo + l;
            y.rule = 1; y.pad = 0;
            y.pa = lp / LB; y.pb = LA + lp % LB;
            y.nonce_lo = g.nonces[2 * slot];
            y.nonce_hi = g.nonces[2 * slot + 1];
            y.ztag = layer_ztag(g.canon_tag, y.nonce_lo, y.nonce_hi);
        }
        if (!identity && y.rule == 1) {
            y.pa = y.pa < Lc ? keep[y.pa] : kInf;
            y.pb = y.pb < Lc ? keep[y.pb] : kInf;
        }
        g.C.layers[clo + to] = y;
    }
    if (tid == 0) g.C.l_cnt[pr] = kept;
}

// ---------------------------------------------------------------- bucket chains
__global__ __launch_bounds__(kLB) void k_large_link(mul_large_args g) {
    const large_desc& d = g.desc[blockIdx.y];
    if (d.direct) return;
    uint32_t* S = g.scratch;
    if (S[d.o_cnt + 2]) return;
    const uint32_t Bm = g.Bm;
    const uint32_t* tkey = S + d.o_tkey;
    uint32_t* info = S + d.o_info;
    uint32_t* nxt = S + d.o_nxt;
    unsigned long long* hkey = (unsigned long long*)w64(S, d.o_hkey);
    uint32_t* hhead = S + d.o_hhead;
    const uint64_t hmask = (1ull << d.hbits) - 1;
    if (d.g_head != kNoGrp) return;   // static bucket groups: no per-pair chains
    for (uint64_t s = (uint64_t)blockIdx.x * kLB + threadIdx.x; s < d.S; s += (uint64_t)gridDim.x * kLB) {
        if (tkey[s] == kInf) continue;
        const uint64_t lp = s / Bm, r = s - lp * Bm;
        const uint64_t key = (lp << 32) | r;
        const uint64_t b = fmod64(key * kGolden, d.nbm);          // std::hash -> bucket
        uint64_t h = ((b + 1) * kGolden) >> (64 - d.hbits);
        for (;;) {
            const unsigned long long prev = atomicCAS(&hkey[h], 0ull, (unsigned long long)(b + 1));
            if (prev == 0ull || prev == b + 1) break;
            h = (h + 1) & hmask;
        }
        nxt[s] = atomicExch(&hhead[h], (uint32_t)(s + 1));
        info[s] = (info[s] & 3u) | ((uint32_t)h << 2);
    }
}

__global__ __launch_bounds__(kLB) void k_large_rank(mul_large_args g) {
    const large_desc& d = g.desc[blockIdx.y];
    if (d.direct) return;
    uint32_t* S = g.scratch;
    if (S[d.o_cnt + 2]) return;
    const uint32_t* tkey = S + d.o_tkey;
    const uint32_t* info = S + d.o_info;
    const uint32_t* nxt = S + d.o_nxt;
    const uint32_t* hhead = S + d.o_hhead;
    uint32_t* tb = S + d.o_tb;
    uint32_t* within = S + d.o_within;
    uint32_t* etot = S + d.o_etot;
    unsigned long long* bpack = (unsigned long long*)w64(S, d.o_bmask);
    const bool stat = d.g_head != kNoGrp;
    const uint32_t* ghead = g.grp + (stat ? d.g_head : 0);
    const uint32_t* gnext = g.grp + (stat ? d.g_next : 0);
    // iblk: bucket-sharing keys move their edges to their leader's A edge count; a pair that fell
    // back marks blocks here, lone leaders included (products did not)
    const bool fb = d.iblk && S[d.o_cnt + kCntIFail];
    const bool ib = d.iblk && !fb;
    if (ib && !S[d.o_cnt + kCntIShared]) return;   // every key alone in its bucket: nothing to rank
    uint32_t* icnt = S + d.o_icnt;
    const uint64_t m = d.nb_m;
    for (uint64_t s = (uint64_t)blockIdx.x * kLB + threadIdx.x; s < d.S; s += (uint64_t)gridDim.x * kLB) {
        // static groups: a key alone in its bucket (the common case) was counted by `products`
        // and `order` takes t_b = its own time, within = 0
        const uint32_t q0 = stat ? ghead[s] : 1u;
        if (!q0 && fb) {
            if (iblk_dead(S, d, s, g.Bm)) continue;
            const uint32_t t = tkey[s];
            const uint32_t E = t == kInf ? 0u : __popc(info[s] & 3u);
            if (E) leader_mark(bpack, t, E);
            continue;
        }
        if (!q0 || iblk_dead(S, d, s, g.Bm)) continue;
        const uint32_t t = tkey[s];
        if (t == kInf) continue;
        uint32_t tmin = t, w = 0, E = 0;
        if (stat) {
            // the bucket's slots are a static property of (bucket count, B): walk them, keep the
            // ones present in this pair
            uint32_t q = q0;
            while (q) {
                const uint32_t s2 = q - 1;
                q = gnext[s2];
                if (s2 >= d.S || iblk_dead(S, d, s2, g.Bm)) continue;
                const uint32_t t2 = tkey[s2];
                if (t2 == kInf) continue;
                const uint32_t e2 = __popc(info[s2] & 3u);
                tmin = t2 < tmin ? t2 : tmin;
                w += t2 > t ? e2 : 0u;
                E += e2;
            }
        } else {
            uint32_t q = hhead[info[s] >> 2];
            while (q) {
                const uint32_t s2 = q - 1;
                const uint32_t t2 = tkey[s2];
                const uint32_t e2 = __popc(info[s2] & 3u);
                tmin = t2 < tmin ? t2 : tmin;
                w += t2 > t ? e2 : 0u;
                E += e2;
                q = nxt[s2];
            }
        }
        tb[s] = tmin;
        within[s] = w;
        if (tmin == t) {
            etot[s] = E;
            if (E && !ib) leader_mark(bpack, t, E);   // one atomic per leader
        } else if (ib) {
            // products counted this key's edges in its own A edge's range: move them to the leader's
            const uint32_t e = __popc(info[s] & 3u);
            uint32_t j;
            const uint32_t is = div_small(t, d.nB, m, j), il = div_small(tmin, d.nB, m, j);
            if (e && is != il) {
                atomicSub(&icnt[is], e);
                atomicAdd(&icnt[il], e);
            }
        }
    }
}

// One workgroup per pair: suffix exclusive scan of the block counts (emit offsets), the
// total, the guard_budget decision and, for canonical pairs, canonical positions.
__global__ __launch_bounds__(kLBig) void k_large_scan(mul_large_args g) {
    __shared__ uint32_t part[kLBig / 64];
    const large_desc& d = g.desc[blockIdx.x];
    if (d.direct) return;   // k_large_scan_direct
    uint32_t* S = g.scratch;
    uint32_t* cnt = S + d.o_cnt;
    if (cnt[2]) return;
    const int tid = threadIdx.x;
    unsigned long long* bpack = (unsigned long long*)w64(S, d.o_bmask);
    const uint32_t nblk = (uint32_t)d.nblk;
    uint32_t total = 0;
    if (d.iblk && !cnt[kCntIFail]) {
        // per-A-edge counts -> exclusive suffix offsets in place (A edge nA-1 first), as below
        uint32_t* icnt = S + d.o_icnt;
        const uint32_t nA = d.nA;
        for (uint32_t base = 0; base < nA; base += 4u * kLBig) {
            const uint32_t r0 = base + 4u * (uint32_t)tid;
            uint32_t v[4];
            uint32_t local = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t r = r0 + (uint32_t)k;
                v[k] = r < nA ? icnt[nA - 1 - r] : 0u;
                local += v[k];
            }
            uint32_t tot;
            uint32_t run = total + wg_exclusive_scan<kLBig>(local, part, tot);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t r = r0 + (uint32_t)k;
                if (r < nA) icnt[nA - 1 - r] = run;
                run += v[k];
            }
            total += tot;
        }
    }
    // reversed block index r (block nblk-1-r) in rounds of 4 kLBig: thread t takes r = base + 4t .. 4t+3
    // (adjacent threads, adjacent words: coalesced), one workgroup scan per round
    for (uint32_t base = 0; base < (d.iblk && !cnt[kCntIFail] ? 0u : nblk); base += 4u * kLBig) {
        const uint32_t r0 = base + 4u * (uint32_t)tid;
        unsigned long long v[4];
        uint32_t local = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t r = r0 + (uint32_t)k;
            v[k] = r < nblk ? bpack[nblk - 1 - r] : 0ull;
            local += (uint32_t)(v[k] >> 32);
        }
        uint32_t tot;
        uint32_t run = total + wg_exclusive_scan<kLBig>(local, part, tot);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t r = r0 + (uint32_t)k;
            if (r < nblk) bpack[nblk - 1 - r] = ((unsigned long long)run << 32) | (v[k] & 0xFFFFFFFFull);
            run += (uint32_t)(v[k] >> 32);
        }
        total += tot;
    }
    const bool canonical = (g.flags & PVAC_MUL_ORDER_CANONICAL) != 0 || total > g.edge_budget;
    if (tid == 0) {
        cnt[3] = total;
        cnt[4] = canonical;
        g.C.e_cnt[d.pair] = total;
        g.pair_status[d.pair] = canonical ? 1 : 0;
    }
    if (!canonical) return;
    const uint32_t* tkey = S + d.o_tkey;
    const uint32_t* info = S + d.o_info;
    uint32_t* cpos = S + d.o_cpos;
    uint32_t carry = 0;
    for (uint64_t s0 = 0; s0 < d.S; s0 += kLBig) {
        const uint64_t s = s0 + tid;
        const uint32_t v = (s < d.S && !iblk_dead(S, d, s, g.Bm) && tkey[s] != kInf) ? (uint32_t)__popc(info[s] & 3u) : 0u;
        uint32_t tot;
        const uint32_t ex = wg_exclusive_scan<kLBig>(v, part, tot);
        if (s < d.S) cpos[s] = carry + ex;
        carry += tot;
    }
}

__global__ __launch_bounds__(kLB) void k_large_order(mul_large_args g) {
    const large_desc& d = g.desc[blockIdx.y];
    if (d.direct) return;
    uint32_t* S = g.scratch;
    const uint32_t* cnt = S + d.o_cnt;
    if (cnt[2]) return;
    const bool canonical = cnt[4] != 0;
    const uint32_t Bm = g.Bm, LB = d.LB, nB = d.nB;
    const uint64_t pr = d.pair;
    const uint64_t aeo = g.A.e_off[pr], beo = g.B.e_off[pr];
    const uint32_t* tkey = S + d.o_tkey;
    const uint32_t* info = S + d.o_info;
    const uint32_t* tb = S + d.o_tb;
    const uint32_t* within = S + d.o_within;
    const uint32_t* etot = S + d.o_etot;
    const unsigned long long* bpack = (const unsigned long long*)w64(S, d.o_bmask);
    const uint32_t* cpos = S + d.o_cpos;
    uint32_t* order = S + d.o_order;
    uint32_t* hpos = S + d.o_hpos;
    const uint32_t* ghead = group_heads(g, d);
    const bool ib = d.iblk && !cnt[kCntIFail];
    if (ib && !canonical && !cnt[kCntIShared]) return;   // k_large_write_ranges
    const uint32_t* icnt = S + d.o_icnt;
    const ulonglong2* imask = (const ulonglong2*)(S + d.o_imask);
    const uint64_t m = d.nb_m;
    // iblk: edges emitted before the emit time (i, j) inside A edge i's range, by probing its later
    // times (i, j'): the key slot of (i, j') is known from the two edges, and (i, j') is an emit time
    // when it is that key's first-insert time and the key is alone in its bucket or leads it
    auto probe_rank = [&](uint32_t i, uint32_t j) {
        const uint64_t ma = g.A.meta[aeo + i];
        const uint32_t sa = meta_layer(ma) * LB, ia = meta_idx(ma);
        uint32_t w = 0;
        for (uint32_t j2 = j + 1; j2 < nB; ++j2) {
            const uint64_t mb = g.B.meta[beo + j2];
            const uint64_t s2 = (uint64_t)(sa + meta_layer(mb)) * Bm + mod_small(ia + meta_idx(mb), Bm);
            const uint32_t t2 = i * nB + j2;
            if (tkey[s2] != t2) continue;
            if (ghead[s2] == 0u) w += __popc(info[s2] & 3u);
            else if (tb[s2] == t2) w += etot[s2];
        }
        return w;
    };
    for (uint64_t s = (uint64_t)blockIdx.x * kLB + threadIdx.x; s < d.S; s += (uint64_t)gridDim.x * kLB) {
        if (iblk_dead(S, d, s, Bm)) continue;
        const uint32_t ts = tkey[s];
        if (ts == kInf) continue;
        const uint32_t inf = info[s];
        const uint32_t eb = inf & 3u;
        if (!eb) continue;
        const bool lone = ghead && ghead[s] == 0u;   // its own bucket leader, nothing before it
        if (ib) {
            uint32_t hp, j0;
            const uint32_t i0 = lone ? div_small(ts, nB, m, j0) : 0u;
            const ulonglong2 mk = lone ? imask[i0] : make_ulonglong2(0ull, 0ull);
            if (lone && !(mk.x >> 63)) {   // a range without shared keys: rank from its masks
                const unsigned long long above = (~0ull << (j0 + 1)) & ~(1ull << 63);
                hp = icnt[i0] + (uint32_t)__popcll(mk.x & above) + (uint32_t)__popcll(mk.y & above);
            } else {
                const uint32_t tu = lone ? ts : tb[s];
                uint32_t j;
                const uint32_t i = div_small(tu, nB, m, j);
                hp = icnt[i] + probe_rank(i, j) + (lone ? 0u : within[s]);
            }
            const uint32_t p = canonical ? cpos[s] : hp;
            const uint32_t s32 = (uint32_t)s;
            if (eb & 1u) {
                order[p] = s32 << 1;
                if (canonical) hpos[p] = hp;
            }
            if (eb & 2u) {
                const uint32_t o = eb & 1u;
                order[p + o] = (s32 << 1) | 1u;
                if (canonical) hpos[p + o] = hp + o;
            }
            continue;
        }
        const uint32_t t = lone ? ts : tb[s], blk = t >> 4, bit = t & 15u;
        const unsigned long long v = bpack[blk];
        // edge codes of the leaders later in this block (2 bits per time): 1 and 2 are their edge
        // counts; 3 (buckets of 3+ edges) is resolved from the leader's slot, found from its
        // (i, j) = (t / |B.E|, t % |B.E|)
        const uint64_t codes = (v & 0xFFFFFFFFull) >> (2u * bit + 2u);
        const uint64_t esc = codes & (codes >> 1) & 0x5555555555555555ull;
        uint32_t hp = (uint32_t)(v >> 32) + (lone ? 0u : within[s]) + (uint32_t)__popcll(codes & 0x5555555555555555ull) +
                      2u * (uint32_t)__popcll(codes & 0xAAAAAAAAAAAAAAAAull) - 3u * (uint32_t)__popcll(esc);
        uint64_t m = esc;
        while (m) {
            const uint32_t b2 = ((uint32_t)__ffsll((long long)m) - 1u) / 2u + bit + 1u;
            m &= m - 1ull;
            const uint32_t t2 = (blk << 4) | b2;
            const uint32_t i2 = t2 / nB, j2 = t2 - i2 * nB;
            const uint64_t ma = g.A.meta[aeo + i2], mb = g.B.meta[beo + j2];
            const uint64_t s2 = (uint64_t)(meta_layer(ma) * LB + meta_layer(mb)) * Bm +
                                mod_small(meta_idx(ma) + meta_idx(mb), Bm);
            hp += etot[s2];
        }
        const uint32_t p = canonical ? cpos[s] : hp;
        const uint32_t s32 = (uint32_t)s;
        if (eb & 1u) {
            order[p] = s32 << 1;
            if (canonical) hpos[p] = hp;
        }
        if (eb & 2u) {
            const uint32_t o = eb & 1u;
            order[p + o] = (s32 << 1) | 1u;
            if (canonical) hpos[p + o] = hp + o;
        }
    }
}

__global__ __launch_bounds__(kLB) void k_large_write(mul_large_args g) {
    const large_desc& d = g.desc[blockIdx.y];
    if (d.direct) return;
    uint32_t* S = g.scratch;
    const uint32_t* cnt = S + d.o_cnt;
    if (cnt[2]) return;
    const uint32_t total = cnt[3];
    const bool canonical = cnt[4] != 0;
    if (d.iblk && !cnt[kCntIFail] && !canonical && !cnt[kCntIShared]) return;   // k_large_write_ranges
    const uint32_t Bm = g.Bm, base = d.LA + d.LB;
    const uint64_t ceo = g.C.e_off[d.pair];
    const uint32_t* order = S + d.o_order;
    const uint32_t* hpos = S + d.o_hpos;
    const uint32_t* remap = S + d.o_used;
    const ulonglong2* sums = (const ulonglong2*)(S + d.o_sums);
    for (uint32_t p = blockIdx.x * kLB + threadIdx.x; p < total; p += gridDim.x * kLB) {
        const uint32_t e = order[p];
        const uint32_t s = e >> 1, ch = e & 1u;
        const uint32_t lp = s / Bm, r = s - lp * Bm;
        const ulonglong2 w = sums[2 * (uint64_t)s + ch];
        g.C.meta[ceo + p] = make_meta(remap[base + lp], r, ch);
        g.C.w_lo[ceo + p] = w.x;
        g.C.w_hi[ceo + p] = w.y;
        if (g.salt_pos) g.salt_pos[ceo + p] = canonical ? hpos[p] : p;
    }
}

// iblk pairs without shared buckets, hash order: the edges are written range by range. A edge
// i's keys take positions [off(i), off(i) + cnt(i)), and off decreases with i, so ranges in DESCENDING
// i are consecutive in the output. A wave takes 64 ranges (lane l: i = nA - 1 - (64 c + l)), scans
// their edge counts and writes its positions coalesced: position q of the chunk finds its lane
// (binary search over the scanned counts) and its key inside the range (j DESC; P before M: the
// k-th edge sits below the highest bit x with popc(P >> x) + popc(M >> x) <= k), the key slot from
// (A edge i, B edge j), and gathers its sum. No order array, no per-slot pass (k_large_order).
__global__ __launch_bounds__(kLB) void k_large_write_ranges(mul_large_args g) {
    __shared__ uint32_t bjt[64];   // B edge j: idx | layer << 16
    const large_desc& d = g.desc[blockIdx.y];
    if (d.direct) return;
    uint32_t* S = g.scratch;
    const uint32_t* cnt = S + d.o_cnt;
    if (cnt[2] || !d.iblk || cnt[kCntIFail] || cnt[4] || cnt[kCntIShared]) return;
    const uint32_t Bm = g.Bm, LB = d.LB, nA = d.nA, nB = d.nB, base = d.LA + d.LB;
    const uint64_t pr = d.pair;
    const uint64_t aeo = g.A.e_off[pr], beo = g.B.e_off[pr], ceo = g.C.e_off[pr];
    if (threadIdx.x < nB) {
        const uint64_t mb = g.B.meta[beo + threadIdx.x];
        bjt[threadIdx.x] = meta_idx(mb) | meta_layer(mb) << 16;
    }
    __syncthreads();
    const uint32_t* off = S + d.o_icnt;
    const ulonglong2* imask = (const ulonglong2*)(S + d.o_imask);
    const uint32_t* remap = S + d.o_used;
    const ulonglong2* sums = (const ulonglong2*)(S + d.o_sums);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nch = (nA + 63u) >> 6;
    for (uint32_t c = blockIdx.x * (kLB / 64) + (threadIdx.x >> 6); c < nch; c += gridDim.x * (kLB / 64)) {
        const uint32_t r = c * 64u + lane;
        const bool live = r < nA;
        const uint32_t i = live ? nA - 1u - r : 0u;
        // the range's edge count from the offsets (off[i - 1] - off[i], the total for i = 0); the
        // masks and the A edge are read only for ranges that hold keys
        const uint32_t oi = live ? off[i] : 0u;
        const uint32_t E = live ? (i ? off[i - 1] : cnt[3]) - oi : 0u;
        const ulonglong2 mk = E ? imask[i] : make_ulonglong2(0ull, 0ull);
        const uint32_t o0 = off[nA - 1u - c * 64u];   // the chunk's first position (lane 0's range)
        const uint64_t ma = E ? g.A.meta[aeo + i] : 0ull;
        const uint32_t la_idx = meta_idx(ma) | meta_layer(ma) << 16;
        const uint32_t incl = wave_incl_scan_u32(E);
        const uint32_t T = __builtin_amdgcn_readlane(incl, 63);
        // position q of the chunk -> key slot s and channel; every lane takes part in the bpermutes
        auto resolve = [&](uint32_t q, uint64_t& s, uint32_t& ch, uint32_t& lp, uint32_t& rr) {
            // lane l of the range holding q: the first lane whose inclusive count exceeds q
            uint32_t l = 0;
#pragma unroll
            for (uint32_t b = 32; b; b >>= 1) {
                const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((l + b - 1u) << 2), (int)incl);
                if (v <= q) l += b;
            }
            l = min(l, 63u);
            const int bl = (int)(l << 2);
            const uint32_t il = (uint32_t)__builtin_amdgcn_ds_bpermute(bl, (int)incl) -
                                (uint32_t)__builtin_amdgcn_ds_bpermute(bl, (int)E);
            const uint64_t mp = (uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(bl, (int)(uint32_t)mk.x) |
                                (uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(bl, (int)(uint32_t)(mk.x >> 32)) << 32;
            const uint64_t mm = (uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(bl, (int)(uint32_t)mk.y) |
                                (uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(bl, (int)(uint32_t)(mk.y >> 32)) << 32;
            const uint32_t ai = (uint32_t)__builtin_amdgcn_ds_bpermute(bl, (int)la_idx);
            const uint32_t k = q - il;   // edge k of the range (q < T)
            // edges of keys at bits >= y: A(y) = popc(mp >> y) + popc(mm >> y), non-increasing; the
            // key holding edge k is the largest j with A(j) > k
            uint32_t j = 0;
#pragma unroll
            for (uint32_t b = 32; b; b >>= 1) {
                const uint32_t y = j + b;
                if ((uint32_t)__popcll(mp >> y) + (uint32_t)__popcll(mm >> y) > k) j = y;
            }
            const uint32_t fa = j == 63u ? 0u : (uint32_t)__popcll(mp >> (j + 1u)) + (uint32_t)__popcll(mm >> (j + 1u));
            const uint32_t hasP = (uint32_t)(mp >> j) & 1u;
            ch = (k - fa == 0u && hasP) ? 0u : 1u;   // a key emits P before M
            const uint32_t bj = bjt[j];
            lp = (ai >> 16) * LB + (bj >> 16);
            rr = mod_small((ai & 0xFFFFu) + (bj & 0xFFFFu), Bm);
            s = (uint64_t)lp * Bm + rr;
        };
        // two positions per lane and round: both gathers in flight before the stores
        for (uint32_t q0 = 0; q0 < T; q0 += 128u) {   // wave-uniform
            uint64_t s[2];
            uint32_t ch[2], lp[2], rr[2];
            ulonglong2 w[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint32_t q = q0 + 64u * (uint32_t)u + lane;
                resolve(min(q, T - 1u), s[u], ch[u], lp[u], rr[u]);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) w[u] = sums[2 * s[u] + ch[u]];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint32_t q = q0 + 64u * (uint32_t)u + lane;
                if (q >= T) break;
                const uint64_t p = ceo + o0 + q;
                g.C.meta[p] = make_meta(remap[base + lp[u]], rr[u], ch[u]);
                g.C.w_lo[p] = w[u].x;
                g.C.w_hi[p] = w[u].y;
                if (g.salt_pos) g.salt_pos[p] = o0 + q;
            }
        }
    }
}

// ---------------------------------------------------------------- static bucket groups
__global__ __launch_bounds__(kLB) void k_grp_insert(fastmod64 nbm, uint32_t Bm, uint64_t S, uint32_t hbits,
                                                    uint32_t* head, uint32_t* next, unsigned long long* tkeyb,
                                                    uint32_t* thead) {
    const uint64_t hmask = (1ull << hbits) - 1;
    for (uint64_t s = (uint64_t)blockIdx.x * kLB + threadIdx.x; s < S; s += (uint64_t)gridDim.x * kLB) {
        const uint64_t lp = s / Bm, r = s - lp * Bm;
        const uint64_t b = fmod64(((lp << 32) | r) * kGolden, nbm);   // std::hash -> bucket
        uint64_t h = ((b + 1) * kGolden) >> (64 - hbits);
        for (;;) {
            const unsigned long long prev = atomicCAS(&tkeyb[h], 0ull, (unsigned long long)(b + 1));
            if (prev == 0ull || prev == b + 1) break;
            h = (h + 1) & hmask;
        }
        next[s] = atomicExch(&thead[h], (uint32_t)(s + 1));
        head[s] = (uint32_t)h;
    }
}

__global__ __launch_bounds__(kLB) void k_grp_finish(uint64_t S, uint32_t* head, const uint32_t* next,
                                                    const uint32_t* thead) {
    for (uint64_t s = (uint64_t)blockIdx.x * kLB + threadIdx.x; s < S; s += (uint64_t)gridDim.x * kLB) {
        const uint32_t h0 = thead[head[s]];
        head[s] = (h0 == (uint32_t)(s + 1) && next[s] == 0u) ? 0u : h0;   // 0: alone in its bucket
    }
}

unsigned grid_x(uint64_t work, uint64_t per_block, uint64_t cap) {
    uint64_t b = (work + per_block - 1) / per_block;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (unsigned)b;
}

}  // namespace

hipError_t launch_grp_build(fastmod64 nbm, uint32_t Bm, uint64_t S, uint32_t hbits, uint32_t* head, uint32_t* next,
                            unsigned long long* tmp_key, uint32_t* tmp_head, hipStream_t st) {
    if (!S) return hipSuccess;
    const unsigned gs = grid_x(S, kLB * 2, 4096);
    hipLaunchKernelGGL(k_grp_insert, dim3(gs), dim3(kLB), 0, st, nbm, Bm, S, hbits, head, next, tmp_key, tmp_head);
    hipLaunchKernelGGL(k_grp_finish, dim3(gs), dim3(kLB), 0, st, S, head, (const uint32_t*)next,
                       (const uint32_t*)tmp_head);
    return hipGetLastError();
}

uint32_t large_direct_lds_bytes(uint32_t Bm, uint32_t nbl) { return dir_lds_bytes(Bm, nbl); }

// ---------------------------------------------------------------- dense chain images -> records
// (k_large_products_direct's image writer; see mul_large_args::A_img) Listed pair y (pairs[y], its
// edges at tmp + 3 pairs[n + y]): the image is copied out, then every slot's edge is written back at
// its hash-order position as (meta, w_lo, w_hi); the flags are cleared last. A launch covers the
// listed pairs y = y0 + blockIdx.y (grid y is capped, so a long list takes several launches).
__global__ __launch_bounds__(256) void k_img_copy(pvac_ct_batch A, const uint32_t* img, const uint64_t* pairs, uint32_t n,
                                                  uint32_t y0, uint64_t* tmp) {
    const uint32_t y = y0 + blockIdx.y;
    const uint64_t pr = pairs[y];
    if (!img[pr]) return;
    const uint64_t eo = A.e_off[pr], ne = A.e_cnt[pr];
    uint64_t* t = tmp + 3u * pairs[n + y];
    const uint32_t* ids = (const uint32_t*)(A.meta + eo);
    for (uint64_t k = (uint64_t)blockIdx.x * 256u + threadIdx.x; k < ne; k += (uint64_t)gridDim.x * 256u) {
        t[3u * k] = ids[k];
        t[3u * k + 1u] = A.w_lo[eo + k];
        t[3u * k + 2u] = A.w_hi[eo + k];
    }
}
__global__ __launch_bounds__(256) void k_img_scatter(pvac_ct_batch A, const uint32_t* img, const uint64_t* pairs, uint32_t n,
                                                     uint32_t y0, const uint64_t* tmp, uint32_t Bm) {
    const uint32_t y = y0 + blockIdx.y;
    const uint64_t pr = pairs[y];
    if (!img[pr]) return;
    const uint64_t eo = A.e_off[pr], ne = A.e_cnt[pr];
    const uint64_t slab = 2u * Bm, first = A.l_cnt[pr] - ne / slab;   // the slabs are the last layers
    const uint64_t* t = tmp + 3u * pairs[n + y];
    for (uint64_t k = (uint64_t)blockIdx.x * 256u + threadIdx.x; k < ne; k += (uint64_t)gridDim.x * 256u) {
        const uint32_t id = (uint32_t)t[3u * k];
        const uint32_t pos = id & 0x1FFFFFu, cell = id >> 21;
        if (pos >= ne) continue;   // not an image slot (never written by the image writer)
        const uint32_t ch = cell >= Bm ? 1u : 0u;
        A.meta[eo + pos] = make_meta((uint32_t)(first + k / slab), cell - ch * Bm, ch);
        A.w_lo[eo + pos] = t[3u * k + 1u];
        A.w_hi[eo + pos] = t[3u * k + 2u];
    }
}
__global__ __launch_bounds__(64) void k_img_clear(uint32_t* img, const uint64_t* pairs, uint32_t n) {
    const uint32_t y = blockIdx.x * 64u + threadIdx.x;
    if (y < n) img[pairs[y]] = 0u;
}
hipError_t launch_image_to_records(const pvac_ct_batch& A, uint32_t* img, const uint64_t* pairs, uint32_t n_pairs,
                                   uint64_t* tmp, uint32_t Bm, uint32_t y_cap, hipStream_t st) {
    if (!n_pairs) return hipSuccess;
    y_cap = std::min<uint32_t>(std::max<uint32_t>(y_cap, 1u), 65535u);   // grid y limit (tests pass small caps)
    for (uint32_t y0 = 0; y0 < n_pairs; y0 += y_cap) {
        const uint32_t ny = std::min<uint32_t>(n_pairs - y0, y_cap);
        hipLaunchKernelGGL(k_img_copy, dim3(64, ny), dim3(256), 0, st, A, img, pairs, n_pairs, y0, tmp);
        hipLaunchKernelGGL(k_img_scatter, dim3(64, ny), dim3(256), 0, st, A, img, pairs, n_pairs, y0, tmp, Bm);
    }
    hipLaunchKernelGGL(k_img_clear, dim3((n_pairs + 63u) / 64u), dim3(64), 0, st, img, pairs, n_pairs);
    return hipGetLastError();
}


hipError_t launch_ct_mul_large(const mul_large_args& a, hipStream_t st) {
    if (!a.nl) return hipSuccess;
    if (a.Bm > kBmax || a.max_lay > kLargeLayersMax) return hipErrorInvalidValue;
    const unsigned nl = a.nl;
    const size_t plds = prod_lds_bytes(a.Bm);
    hipLaunchKernelGGL(k_large_init, dim3(grid_x(a.max_zero > a.max_S ? a.max_zero : a.max_S, kLB * 4, 4096), nl),
                       dim3(kLB), 0, st, a);
    hipLaunchKernelGGL(k_large_lists, dim3(nl), dim3(kLBig), (size_t)a.max_lay * 4, st, a);
#ifndef PVAC_LARGE_PRODUCTS_COL26
    if (a.any_direct && a.n_la && a.max_la_wg) {
        // direct pairs: presence counts, offsets, compact_layers, then products straight to C
        mul_large_args b = a;
        b.lds_task = cnt_lds_bytes(a.Bm);
        const dim3 grid((unsigned)a.max_la_wg, a.n_la);
        hipLaunchKernelGGL((k_large_count_la<kLPX>), grid, dim3(kLPX),
                           (size_t)b.lds_task + kLaMaxLB * kMxMaxSparse * 16u + kIblkBjtBytes + kLaMaxLB * 4u * a.Bm, st, b);
        hipLaunchKernelGGL(k_large_scan_direct, dim3(nl), dim3(kLBig), 0, st, b);
        b.layers_direct = 1;
        hipLaunchKernelGGL(k_large_layers, dim3(nl), dim3(kLBig), (size_t)a.max_lay * 4, st, b);
        hipLaunchKernelGGL((k_large_products_direct<kLPX>), grid, dim3(kLPX), (size_t)dir_lds_bytes(a.Bm, a.dir_lb), st, b);
        hipLaunchKernelGGL(k_large_direct_redo, dim3((nl + 63) / 64), dim3(64), 0, st, b);
        if (a.all_direct) return hipGetLastError();
    }
#endif
    // products: the matrix-core dense mode in 4-wave workgroups (A-layer-major for pairs with few B
    // layers, one task per workgroup for the rest). A/B builds with -DPVAC_LARGE_PRODUCTS_COL26 run
    // the column-accumulator kernel of round 2 for every pair instead (never the shipped library).
#ifdef PVAC_LARGE_PRODUCTS_COL26
    {
        mul_large_args b = a;
        b.n_la = 0;
        hipLaunchKernelGGL((k_large_products<kLP, false>), dim3((unsigned)a.max_tasks_all, nl), dim3(kLP), plds, st, b);
    }
#else
    {
        const size_t lx = std::max<size_t>(plds, mx_lds_bytes(a.Bm) + kMxSparseBytes);
        if (nl > a.n_la && a.max_tasks)
            hipLaunchKernelGGL((k_large_products<kLPX, true>), dim3((unsigned)a.max_tasks, nl - a.n_la), dim3(kLPX), lx, st, a);
        if (a.n_la && a.max_la_wg) {
            mul_large_args b = a;
            b.lds_task = mx_lds_bytes(a.Bm);   // the scatter mode (52 B per slot) fits below it
            hipLaunchKernelGGL((k_large_products_la<kLPX>), dim3((unsigned)a.max_la_wg, a.la_xcd ? (a.n_la + 7u) & ~7u : a.n_la),
                               dim3(kLPX),
                               (size_t)b.lds_task + kLaMaxLB * kMxSparseBytes + kIblkBjtBytes + kLaMaxLB * 4u * a.Bm, st, b);
            hipLaunchKernelGGL((k_large_products_defer<kLPX>), dim3(kDeferWG, a.n_la), dim3(kLPX), plds, st, a);
        }
    }
#endif
    hipLaunchKernelGGL(k_large_layers, dim3(nl), dim3(kLBig), (size_t)a.max_lay * 4, st, a);
    const unsigned gs = grid_x(a.max_S, kLB * 2, 4096);
    // a batch of iblk pairs runs rank / order / write only for the few that share buckets, need the
    // canonical order or fell back: 1/16 of the workgroups (grid-stride loops; an empty workgroup per
    // 512 slots cost 5 ms per sub-batch and kernel at cfg 4's depth 8)
    const unsigned sh = a.all_iblk ? 4u : 0u;
    const unsigned gsr = (gs + (1u << sh) - 1u) >> sh;
    if (a.any_dyn) hipLaunchKernelGGL(k_large_link, dim3(gs, nl), dim3(kLB), 0, st, a);
    hipLaunchKernelGGL(k_large_rank, dim3(gsr, nl), dim3(kLB), 0, st, a);
    hipLaunchKernelGGL(k_large_scan, dim3(nl), dim3(kLBig), 0, st, a);
    hipLaunchKernelGGL(k_large_order, dim3(gsr, nl), dim3(kLB), 0, st, a);
    const unsigned gw = grid_x(a.max_capE, kLB * 2, 4096);
    hipLaunchKernelGGL(k_large_write, dim3((gw + (1u << sh) - 1u) >> sh, nl), dim3(kLB), 0, st, a);
    if (a.max_nA) hipLaunchKernelGGL(k_large_write_ranges, dim3(grid_x(a.max_nA, kLB, 4096), nl), dim3(kLB), 0, st, a);
    return hipGetLastError();
}

}  // namespace pvhip
