// k_ct.hip — batched ciphertext plumbing: sizing plans, u64 scans, ct_add / ct_sub.
//
// ct_mul itself lives in k_mul_fresh.hip (LDS-resident fresh-shape pairs) and
// k_mul_large.hip (general pairs: chains, squares, dense layers).
#include <cstddef>

#include "common.hpp"

namespace pvhip {

namespace {

constexpr int kPlanBlock = 256;

// ---------------------------------------------------------------- plans
// wave64 butterfly reductions
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t o = __shfl_xor(v, d, 64);
        v = o > v ? o : v;
    }
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Block-wide reduction of per-thread statistics, then one global atomic per block per field:
// per-wave atomics on the same few addresses serialised at L2 (1.3 ms for 2^20 pairs).
template <int N>
__device__ __forceinline__ void block_reduce_stats(uint32_t (&v)[N], const bool (&is_sum)[N], uint32_t* lds) {
#pragma unroll
    for (int f = 0; f < N; ++f) v[f] = is_sum[f] ? wave_sum_u32(v[f]) : wave_max_u32(v[f]);
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int f = 0; f < N; ++f) lds[wave * N + f] = v[f];
    __syncthreads();
    if (threadIdx.x == 0)
        for (int w = 1; w < nw; ++w)
#pragma unroll
            for (int f = 0; f < N; ++f) {
                const uint32_t o = lds[w * N + f];
                v[f] = is_sum[f] ? v[f] + o : (o > v[f] ? o : v[f]);
            }
}

// atomicMax only when the block's value beats what is already there: the maxima of a uniform
// batch are reached by the first blocks, so the rest issue no atomic (thousands of same-address
// atomics serialise at one L2 channel). Skipping is exact: the stored maximum never decreases.
__device__ __forceinline__ void max_if_greater(unsigned int* p, uint32_t v) {
    if (v > __atomic_load_n(p, __ATOMIC_RELAXED)) atomicMax(p, v);
}

// one pair per thread up to 2^20 pairs (a second grid-stride round only beyond): the loop's loads
// are not overlapped across rounds
inline unsigned plan_grid(uint64_t n) {
    const uint64_t b = (n + kPlanBlock - 1) / kPlanBlock;
    return (unsigned)(b < 4096 ? b : 4096);
}
static_assert(offsetof(plan_stats, max_layers) == offsetof(plan_stats, max_keys) + 5 * sizeof(unsigned int),
              "k_plan_mul updates the six maxima as consecutive words");

// Classifies every pair (fresh-shape kernel or general path), writes per-pair output
// capacities (scanned in place afterwards) and the launch maxima of the fresh kernel.
// Grid-stride over pairs; one atomic per block per statistic.
__global__ __launch_bounds__(kPlanBlock) void k_plan_mul(pvac_ct_batch A, pvac_ct_batch B, pvac_ct_batch C,
                                                        uint8_t* pair_class, uint64_t* large_ids, plan_stats* stats,
                                                        const uint32_t* nb_table, uint32_t nb_len, uint32_t Bm) {
    __shared__ uint32_t red[(kPlanBlock / 64) * 6];
    uint32_t mk = 0, mp = 0, ma = 0, mb = 0, mbk = 0, ml = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kPlanBlock + threadIdx.x; i < A.n; i += (uint64_t)gridDim.x * kPlanBlock) {
        const uint64_t LA = A.l_cnt[i], LB = B.l_cnt[i], nA = A.e_cnt[i], nB = B.e_cnt[i];
        const uint64_t keys = LA * LB * Bm;
        const uint64_t prod = nA * nB;
        const uint64_t capL = LA + LB + LA * LB;
        const uint64_t capE = 2 * (prod < keys ? prod : keys);
        C.l_off[i] = capL;   // scanned in place afterwards
        C.e_off[i] = capE;
        if (C.l_cnt) C.l_cnt[i] = 0;   // exec's counts start from zero (no separate fill by the caller)
        if (C.e_cnt) C.e_cnt[i] = 0;
        const bool sm = keys <= kFreshKeysMax && prod <= kFreshProdMax && prod < nb_len && nA <= kFreshEdgesMax &&
                        nB <= kFreshEdgesMax && capL <= kFreshLayersMax &&
                        nb_table[prod < nb_len ? prod : 0] + prod + 3 <= 3 * keys;   // chains + key sums fit in LDS
        pair_class[i] = sm ? PAIR_SMALL : PAIR_LARGE;
        if (sm) {
            mk = max(mk, (uint32_t)keys); mp = max(mp, (uint32_t)prod); ma = max(ma, (uint32_t)nA);
            mb = max(mb, (uint32_t)nB); mbk = max(mbk, nb_table[prod]); ml = max(ml, (uint32_t)capL);
        } else {
            const unsigned long long slot = atomicAdd(&stats->n_large, 1ull);
            large_ids[slot] = i;
        }
    }
    // n_small = n - n_large on the host: no per-block count
    uint32_t v[6] = {mk, mp, ma, mb, mbk, ml};
    const bool is_sum[6] = {false, false, false, false, false, false};
    block_reduce_stats<6>(v, is_sum, red);
    // the six maxima (consecutive plan_stats fields) by six lanes at once: one read and at most one
    // atomic round trip at the block's end instead of six of each in sequence
    __syncthreads();   // red[] was read by thread 0 inside block_reduce_stats
    if (threadIdx.x == 0)
#pragma unroll
        for (int f = 0; f < 6; ++f) red[f] = v[f];
    __syncthreads();
    if (threadIdx.x < 6) max_if_greater(&stats->max_keys + threadIdx.x, red[threadIdx.x]);
}

__global__ __launch_bounds__(kPlanBlock) void k_plan_add(pvac_ct_batch A, pvac_ct_batch B, pvac_ct_batch C,
                                                        plan_stats* stats, uint8_t* pair_class, uint64_t* merge_ids,
                                                        uint64_t edge_budget) {
    __shared__ uint32_t red[kPlanBlock / 64];
    uint32_t ml = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kPlanBlock + threadIdx.x; i < A.n; i += (uint64_t)gridDim.x * kPlanBlock) {
        const uint64_t capL = A.l_cnt[i] + B.l_cnt[i];
        const uint64_t capE = A.e_cnt[i] + B.e_cnt[i];
        C.l_off[i] = capL;
        C.e_off[i] = capE;
        // guard_budget (encrypt.hpp:106-111): over-budget pairs take the merge path (k_add_merge.hip)
        const bool merge = capE > edge_budget;
        pair_class[i] = merge ? PAIR_LARGE : PAIR_SMALL;
        if (merge) merge_ids[atomicAdd(&stats->n_large, 1ull)] = i;
        ml = max(ml, (uint32_t)(capL > 0xFFFFFFFFull ? 0xFFFFFFFFull : capL));
    }
    uint32_t v[1] = {ml};
    const bool is_sum[1] = {false};
    block_reduce_stats<1>(v, is_sum, red);
    if (threadIdx.x == 0) max_if_greater(&stats->max_layers, v[0]);
}

// shapes and offsets of the over-budget ct_add pairs: {pair, LA, LB, nA, nB, aeo, beo, ceo}
__global__ __launch_bounds__(kPlanBlock) void k_gather_merge(pvac_ct_batch A, pvac_ct_batch B, pvac_ct_batch C,
                                                            const uint64_t* ids, uint64_t n, uint64_t* out) {
    const uint64_t k = (uint64_t)blockIdx.x * kPlanBlock + threadIdx.x;
    if (k >= n) return;
    const uint64_t p = ids[k];
    uint64_t* o = out + 8 * k;
    o[0] = p;
    o[1] = A.l_cnt[p];
    o[2] = B.l_cnt[p];
    o[3] = A.e_cnt[p];
    o[4] = B.e_cnt[p];
    o[5] = A.e_off[p];
    o[6] = B.e_off[p];
    o[7] = C.e_off[p];
}

// shapes of the general-path pairs for the host's descriptor build: {pair, LA, LB, nA, nB}
__global__ __launch_bounds__(kPlanBlock) void k_gather_large(pvac_ct_batch A, pvac_ct_batch B, const uint64_t* ids,
                                                            uint64_t n, uint64_t* out) {
    const uint64_t k = (uint64_t)blockIdx.x * kPlanBlock + threadIdx.x;
    if (k >= n) return;
    const uint64_t p = ids[k];
    out[5 * k + 0] = p;
    out[5 * k + 1] = A.l_cnt[p];
    out[5 * k + 2] = B.l_cnt[p];
    out[5 * k + 3] = A.e_cnt[p];
    out[5 * k + 4] = B.e_cnt[p];
}

// ---------------------------------------------------------------- exclusive scan (u64)
constexpr int kScanBlock = 256;
constexpr int kScanPer = 8;
constexpr int kScanTile = kScanBlock * kScanPer;

template <int BS>
__device__ __forceinline__ uint64_t block_scan_u64(uint64_t v, uint64_t* part, uint64_t& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) part[wave] = x;
    __syncthreads();
    uint64_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < BS / 64; ++w) {
        base += (w < wave) ? part[w] : 0ull;
        tot += part[w];
    }
    total = tot;
    __syncthreads();
    return base + x - v;
}

// The scan kernels take up to two arrays of n values (blockIdx.y picks one, its tile sums at
// tile_sums + y * stride): a plan's two capacity arrays are scanned by one launch of each kernel.
struct scan_arrays {
    uint64_t* data[2];
    unsigned long long* total[2];
    size_t stride;   // tile-sum words per array
};

__global__ __launch_bounds__(kScanBlock) void k_scan_reduce(scan_arrays a, size_t n, uint64_t* tile_sums) {
    __shared__ uint64_t part[kScanBlock / 64];
    const uint64_t* data = a.data[blockIdx.y];
    tile_sums += blockIdx.y * a.stride;
    const size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanPer;
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k)
        if (base + k < n) s += data[base + k];
    uint64_t tot;
    (void)block_scan_u64<kScanBlock>(s, part, tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

// single workgroup: exclusive scan of tile sums (any count), writes grand total
__global__ __launch_bounds__(kScanBlock) void k_scan_tiles(scan_arrays a, uint64_t* tile_sums, size_t ntiles) {
    __shared__ uint64_t part[kScanBlock / 64];
    tile_sums += blockIdx.x * a.stride;
    unsigned long long* total_out = a.total[blockIdx.x];
    uint64_t carry = 0;
    for (size_t b = 0; b < ntiles; b += kScanBlock) {
        const size_t i = b + threadIdx.x;
        const uint64_t v = i < ntiles ? tile_sums[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_scan_u64<kScanBlock>(v, part, tot);
        if (i < ntiles) tile_sums[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0 && total_out) *total_out = carry;
}

__global__ __launch_bounds__(kScanBlock) void k_scan_apply(scan_arrays a, size_t n, const uint64_t* tile_offs) {
    __shared__ uint64_t part[kScanBlock / 64];
    uint64_t* data = a.data[blockIdx.y];
    tile_offs += blockIdx.y * a.stride;
    const size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanPer;
    uint64_t v[kScanPer];
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        v[k] = base + k < n ? data[base + k] : 0;
        s += v[k];
    }
    uint64_t tot;
    uint64_t run = tile_offs[blockIdx.x] + block_scan_u64<kScanBlock>(s, part, tot);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        if (base + k < n) data[base + k] = run;
        run += v[k];
    }
}

// ---------------------------------------------------------------- ct_add / ct_sub
constexpr int kAddBlock = 256;

__global__ __launch_bounds__(kAddBlock) void k_ct_add(pvac_ct_batch A, pvac_ct_batch B, pvac_ct_batch C, int negate_b,
                                                     uint32_t lds_layers, const uint8_t* pair_class) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint32_t* keep = (uint32_t*)lds;                 // [lds_layers] then remap in place
    __shared__ uint32_t flags[4];
    __shared__ uint32_t part[kAddBlock / 64];
    const uint64_t pr = blockIdx.x;
    if (pr >= A.n) return;
    if (pair_class && pair_class[pr] == PAIR_LARGE) return;   // over edge_budget: k_add_merge.hip
    const int tid = threadIdx.x;
    const uint32_t LA = (uint32_t)A.l_cnt[pr], LB = (uint32_t)B.l_cnt[pr];
    const uint32_t L = LA + LB;
    const uint64_t nA = A.e_cnt[pr], nB = B.e_cnt[pr];
    const uint64_t alo = A.l_off[pr], blo = B.l_off[pr], aeo = A.e_off[pr], beo = B.e_off[pr];
    const uint64_t clo = C.l_off[pr], ceo = C.e_off[pr];

    for (uint32_t l = tid; l < L; l += kAddBlock) keep[l] = 0;
    if (tid == 0) { flags[0] = 0; flags[1] = 0; }
    __syncthreads();
    // used by edges (encrypt.hpp:78)
    for (uint64_t e = tid; e < nA; e += kAddBlock) {
        const uint32_t lid = meta_layer(A.meta[aeo + e]);
        if (lid < L) keep[lid] = 1;
    }
    for (uint64_t e = tid; e < nB; e += kAddBlock) {
        const uint32_t lid = meta_layer(B.meta[beo + e]) + LA;
        if (lid < L) keep[lid] = 1;
    }
    __syncthreads();
    // transitive closure over PROD parents, parallel sweeps until stable
    for (;;) {
        if (tid == 0) flags[0] = 0;
        __syncthreads();
        for (uint32_t l = tid; l < L; l += kAddBlock) {
            if (!keep[l]) continue;
            const pvac_layer& x = l < LA ? A.layers[alo + l] : B.layers[blo + (l - LA)];
            if (x.rule != 1) continue;
            const uint32_t off = l < LA ? 0u : LA;
            const uint32_t pa = x.pa + off, pb = x.pb + off;
            if (pa < L && !keep[pa]) { keep[pa] = 1; flags[0] = 1; }
            if (pb < L && !keep[pb]) { keep[pb] = 1; flags[0] = 1; }
        }
        __syncthreads();
        if (!flags[0]) break;
        __syncthreads();
    }
    // remap = exclusive count of kept layers (chunked block scan)
    const uint32_t per = (L + kAddBlock - 1) / kAddBlock;
    uint32_t local = 0;
    for (uint32_t l = tid * per; l < (tid + 1) * per && l < L; ++l) local += keep[l];
    uint32_t kept;
    uint32_t run = block_exclusive_scan<kAddBlock>(local, part, kept);
    for (uint32_t l = tid * per; l < (tid + 1) * per && l < L; ++l) {
        const uint32_t k = keep[l];
        keep[l] = k ? run : 0xFFFFFFFFu;
        run += k;
    }
    __syncthreads();
    const bool identity = kept == L;
    // layers
    for (uint32_t l = tid; l < L; l += kAddBlock) {
        const uint32_t to = keep[l];
        if (to == 0xFFFFFFFFu) continue;
        pvac_layer y = l < LA ? A.layers[alo + l] : B.layers[blo + (l - LA)];
        if (l >= LA && y.rule == 1) { y.pa += LA; y.pb += LA; }
        if (!identity && y.rule == 1) {
            y.pa = y.pa < L ? keep[y.pa] : 0xFFFFFFFFu;
            y.pb = y.pb < L ? keep[y.pb] : 0xFFFFFFFFu;
        }
        C.layers[clo + to] = y;
    }
    if (tid == 0) {
        C.l_cnt[pr] = kept;
        C.e_cnt[pr] = nA + nB;
    }
    // edges (concat; B shifted and optionally scaled by p-1)
    const fp pm1{kAll - 1, kM63};
    for (uint64_t e = tid; e < nA + nB; e += kAddBlock) {
        const bool fromB = e >= nA;
        const uint64_t src = fromB ? beo + (e - nA) : aeo + e;
        uint64_t m = fromB ? B.meta[src] : A.meta[src];
        uint64_t wl = fromB ? B.w_lo[src] : A.w_lo[src];
        uint64_t wh = fromB ? B.w_hi[src] : A.w_hi[src];
        uint32_t lid = meta_layer(m) + (fromB ? LA : 0u);
        if (!identity) lid = lid < L ? keep[lid] : 0xFFFFFFFFu;
        m = (m & ~0xFFFFFFFFull) | lid;
        if (fromB && negate_b) {
            const fp r = fp_mul(fp{wl, wh}, pm1);
            wl = r.lo; wh = r.hi;
        }
        __builtin_nontemporal_store((unsigned long long)m, (unsigned long long*)C.meta + ceo + e);
        __builtin_nontemporal_store((unsigned long long)wl, (unsigned long long*)C.w_lo + ceo + e);
        __builtin_nontemporal_store((unsigned long long)wh, (unsigned long long*)C.w_hi + ceo + e);
    }
    // sigma carry: one 16-byte lane chunk per work item
    if (C.sigma && A.sigma && B.sigma) {
        const uint32_t sw = C.sigma_words;
        const uint64_t chunks_per_edge = sw / 2;
        const uint64_t total = (nA + nB) * chunks_per_edge;
        for (uint64_t c = tid; c < total; c += kAddBlock) {
            const uint64_t e = c / chunks_per_edge, k = c - e * chunks_per_edge;
            const bool fromB = e >= nA;
            const ulonglong2* srcp = fromB ? (const ulonglong2*)(B.sigma + (beo + (e - nA)) * B.sigma_words)
                                           : (const ulonglong2*)(A.sigma + (aeo + e) * A.sigma_words);
            ((ulonglong2*)(C.sigma + (ceo + e) * sw))[k] = srcp[k];
        }
    }
}


// Pairs of at most 64 layers (every fresh and most chain ciphers): a group of G lanes per pair,
// G = 64 (one wave) or 32 (two pairs per wave, for pairs of at most 32 layers: twice the pairs in
// flight per wave; the kernel is bound by each pair's chain of dependent memory round trips).
// No barriers: compact_layers is a 64-bit mask closure (lane l of the group holds layer l's PROD
// parents, as in k_ct_mul_fresh), the remap a popcount below each kept layer, kept in a per-group
// LDS table for the edges' lookups. k_ct_add's one workgroup per pair spent six barriers on ~80
// edges and ran at 14% of the HBM roofline.
constexpr int kAddWaves = 4;
constexpr int kPre = 3;   // edges per lane held in registers by k_ct_add_wave (fresh pairs: all)

template <int G>
__device__ __forceinline__ uint64_t group_or_u64(uint64_t v) {
#pragma unroll
    for (int d = 1; d < G; d <<= 1) v |= (uint64_t)__shfl_xor((long long)v, d, 64);
    return v;
}

template <int G>
__global__ __launch_bounds__(64 * kAddWaves) void k_ct_add_wave(pvac_ct_batch A, pvac_ct_batch B, pvac_ct_batch C,
                                                               int negate_b, const uint8_t* pair_class) {
    static_assert(G == 32 || G == 64, "lane groups of 32 or 64 (16 measured no faster than 32)");
    __shared__ uint32_t remap_s[kAddWaves][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t gl = (uint32_t)lane & (G - 1);   // lane within the pair's group
    const uint64_t pr = ((uint64_t)blockIdx.x * kAddWaves + wave) * (64 / G) + (uint32_t)lane / G;
    // a group without a pair (batch tail, over-budget pair: k_add_merge.hip) runs with zero counts
    // and stores nothing, so every group reaches the same shuffles
    const bool live = pr < A.n && !(pair_class && pair_class[pr] == PAIR_LARGE);
    const uint32_t LA = live ? (uint32_t)A.l_cnt[pr] : 0u, LB = live ? (uint32_t)B.l_cnt[pr] : 0u;
    const uint32_t L = LA + LB;   // <= G (host-checked)
    const uint64_t nA = live ? A.e_cnt[pr] : 0ull, nB = live ? B.e_cnt[pr] : 0ull;
    const uint64_t alo = live ? A.l_off[pr] : 0ull, blo = live ? B.l_off[pr] : 0ull;
    const uint64_t aeo = live ? A.e_off[pr] : 0ull, beo = live ? B.e_off[pr] : 0ull;
    const uint64_t clo = live ? C.l_off[pr] : 0ull, ceo = live ? C.e_off[pr] : 0ull;
    // The group's first kPre*G edges (every fresh pair: 80 edges) are loaded once, up front, with
    // the layer record below in flight beside them: they feed both the used-layer mask and the
    // output, so the pair pays one dependent memory round trip for its edges instead of two.
    const uint64_t nE = nA + nB;
    uint64_t pm[kPre], pwl[kPre], pwh[kPre];
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
        const uint64_t e = gl + (uint64_t)u * G;
        const bool fromB = e >= nA;
        const uint64_t src = fromB ? beo + (e - nA) : aeo + e;
        const uint64_t* mp = fromB ? B.meta : A.meta;
        const uint64_t* lp = fromB ? B.w_lo : A.w_lo;
        const uint64_t* hp = fromB ? B.w_hi : A.w_hi;
        pm[u] = 0; pwl[u] = 0; pwh[u] = 0;
        if (e < nE) { pm[u] = mp[src]; pwl[u] = lp[src]; pwh[u] = hp[src]; }
    }
    const uint32_t l = gl;
    pvac_layer x{};
    if (l < L) x = l < LA ? A.layers[alo + l] : B.layers[blo + (l - LA)];
    // layers used by edges (encrypt.hpp:78)
    uint64_t used = 0;
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
        const uint64_t e = gl + (uint64_t)u * G;
        const uint32_t lid = meta_layer(pm[u]) + (e >= nA ? LA : 0u);
        used |= (e < nE && lid < L) ? 1ull << lid : 0ull;
    }
    for (uint64_t e = gl + (uint64_t)kPre * G; e < nE; e += G) {
        const bool fromB = e >= nA;
        const uint32_t lid = fromB ? meta_layer(B.meta[beo + (e - nA)]) + LA : meta_layer(A.meta[aeo + e]);
        used |= lid < L ? 1ull << lid : 0ull;
    }
    used = group_or_u64<G>(used);
    // transitive PROD parents (encrypt.hpp:80-93)
    const uint32_t off = l < LA ? 0u : LA;
    const uint32_t pa = x.pa + off, pb = x.pb + off;
    const uint64_t mypm = (l < L && x.rule == 1) ? ((pa < L ? 1ull << pa : 0ull) | (pb < L ? 1ull << pb : 0ull)) : 0ull;
    uint64_t keep = used;
    for (;;) {   // depth-bounded by L; the wave stops when every group has reached its fixpoint
        const uint64_t nk = keep | group_or_u64<G>(((keep >> l) & 1ull) ? mypm : 0ull);
        const bool moved = nk != keep;
        keep = nk;
        if (!__any(moved)) break;
    }
    const uint32_t kept = (uint32_t)__popcll(keep);
    const bool identity = kept == L;
    const uint32_t to = ((keep >> l) & 1ull) ? (uint32_t)__popcll(keep & ((1ull << l) - 1ull)) : 0xFFFFFFFFu;
    uint32_t* remap = remap_s[wave] + ((uint32_t)lane & ~(uint32_t)(G - 1));
    remap[l] = to;
    __builtin_amdgcn_wave_barrier();
    if (l < L && to != 0xFFFFFFFFu) {
        pvac_layer y = x;
        if (l >= LA && y.rule == 1) { y.pa += LA; y.pb += LA; }
        if (!identity && y.rule == 1) {
            y.pa = y.pa < L ? remap[y.pa] : 0xFFFFFFFFu;
            y.pb = y.pb < L ? remap[y.pb] : 0xFFFFFFFFu;
        }
        C.layers[clo + to] = y;
    }
    if (live && gl == 0) {
        C.l_cnt[pr] = kept;
        C.e_cnt[pr] = nA + nB;
    }
    // edges (concat; B shifted and optionally scaled by p-1)
    const fp pm1{kAll - 1, kM63};
    auto emit = [&](uint64_t e, uint64_t m, uint64_t wl, uint64_t wh) {
        const bool fromB = e >= nA;
        uint32_t lid = meta_layer(m) + (fromB ? LA : 0u);
        if (!identity) lid = lid < L ? remap[lid] : 0xFFFFFFFFu;
        m = (m & ~0xFFFFFFFFull) | lid;
        if (fromB && negate_b) {
            const fp r = fp_mul(fp{wl, wh}, pm1);
            wl = r.lo; wh = r.hi;
        }
        // streaming stores: ct_add 0.93 -> 0.90 ms, ct_sub 0.94 -> 0.90 ms per 2^20 fresh pairs (A/B)
        __builtin_nontemporal_store((unsigned long long)m, (unsigned long long*)C.meta + ceo + e);
        __builtin_nontemporal_store((unsigned long long)wl, (unsigned long long*)C.w_lo + ceo + e);
        __builtin_nontemporal_store((unsigned long long)wh, (unsigned long long*)C.w_hi + ceo + e);
    };
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
        const uint64_t e = gl + (uint64_t)u * G;
        if (e < nE) emit(e, pm[u], pwl[u], pwh[u]);
    }
    for (uint64_t e = gl + (uint64_t)kPre * G; e < nE; e += G) {
        const bool fromB = e >= nA;
        const uint64_t src = fromB ? beo + (e - nA) : aeo + e;
        emit(e, fromB ? B.meta[src] : A.meta[src], fromB ? B.w_lo[src] : A.w_lo[src],
             fromB ? B.w_hi[src] : A.w_hi[src]);
    }
    if (C.sigma && A.sigma && B.sigma) {   // sigma carry: 16 bytes per lane
        const uint32_t sw = C.sigma_words;
        const uint64_t chunks_per_edge = sw / 2;
        const uint64_t total = (nA + nB) * chunks_per_edge;
        for (uint64_t c = gl; c < total; c += G) {
            const uint64_t e = c / chunks_per_edge, k = c - e * chunks_per_edge;
            const bool fromB = e >= nA;
            const ulonglong2* srcp = fromB ? (const ulonglong2*)(B.sigma + (beo + (e - nA)) * B.sigma_words)
                                           : (const ulonglong2*)(A.sigma + (aeo + e) * A.sigma_words);
            ((ulonglong2*)(C.sigma + (ceo + e) * sw))[k] = srcp[k];
        }
    }
}

}  // namespace

// ==================================================================== launch wrappers
hipError_t launch_plan_mul(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, uint8_t* pair_class,
                           uint64_t* large_ids, plan_stats* stats, const uint32_t* nb_table, uint32_t nb_len,
                           uint32_t Bm, hipStream_t st) {
    if (!A.n) return hipSuccess;
    hipLaunchKernelGGL(k_plan_mul, dim3(plan_grid(A.n)), dim3(kPlanBlock), 0, st, A,
                       B, C, pair_class, large_ids, stats, nb_table, nb_len, Bm);
    return hipGetLastError();
}

hipError_t launch_gather_large(const pvac_ct_batch& A, const pvac_ct_batch& B, const uint64_t* ids, uint64_t n,
                               uint64_t* out, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gather_large, dim3((unsigned)((n + kPlanBlock - 1) / kPlanBlock)), dim3(kPlanBlock), 0, st, A,
                       B, ids, n, out);
    return hipGetLastError();
}

hipError_t launch_plan_add(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, plan_stats* stats,
                           uint8_t* pair_class, uint64_t* merge_ids, uint64_t edge_budget, hipStream_t st) {
    if (!A.n) return hipSuccess;
    hipLaunchKernelGGL(k_plan_add, dim3(plan_grid(A.n)), dim3(kPlanBlock), 0, st, A,
                       B, C, stats, pair_class, merge_ids, edge_budget);
    return hipGetLastError();
}

hipError_t launch_gather_merge(const pvac_ct_batch& A, const pvac_ct_batch& B, const pvac_ct_batch& C,
                               const uint64_t* ids, uint64_t n, uint64_t* out, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gather_merge, dim3((unsigned)((n + kPlanBlock - 1) / kPlanBlock)), dim3(kPlanBlock), 0, st, A,
                       B, C, ids, n, out);
    return hipGetLastError();
}

size_t scan_scratch_words(size_t n) { return 2 * ((n + kScanTile - 1) / kScanTile + 1); }

namespace {
hipError_t launch_scans(const scan_arrays& a, unsigned arrays, size_t n, uint64_t* scratch, hipStream_t st) {
    if (!n) return hipSuccess;
    const size_t tiles = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)tiles, arrays), dim3(kScanBlock), 0, st, a, n, scratch);
    hipLaunchKernelGGL(k_scan_tiles, dim3(arrays), dim3(kScanBlock), 0, st, a, scratch, tiles);
    hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)tiles, arrays), dim3(kScanBlock), 0, st, a, n, scratch);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_exclusive_scan_u64(uint64_t* data, size_t n, uint64_t* scratch, unsigned long long* total_out,
                                     hipStream_t st) {
    const scan_arrays a{{data, data}, {total_out, total_out}, (n + kScanTile - 1) / kScanTile + 1};
    return launch_scans(a, 1, n, scratch, st);
}

hipError_t launch_exclusive_scan2_u64(uint64_t* d0, uint64_t* d1, size_t n, uint64_t* scratch,
                                      unsigned long long* total0, unsigned long long* total1, hipStream_t st) {
    const scan_arrays a{{d0, d1}, {total0, total1}, (n + kScanTile - 1) / kScanTile + 1};
    return launch_scans(a, 2, n, scratch, st);
}

hipError_t launch_ct_add(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, int negate_b,
                         uint32_t max_layers, const uint8_t* pair_class, hipStream_t st) {
    if (!A.n) return hipSuccess;
    if (max_layers <= 32) {
        hipLaunchKernelGGL(k_ct_add_wave<32>, dim3((unsigned)((A.n + 2 * kAddWaves - 1) / (2 * kAddWaves))),
                           dim3(64 * kAddWaves), 0, st, A, B, C, negate_b, pair_class);
        return hipGetLastError();
    }
    if (max_layers <= 64) {
        hipLaunchKernelGGL(k_ct_add_wave<64>, dim3((unsigned)((A.n + kAddWaves - 1) / kAddWaves)), dim3(64 * kAddWaves),
                           0, st, A, B, C, negate_b, pair_class);
        return hipGetLastError();
    }
    const size_t lds = ((size_t)max_layers * 4 + 15) & ~(size_t)15;
    if (lds > 120 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ct_add, dim3((unsigned)A.n), dim3(kAddBlock), lds, st, A, B, C, negate_b, max_layers,
                       pair_class);
    return hipGetLastError();
}

}  // namespace pvhip
