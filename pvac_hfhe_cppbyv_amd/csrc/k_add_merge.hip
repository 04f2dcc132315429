// k_add_merge.hip — guard_budget for ct_add / ct_sub (ops/encrypt.hpp:39-71,106-111 then
// compact_layers :73-104), the path taken by a pair whose |A.E| + |B.E| exceeds edge_budget.
//
// The reference merges every (layer, idx, ch) group with a sequential fp_add chain in edge order
// (A's edges, then B's, each in input order) and XORs the group's sigmas; it drops a group whose
// sum and sigma are both zero and emits the rest sorted by (layer, idx, P before M). fp_add
// truncates the high word for non-canonical addends (field.hpp:53-55), which makes the chain
// order-dependent, so the GPU path keeps the order exactly: a STABLE radix sort of
// (key, edge index) groups each key's edges in input order, and one thread folds each group.
//
// One over-budget pair at a time (each holds > edge_budget = 1.2 M edges by default):
//   keys -> stable sort -> group heads + scan -> group starts -> fold (w) -> sigma-nonzero test
//   -> keep + scan -> write (meta, w, sigma XOR) -> compact_layers (one block) -> edge relabel.
#include "common.hpp"
#include <hipcub/hipcub.hpp>

namespace pvhip {
namespace {

constexpr uint32_t kBadKey = 0xFFFFFFFFu;
constexpr int kMB = 256;

struct pair_src {
    const uint64_t *am, *al, *ah, *bm, *bl, *bh;   // A / B edge arrays at the pair's offsets
    const uint64_t *as, *bs;                        // sigma rows (nullable)
    uint32_t nA, nB, LA, L, Bm, sw;
    int negate_b;
};

__device__ __forceinline__ fp edge_w(const pair_src& p, uint32_t e) {
    if (e < p.nA) return fp{p.al[e], p.ah[e]};
    const fp w{p.bl[e - p.nA], p.bh[e - p.nA]};
    // ct_sub = ct_add(A, ct_neg(B)), ct_neg = ct_scale by p - 1 (arithmetic.hpp:39-45)
    return p.negate_b ? fp_mul(w, fp{kAll - 1, kM63}) : w;
}
__device__ __forceinline__ const uint64_t* edge_sigma(const pair_src& p, uint32_t e) {
    return e < p.nA ? p.as + (uint64_t)e * p.sw : p.bs + (uint64_t)(e - p.nA) * p.sw;
}

__global__ __launch_bounds__(kMB) void k_merge_keys(pair_src p, uint32_t* keys, uint32_t* vals) {
    const uint32_t e = blockIdx.x * kMB + threadIdx.x;
    if (e >= p.nA + p.nB) return;
    const bool fromB = e >= p.nA;
    const uint64_t m = fromB ? p.bm[e - p.nA] : p.am[e];
    const uint32_t lid = meta_layer(m) + (fromB ? p.LA : 0u);
    const uint32_t idx = meta_idx(m);
    const uint32_t ch = meta_ch(m) != 0 ? 1u : 0u;   // anything but SGN_P aggregates as M
    // out-of-range references (undefined in the reference) sort last and are dropped
    keys[e] = (lid < p.L && idx < p.Bm) ? (lid * p.Bm + idx) * 2u + ch : kBadKey;
    vals[e] = e;
}

__global__ __launch_bounds__(kMB) void k_merge_heads(const uint32_t* keys, uint32_t n, uint64_t* heads) {
    const uint32_t i = blockIdx.x * kMB + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = keys[i];
    heads[i] = (k != kBadKey && (i == 0 || keys[i - 1] != k)) ? 1u : 0u;
}

// heads (exclusive-scanned in place) -> start[g] of every group; start[ngroups] = first bad key
__global__ __launch_bounds__(kMB) void k_merge_starts(const uint32_t* keys, uint32_t n, const uint64_t* gid,
                                                      const unsigned long long* ngroups, uint32_t* start) {
    const uint32_t i = blockIdx.x * kMB + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = keys[i];
    if (k == kBadKey) return;
    if (i == 0 || keys[i - 1] != k) start[gid[i]] = i;
    if (i + 1 == n || keys[i + 1] == kBadKey) start[*ngroups] = i + 1;
}

// sequential fp_add chain per group, starting from 0 (encrypt.hpp:46-56)
__global__ __launch_bounds__(kMB) void k_merge_fold(pair_src p, const uint32_t* vals, const uint32_t* start,
                                                    const unsigned long long* ngroups, uint64_t* glo, uint64_t* ghi,
                                                    uint64_t* keep) {
    const uint32_t g = blockIdx.x * kMB + threadIdx.x;
    if (g >= *ngroups) return;
    fp acc{0, 0};
    for (uint32_t i = start[g]; i < start[g + 1]; ++i) acc = fp_add(acc, edge_w(p, vals[i]));
    glo[g] = acc.lo;
    ghi[g] = acc.hi;
    keep[g] = fp_nonzero(acc) ? 1u : 0u;
}

// sigma XOR of a group is nonzero -> keep (one wave per group; lanes own words lane, lane + 64, ...)
__global__ __launch_bounds__(kMB) void k_merge_signz(pair_src p, const uint32_t* vals, const uint32_t* start,
                                                     const unsigned long long* ngroups, uint64_t* keep) {
    const uint32_t g = blockIdx.x * (kMB / 64) + threadIdx.x / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (g >= *ngroups || keep[g]) return;   // wave-uniform
    uint64_t any = 0;
    for (uint32_t w = lane; w < p.sw; w += 64) {
        uint64_t x = 0;
        for (uint32_t i = start[g]; i < start[g + 1]; ++i) x ^= edge_sigma(p, vals[i])[w];
        any |= x;
    }
    if (__ballot(any != 0) && lane == 0) keep[g] = 1;
}

__global__ __launch_bounds__(kMB) void k_merge_write(pair_src p, const uint32_t* keys, const uint32_t* start,
                                                     const unsigned long long* ngroups, const uint64_t* glo,
                                                     const uint64_t* ghi, const uint64_t* pos, uint64_t* cm,
                                                     uint64_t* cl, uint64_t* ch_) {
    const uint32_t g = blockIdx.x * kMB + threadIdx.x;
    if (g >= *ngroups) return;
    const uint64_t q = pos[g];
    if (pos[g + 1] == q) return;   // dropped (pos is the exclusive scan of the keep flags)
    const uint32_t k = keys[start[g]];
    const uint32_t slot = k >> 1;
    const uint32_t lid = slot / p.Bm, idx = slot - lid * p.Bm;
    cm[q] = make_meta(lid, idx, k & 1u);
    cl[q] = glo[g];
    ch_[q] = ghi[g];
}

__global__ __launch_bounds__(kMB) void k_merge_sigma(pair_src p, const uint32_t* vals, const uint32_t* start,
                                                     const unsigned long long* ngroups, const uint64_t* pos,
                                                     uint64_t* csig) {
    const uint32_t g = blockIdx.x * (kMB / 64) + threadIdx.x / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (g >= *ngroups) return;
    const uint64_t q = pos[g];
    if (pos[g + 1] == q) return;
    for (uint32_t w = lane; w < p.sw; w += 64) {
        uint64_t x = 0;
        for (uint32_t i = start[g]; i < start[g + 1]; ++i) x ^= edge_sigma(p, vals[i])[w];
        csig[q * p.sw + w] = x;
    }
}

// compact_layers over the merged edges (encrypt.hpp:73-104), one block; keep[] is global scratch
constexpr int kLB = 1024;
__global__ __launch_bounds__(kLB) void k_merge_layers(pvac_ct_batch A, pvac_ct_batch B, pvac_ct_batch C, uint64_t pr,
                                                      const uint64_t* cm, const unsigned long long* nout,
                                                      uint32_t* keep, uint32_t* flag_ident) {
    __shared__ uint32_t flags[2];
    __shared__ uint32_t part[kLB / 64];
    const int tid = threadIdx.x;
    const uint32_t LA = (uint32_t)A.l_cnt[pr], LB = (uint32_t)B.l_cnt[pr], L = LA + LB;
    const uint64_t alo = A.l_off[pr], blo = B.l_off[pr], clo = C.l_off[pr];
    const uint64_t ne = *nout;
    for (uint32_t l = tid; l < L; l += kLB) keep[l] = 0;
    __syncthreads();
    for (uint64_t e = tid; e < ne; e += kLB) keep[meta_layer(cm[e])] = 1;   // lids < L by construction
    __syncthreads();
    for (;;) {   // transitive PROD parents until stable
        if (tid == 0) flags[0] = 0;
        __syncthreads();
        for (uint32_t l = tid; l < L; l += kLB) {
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
    const uint32_t per = (L + kLB - 1) / kLB;
    uint32_t local = 0;
    for (uint32_t l = tid * per; l < (tid + 1) * per && l < L; ++l) local += keep[l];
    uint32_t kept;
    uint32_t run = block_exclusive_scan<kLB>(local, part, kept);
    for (uint32_t l = tid * per; l < (tid + 1) * per && l < L; ++l) {
        const uint32_t k = keep[l];
        keep[l] = k ? run : 0xFFFFFFFFu;
        run += k;
    }
    __syncthreads();
    const bool identity = kept == L;
    for (uint32_t l = tid; l < L; l += kLB) {
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
        C.e_cnt[pr] = ne;
        *flag_ident = identity ? 1u : 0u;
    }
}

__global__ __launch_bounds__(kMB) void k_merge_relabel(uint64_t* cm, const unsigned long long* nout,
                                                       const uint32_t* remap, const uint32_t* flag_ident) {
    const uint64_t e = (uint64_t)blockIdx.x * kMB + threadIdx.x;
    if (e >= *nout || *flag_ident) return;
    const uint64_t m = cm[e];
    cm[e] = (m & ~0xFFFFFFFFull) | remap[meta_layer(m)];
}

}  // namespace

size_t merge_scratch_bytes(uint64_t n, uint32_t L) {
    size_t cub = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, cub, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                       (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 32);
    const size_t al = 256;
    auto up = [&](size_t b) { return (b + al - 1) / al * al; };
    return up(cub) + 4 * up(n * 4) + 5 * up((n + 2) * 8) + up((size_t)L * 4) + up(64);
}

hipError_t launch_add_merge(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, uint64_t pr,
                            const merge_pair_info& info, uint32_t Bm, int negate_b, void* scratch, size_t scratch_bytes,
                            unsigned long long* counters, hipStream_t st) {
    const uint64_t n = info.nA + info.nB;
    if (!n) return hipSuccess;
    const size_t al = 256;
    auto up = [&](size_t b) { return (b + al - 1) / al * al; };
    size_t cub = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, cub, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                      (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 32);
    if (e != hipSuccess) return e;
    uint8_t* s = (uint8_t*)scratch;
    uint8_t* end = s + scratch_bytes;
    auto take = [&](size_t b) { uint8_t* r = s; s += up(b); return r; };
    void* tmp = take(cub);
    uint32_t* kin = (uint32_t*)take(n * 4);
    uint32_t* kout = (uint32_t*)take(n * 4);
    uint32_t* vin = (uint32_t*)take(n * 4);
    uint32_t* vout = (uint32_t*)take(n * 4);
    uint64_t* heads = (uint64_t*)take((n + 2) * 8);
    uint64_t* glo = (uint64_t*)take((n + 2) * 8);
    uint64_t* ghi = (uint64_t*)take((n + 2) * 8);
    uint64_t* keep = (uint64_t*)take((n + 2) * 8);
    uint32_t* start = (uint32_t*)take((n + 2) * 8);
    uint32_t* lkeep = (uint32_t*)take((size_t)info.L * 4);
    uint32_t* ident = (uint32_t*)take(64);
    if (s > end) return hipErrorInvalidValue;

    pair_src p{};
    const uint64_t aeo = info.aeo, beo = info.beo;
    p.am = A.meta + aeo; p.al = A.w_lo + aeo; p.ah = A.w_hi + aeo;
    p.bm = B.meta + beo; p.bl = B.w_lo + beo; p.bh = B.w_hi + beo;
    const bool sig = C.sigma && A.sigma && B.sigma;
    p.as = sig ? A.sigma + aeo * A.sigma_words : nullptr;
    p.bs = sig ? B.sigma + beo * B.sigma_words : nullptr;
    p.nA = (uint32_t)info.nA; p.nB = (uint32_t)info.nB;
    p.LA = info.LA; p.L = info.L; p.Bm = Bm;
    p.sw = sig ? C.sigma_words : 0u;
    p.negate_b = negate_b;

    const unsigned blocks = (unsigned)((n + kMB - 1) / kMB);
    hipLaunchKernelGGL(k_merge_keys, dim3(blocks), dim3(kMB), 0, st, p, kin, vin);
    e = hipcub::DeviceRadixSort::SortPairs(tmp, cub, kin, kout, vin, vout, (int)n, 0, 32, st);   // stable
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_merge_heads, dim3(blocks), dim3(kMB), 0, st, kout, (uint32_t)n, heads);
    unsigned long long* ngroups = counters;       // [0] groups, [1] kept edges
    unsigned long long* nout = counters + 1;
    e = launch_exclusive_scan_u64(heads, n, glo /* scratch: reused below */, ngroups, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_merge_starts, dim3(blocks), dim3(kMB), 0, st, kout, (uint32_t)n, heads, ngroups, start);
    e = hipMemsetAsync(keep, 0, (n + 1) * 8, st);   // flags past the last group must read 0
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_merge_fold, dim3(blocks), dim3(kMB), 0, st, p, vout, start, ngroups, glo, ghi, keep);
    if (sig)
        hipLaunchKernelGGL(k_merge_signz, dim3((unsigned)((n + kMB / 64 - 1) / (kMB / 64))), dim3(kMB), 0, st, p, vout,
                           start, ngroups, keep);
    // keep -> positions (n + 1 entries so pos[g + 1] - pos[g] is the keep flag of the last group)
    e = launch_exclusive_scan_u64(keep, n + 1, heads /* scan scratch */, nout, st);
    if (e != hipSuccess) return e;
    const uint64_t ceo = info.ceo;
    hipLaunchKernelGGL(k_merge_write, dim3(blocks), dim3(kMB), 0, st, p, kout, start, ngroups, glo, ghi, keep,
                       C.meta + ceo, C.w_lo + ceo, C.w_hi + ceo);
    if (sig)
        hipLaunchKernelGGL(k_merge_sigma, dim3((unsigned)((n + kMB / 64 - 1) / (kMB / 64))), dim3(kMB), 0, st, p, vout,
                           start, ngroups, keep, C.sigma + ceo * C.sigma_words);
    hipLaunchKernelGGL(k_merge_layers, dim3(1), dim3(kLB), 0, st, A, B, C, pr, C.meta + ceo, nout, lkeep, ident);
    hipLaunchKernelGGL(k_merge_relabel, dim3(blocks), dim3(kMB), 0, st, C.meta + ceo, nout, lkeep, ident);
    return hipGetLastError();
}

}  // namespace pvhip
