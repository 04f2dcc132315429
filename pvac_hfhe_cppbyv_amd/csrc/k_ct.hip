// k_ct.hip — batched ciphertext kernels: sizing plans, scans, ct_mul (fresh-shape, LDS
// resident) and ct_add / ct_sub.
//
// ct_mul (reference ops/arithmetic.hpp:47-106) per pair C = A * B:
//   layers : C.L = A.L ++ B.L (PROD pa/pb += |A.L|) ++ |A.L||B.L| new PROD layers with
//            caller nonces and ztag = SHA-256 layer tag (crypto/matrix.hpp:254-264)
//   weights: for every (i in A.E, j in B.E): slot (la*LB+lb, (idx_i+idx_j) mod B),
//            channel P if ch_i == ch_j else M, acc += fp_mul(w_i, w_j)
//   order  : the reference iterates a std::unordered_map reserved for |A.E||B.E| keys.
//            libstdc++ links a new node first in its bucket when the bucket is non-empty,
//            and at the list front when it is empty, so iteration order is
//            (bucket first-insert time DESC, key first-insert time DESC), where a key's
//            first-insert time is t = i*|B.E| + j of its first product. The kernel
//            reproduces this closed form exactly: per-key t via LDS atomicMin, bucket
//            chains via LDS atomicExch, a counting sort over t, no hash table.
//   then guard_budget / compact_layers (ops/encrypt.hpp:73-111).
//
// Kernel "small" (K3) serves fresh-shaped pairs (|A.L||B.L|B <= 1536 slots, |A.E||B.E| <=
// 4096): one 256-thread workgroup per pair, persistent over the batch, ~72 KB LDS so two
// workgroups share a CU. Sums are exact: each canonical product is split into 43/42/42-bit
// limbs accumulated with ds_add_u64 (order independent, no overflow below 2^21 addends).
#include "common.hpp"
#include "sha256.hpp"

namespace pvhip {

namespace {

constexpr int kPlanBlock = 256;

// ---------------------------------------------------------------- plans
__global__ __launch_bounds__(kPlanBlock) void k_plan_mul(pvac_ct_batch A, pvac_ct_batch B, pvac_ct_batch C,
                                                        uint8_t* pair_class, plan_stats* stats,
                                                        const uint32_t* nb_table, uint32_t nb_len, uint32_t Bm,
                                                        uint32_t ks_small_max, uint32_t prod_small_max) {
    const uint64_t i = (uint64_t)blockIdx.x * kPlanBlock + threadIdx.x;
    if (i >= A.n) return;
    const uint64_t LA = A.l_cnt[i], LB = B.l_cnt[i], nA = A.e_cnt[i], nB = B.e_cnt[i];
    const uint64_t keys = LA * LB * Bm;
    const uint64_t prod = nA * nB;
    const uint64_t capL = LA + LB + LA * LB;
    const uint64_t capE = 2 * (prod < keys ? prod : keys);
    C.l_off[i] = capL;   // scanned in place afterwards
    C.e_off[i] = capE;
    const bool small = keys <= ks_small_max && prod <= prod_small_max && prod < nb_len && nA <= 256 && nB <= 256 &&
                       capL <= 64;
    pair_class[i] = small ? 1 : 2;
    if (small) {
        atomicAdd(&stats->n_small, 1ull);
        atomicMax(&stats->max_keys, (unsigned)keys);
        atomicMax(&stats->max_prod, (unsigned)prod);
        atomicMax(&stats->max_na, (unsigned)nA);
        atomicMax(&stats->max_nb, (unsigned)nB);
        atomicMax(&stats->max_buckets, nb_table[prod]);
        atomicMax(&stats->max_layers, (unsigned)capL);
    } else {
        atomicAdd(&stats->n_large, 1ull);
    }
}

__global__ __launch_bounds__(kPlanBlock) void k_plan_add(pvac_ct_batch A, pvac_ct_batch B, pvac_ct_batch C,
                                                        plan_stats* stats) {
    const uint64_t i = (uint64_t)blockIdx.x * kPlanBlock + threadIdx.x;
    if (i >= A.n) return;
    const uint64_t capL = A.l_cnt[i] + B.l_cnt[i];
    C.l_off[i] = capL;
    C.e_off[i] = A.e_cnt[i] + B.e_cnt[i];
    atomicMax(&stats->max_layers, (unsigned)(capL > 0xFFFFFFFFull ? 0xFFFFFFFFull : capL));
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

__global__ __launch_bounds__(kScanBlock) void k_scan_reduce(const uint64_t* data, size_t n, uint64_t* tile_sums) {
    __shared__ uint64_t part[kScanBlock / 64];
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
__global__ __launch_bounds__(kScanBlock) void k_scan_tiles(uint64_t* tile_sums, size_t ntiles,
                                                          unsigned long long* total_out) {
    __shared__ uint64_t part[kScanBlock / 64];
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

__global__ __launch_bounds__(kScanBlock) void k_scan_apply(uint64_t* data, size_t n, const uint64_t* tile_offs) {
    __shared__ uint64_t part[kScanBlock / 64];
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

// ---------------------------------------------------------------- ct_mul, fresh-shape kernel
constexpr int kMulBlock = 256;
constexpr int kMulSlots = 6;                       // key slots owned per thread
constexpr uint32_t kSmallKeysMax = kMulBlock * kMulSlots;
constexpr uint32_t kTInf = 0xFFFFFFFFu;

struct mul_lds_layout {
    // byte offsets into dynamic LDS
    uint32_t acc, tkey, a_lo, a_hi, a_inf, b_lo, b_hi, b_inf, ztag, remap, misc, total;
};

__host__ __device__ inline uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ inline mul_lds_layout mul_layout(uint32_t ks, uint32_t na, uint32_t nb_e) {
    mul_lds_layout L;
    uint32_t o = 0;
    L.acc = o;   o = align16(o + ks * 48u);          // 2 channels x 3 u64 limbs per key slot
    L.tkey = o;  o = align16(o + ks * 4u);
    L.a_lo = o;  o = align16(o + na * 8u);
    L.a_hi = o;  o = align16(o + na * 8u);
    L.a_inf = o; o = align16(o + na * 4u);
    L.b_lo = o;  o = align16(o + nb_e * 8u);
    L.b_hi = o;  o = align16(o + nb_e * 8u);
    L.b_inf = o; o = align16(o + nb_e * 4u);
    L.ztag = o;  o = align16(o + 64u * 8u);           // product-layer ztags (<= 64 layers)
    L.remap = o; o = align16(o + 64u * 4u);           // output layer remap
    L.misc = o;  o = align16(o + 64u * 4u);           // scan partials + flags
    L.total = o;
    return L;
}

// misc word indices
enum : int { MISC_PART = 0, MISC_FLAG = 8, MISC_TOTAL = 9, MISC_LPUSED = 12 /* u64 at words 12..13 */ };

__global__ __launch_bounds__(kMulBlock, 2) void k_ct_mul_small(mul_small_args g, mul_lds_layout Ls) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    unsigned long long* acc = (unsigned long long*)(lds + Ls.acc);
    uint32_t* tkey = (uint32_t*)(lds + Ls.tkey);
    uint64_t* a_lo = (uint64_t*)(lds + Ls.a_lo);
    uint64_t* a_hi = (uint64_t*)(lds + Ls.a_hi);
    uint32_t* a_inf = (uint32_t*)(lds + Ls.a_inf);
    uint64_t* b_lo = (uint64_t*)(lds + Ls.b_lo);
    uint64_t* b_hi = (uint64_t*)(lds + Ls.b_hi);
    uint32_t* b_inf = (uint32_t*)(lds + Ls.b_inf);
    uint64_t* ztag = (uint64_t*)(lds + Ls.ztag);
    uint32_t* remap = (uint32_t*)(lds + Ls.remap);
    uint32_t* misc = (uint32_t*)(lds + Ls.misc);
    // scratch re-uses the accumulator region after the sums are folded into registers:
    //   heads[nb] (slot+1, 0 = empty) | G[n] (emit counts by first-insert time) | nxt[ks]
    uint32_t* heads = (uint32_t*)(lds + Ls.acc);

    const int tid = threadIdx.x;
    const uint32_t Bm = g.Bm;

    // one-time clear: accumulators 0, tkey = INF
    for (uint32_t w = tid; w < g.ks_max * 6; w += kMulBlock) acc[w] = 0ull;
    for (uint32_t s = tid; s < g.ks_max; s += kMulBlock) tkey[s] = kTInf;
    if (tid == 0) { misc[MISC_FLAG] = 0; *(unsigned long long*)(misc + MISC_LPUSED) = 0ull; }
    __syncthreads();
    unsigned long long* lp_used = (unsigned long long*)(misc + MISC_LPUSED);

    for (uint64_t pr = blockIdx.x; pr < g.A.n; pr += gridDim.x) {
        if (g.pair_class[pr] != 1) continue;   // wave-uniform: served by the large path
        const uint32_t LA = (uint32_t)g.A.l_cnt[pr], LB = (uint32_t)g.B.l_cnt[pr];
        const uint32_t nA = (uint32_t)g.A.e_cnt[pr], nB = (uint32_t)g.B.e_cnt[pr];
        const uint64_t aeo = g.A.e_off[pr], beo = g.B.e_off[pr];
        const uint32_t LP = LA * LB;
        const uint32_t KS = LP * Bm;
        const uint32_t n = nA * nB;
        const uint32_t nbk = g.nb_table[n];
        const uint32_t base = LA + LB;   // first product-layer id in C (before compaction)
        const uint64_t clo = g.C.l_off[pr], ceo = g.C.e_off[pr];

        // ---- S0: stage edges, product-layer ztags, validation (flags were cleared behind
        //      the previous pair's final barrier)
        for (uint32_t i = tid; i < nA; i += kMulBlock) {
            const uint64_t m = g.A.meta[aeo + i];
            const uint32_t la = meta_layer(m), idx = meta_idx(m), ch = meta_ch(m);
            if (la >= LA || idx >= Bm || ch > 1) atomicOr(&misc[MISC_FLAG], 1u);
            a_lo[i] = g.A.w_lo[aeo + i];
            a_hi[i] = g.A.w_hi[aeo + i];
            a_inf[i] = idx | ((la & 0x7FFFu) << 16) | (ch << 31);
        }
        for (uint32_t j = tid; j < nB; j += kMulBlock) {
            const uint64_t m = g.B.meta[beo + j];
            const uint32_t lb = meta_layer(m), idx = meta_idx(m), ch = meta_ch(m);
            if (lb >= LB || idx >= Bm || ch > 1) atomicOr(&misc[MISC_FLAG], 1u);
            b_lo[j] = g.B.w_lo[beo + j];
            b_hi[j] = g.B.w_hi[beo + j];
            b_inf[j] = idx | ((lb & 0x7FFFu) << 16) | (ch << 31);
        }
        for (uint32_t lp = tid; lp < LP; lp += kMulBlock) {
            const uint64_t slot = clo + base + lp;
            ztag[lp] = layer_ztag(g.canon_tag, g.nonces[2 * slot], g.nonces[2 * slot + 1]);
        }
        __syncthreads();
        if (misc[MISC_FLAG]) {   // invalid references: reject the pair (reference behaviour is UB)
            __syncthreads();
            if (tid == 0) {
                g.pair_status[pr] = 2;
                g.C.l_cnt[pr] = 0;
                g.C.e_cnt[pr] = 0;
                misc[MISC_FLAG] = 0;
            }
            __syncthreads();
            continue;
        }

        // ---- S1: all |A.E||B.E| products into LDS limb accumulators + first-insert times
        for (uint32_t t = tid; t < n; t += kMulBlock) {
            const uint32_t i = t / nB, j = t - i * nB;
            const uint32_t ai = a_inf[i], bj = b_inf[j];
            const uint32_t la = (ai >> 16) & 0x7FFFu, lb = (bj >> 16) & 0x7FFFu;
            uint32_t r = (ai & 0xFFFFu) + (bj & 0xFFFFu);
            r = r >= Bm ? r - Bm : r;
            const uint32_t s = (la * LB + lb) * Bm + r;
            const uint32_t chn = (ai ^ bj) >> 31;   // 0 = P (same sign), 1 = M
            const fp prod = fp_mul(fp{a_lo[i], a_hi[i]}, fp{b_lo[j], b_hi[j]});
            uint64_t l0, l1, l2;
            fp_split3(prod, l0, l1, l2);
            unsigned long long* q = acc + (size_t)(s * 2 + chn) * 3;
            atomicAdd(q + 0, (unsigned long long)l0);
            atomicAdd(q + 1, (unsigned long long)l1);
            atomicAdd(q + 2, (unsigned long long)l2);
            atomicMin(&tkey[s], t);
        }
        __syncthreads();

        // ---- S2a: fold owned slots into registers, clear their limbs
        fp sumP[kMulSlots], sumM[kMulSlots];
        uint32_t tk[kMulSlots], ebits[kMulSlots];
#pragma unroll
        for (int k = 0; k < kMulSlots; ++k) {
            const uint32_t s = tid + k * kMulBlock;
            tk[k] = kTInf;
            ebits[k] = 0;
            sumP[k] = fp{0, 0};
            sumM[k] = fp{0, 0};
            if (s < KS) {
                tk[k] = tkey[s];
                if (tk[k] != kTInf) {
                    unsigned long long* q = acc + (size_t)s * 6;
                    sumP[k] = fp_fold3(q[0], q[1], q[2]);
                    sumM[k] = fp_fold3(q[3], q[4], q[5]);
                    ebits[k] = (fp_nonzero(sumP[k]) ? 1u : 0u) | (fp_nonzero(sumM[k]) ? 2u : 0u);
                    q[0] = 0; q[1] = 0; q[2] = 0; q[3] = 0; q[4] = 0; q[5] = 0;
                }
            }
        }
        __syncthreads();

        // ---- S2b: bucket chains (scratch over the now-zero accumulator region)
        uint32_t* G = heads + nbk;
        uint32_t* nxt = G + n;
        uint32_t bk[kMulSlots];
#pragma unroll
        for (int k = 0; k < kMulSlots; ++k) {
            const uint32_t s = tid + k * kMulBlock;
            bk[k] = 0;
            if (tk[k] != kTInf) {
                const uint32_t lp = s / Bm, idx = s - lp * Bm;
                const uint64_t key = ((uint64_t)lp << 32) | idx;
                bk[k] = (uint32_t)((key * kGolden) % (uint64_t)nbk);   // std::hash -> bucket
                const uint32_t prev = atomicExch(&heads[bk[k]], s + 1);
                nxt[s] = prev | (ebits[k] << 30);
                if (ebits[k]) atomicOr(lp_used, 1ull << lp);
            }
        }
        __syncthreads();

        // ---- S2c: walk chains: bucket first-insert time, rank inside the bucket, group sizes
        uint32_t tb[kMulSlots], within[kMulSlots];
#pragma unroll
        for (int k = 0; k < kMulSlots; ++k) {
            tb[k] = 0;
            within[k] = 0;
            if (tk[k] != kTInf) {
                uint32_t q = heads[bk[k]], tmin = tk[k], w = 0, E = 0;
                while (q) {
                    const uint32_t s2 = q - 1;
                    const uint32_t t2 = tkey[s2];
                    const uint32_t nx = nxt[s2];
                    const uint32_t e2 = __popc(nx >> 30);
                    tmin = t2 < tmin ? t2 : tmin;
                    w += t2 > tk[k] ? e2 : 0u;
                    E += e2;
                    q = nx & 0x3FFFFFFFu;
                }
                tb[k] = tmin;
                within[k] = w;
                if (tmin == tk[k]) G[tmin] = E;
            }
        }
        // layer bookkeeping: compact_layers over C.L (encrypt.hpp:73-104), one lane
        if (tid == 0) {
            const unsigned long long used_lp = *lp_used;
            const uint32_t Lc = base + LP;
            uint64_t keep = 0;   // Lc <= 64
            for (uint32_t lp = 0; lp < LP; ++lp)
                if ((used_lp >> lp) & 1ull) keep |= 1ull << (base + lp);
            bool grew = true;
            while (grew) {
                grew = false;
                for (uint32_t l = 0; l < Lc; ++l) {
                    if (!((keep >> l) & 1ull)) continue;
                    uint32_t rule, pa, pb;
                    if (l < LA) {
                        const pvac_layer& x = g.A.layers[g.A.l_off[pr] + l];
                        rule = x.rule; pa = x.pa; pb = x.pb;
                    } else if (l < base) {
                        const pvac_layer& x = g.B.layers[g.B.l_off[pr] + (l - LA)];
                        rule = x.rule; pa = x.pa + LA; pb = x.pb + LA;
                    } else {
                        rule = 1; pa = (l - base) / LB; pb = LA + (l - base) % LB;
                    }
                    if (rule != 1) continue;
                    if (pa < Lc && !((keep >> pa) & 1ull)) { keep |= 1ull << pa; grew = true; }
                    if (pb < Lc && !((keep >> pb) & 1ull)) { keep |= 1ull << pb; grew = true; }
                }
            }
            const bool all = __popcll(keep) == Lc;
            uint32_t nl = 0;
            for (uint32_t l = 0; l < Lc; ++l) remap[l] = ((keep >> l) & 1ull) ? nl++ : 0xFFFFFFFFu;
            for (uint32_t l = 0; l < Lc; ++l) {
                if (!((keep >> l) & 1ull)) continue;
                pvac_layer y;
                if (l < LA) {
                    y = g.A.layers[g.A.l_off[pr] + l];
                } else if (l < base) {
                    y = g.B.layers[g.B.l_off[pr] + (l - LA)];
                    if (y.rule == 1) { y.pa += LA; y.pb += LA; }
                } else {
                    const uint32_t lp = l - base;
                    const uint64_t slot = clo + l;
                    y.rule = 1; y.pad = 0;
                    y.pa = lp / LB; y.pb = LA + lp % LB;
                    y.nonce_lo = g.nonces[2 * slot];
                    y.nonce_hi = g.nonces[2 * slot + 1];
                    y.ztag = ztag[lp];
                }
                if (!all && y.rule == 1) {
                    y.pa = y.pa < Lc ? remap[y.pa] : 0xFFFFFFFFu;
                    y.pb = y.pb < Lc ? remap[y.pb] : 0xFFFFFFFFu;
                }
                g.C.layers[clo + remap[l]] = y;
            }
            g.C.l_cnt[pr] = nl;
        }
        __syncthreads();

        // ---- S3: exclusive SUFFIX scan of G over t in [0, n): emit offset of each bucket group
        {
            const uint32_t per = (n + kMulBlock - 1) / kMulBlock;
            // thread c owns reversed positions r in [c*per, (c+1)*per); t = n-1-r
            const uint32_t r0 = tid * per;
            uint32_t local = 0;
            for (uint32_t r = r0; r < r0 + per && r < n; ++r) local += G[n - 1 - r];
            uint32_t total;
            uint32_t run = block_exclusive_scan<kMulBlock>(local, misc + MISC_PART, total);
            for (uint32_t r = r0; r < r0 + per && r < n; ++r) {
                const uint32_t t = n - 1 - r;
                const uint32_t v = G[t];
                G[t] = run;   // number of edges emitted before every group with t_bkt > t ... exclusive
                run += v;
            }
            if (tid == 0) misc[MISC_TOTAL] = total;
        }
        __syncthreads();

        // ---- S4: write edges at their emit positions
        const uint32_t total = misc[MISC_TOTAL];
        // guard_budget (encrypt.hpp:106-111): above edge_budget the reference runs
        // compact_edges, whose output is (layer, idx, P before M) order; product edges are
        // already unique per (layer, idx, ch) and nonzero, so it only re-orders them.
        const bool canonical = (g.flags & PVAC_MUL_ORDER_CANONICAL) != 0 || total > g.edge_budget;
        uint32_t rowbase = 0;
#pragma unroll
        for (int k = 0; k < kMulSlots; ++k) {
            uint32_t pos = 0;
            if (canonical) {   // block-uniform branch: slot order s = tid + k*BS
                uint32_t rowtot;
                pos = rowbase + block_exclusive_scan<kMulBlock>(__popc(ebits[k]), misc + MISC_PART, rowtot);
                rowbase += rowtot;
            } else {
                pos = G[tb[k]] + within[k];
            }
            if (ebits[k]) {
                const uint32_t s = tid + k * kMulBlock;
                const uint32_t lp = s / Bm, idx = s - lp * Bm;
                const uint32_t lid = remap[base + lp];
                const uint32_t hpos = G[tb[k]] + within[k];   // hash-order index (salt stream position)
                if (ebits[k] & 1u) {
                    g.C.meta[ceo + pos] = make_meta(lid, idx, 0);
                    g.C.w_lo[ceo + pos] = sumP[k].lo;
                    g.C.w_hi[ceo + pos] = sumP[k].hi;
                    if (g.salt_pos) g.salt_pos[ceo + pos] = hpos;
                    ++pos;
                }
                if (ebits[k] & 2u) {
                    g.C.meta[ceo + pos] = make_meta(lid, idx, 1);
                    g.C.w_lo[ceo + pos] = sumM[k].lo;
                    g.C.w_hi[ceo + pos] = sumM[k].hi;
                    if (g.salt_pos) g.salt_pos[ceo + pos] = hpos + (ebits[k] & 1u);
                }
            }
        }
        if (tid == 0) {
            g.C.e_cnt[pr] = total;
            g.pair_status[pr] = canonical ? 1 : 0;
            *lp_used = 0ull;
        }
        __syncthreads();
        // clear scratch (heads/G/nxt live in the accumulator region) and first-insert times
        for (uint32_t w = tid; w < nbk + n + KS; w += kMulBlock) heads[w] = 0;
#pragma unroll
        for (int k = 0; k < kMulSlots; ++k) {
            const uint32_t s = tid + k * kMulBlock;
            if (tk[k] != kTInf) tkey[s] = kTInf;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- ct_add / ct_sub
constexpr int kAddBlock = 256;

__global__ __launch_bounds__(kAddBlock) void k_ct_add(pvac_ct_batch A, pvac_ct_batch B, pvac_ct_batch C, int negate_b,
                                                     uint32_t lds_layers) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint32_t* keep = (uint32_t*)lds;                 // [lds_layers] then remap in place
    __shared__ uint32_t flags[4];
    __shared__ uint32_t part[kAddBlock / 64];
    const uint64_t pr = blockIdx.x;
    if (pr >= A.n) return;
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
        C.meta[ceo + e] = m;
        C.w_lo[ceo + e] = wl;
        C.w_hi[ceo + e] = wh;
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

}  // namespace

// ==================================================================== launch wrappers
hipError_t launch_plan_mul(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, uint8_t* pair_class,
                           plan_stats* stats, const uint32_t* nb_table, uint32_t nb_len, uint32_t Bm,
                           uint32_t ks_small_max, uint32_t prod_small_max, hipStream_t st) {
    if (!A.n) return hipSuccess;
    if (ks_small_max > kSmallKeysMax) ks_small_max = kSmallKeysMax;
    hipLaunchKernelGGL(k_plan_mul, dim3((unsigned)((A.n + kPlanBlock - 1) / kPlanBlock)), dim3(kPlanBlock), 0, st, A,
                       B, C, pair_class, stats, nb_table, nb_len, Bm, ks_small_max, prod_small_max);
    return hipGetLastError();
}

hipError_t launch_plan_add(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, plan_stats* stats,
                           hipStream_t st) {
    if (!A.n) return hipSuccess;
    hipLaunchKernelGGL(k_plan_add, dim3((unsigned)((A.n + kPlanBlock - 1) / kPlanBlock)), dim3(kPlanBlock), 0, st, A,
                       B, C, stats);
    return hipGetLastError();
}

size_t scan_scratch_words(size_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

hipError_t launch_exclusive_scan_u64(uint64_t* data, size_t n, uint64_t* scratch, unsigned long long* total_out,
                                     hipStream_t st) {
    if (!n) return hipSuccess;
    const size_t tiles = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)tiles), dim3(kScanBlock), 0, st, data, n, scratch);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kScanBlock), 0, st, scratch, tiles, total_out);
    hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)tiles), dim3(kScanBlock), 0, st, data, n, scratch);
    return hipGetLastError();
}

hipError_t launch_ct_mul_small(const mul_small_args& a, int num_cus, hipStream_t st, int* blocks_used) {
    if (!a.A.n) return hipSuccess;
    if (a.ks_max > kSmallKeysMax) return hipErrorInvalidValue;
    const mul_lds_layout L = mul_layout(a.ks_max, a.na_max, a.nb_max);
    // scratch (heads|G|nxt) must fit inside the accumulator region
    if ((uint64_t)(a.buckets_max + a.prod_max + a.ks_max) * 4u > (uint64_t)a.ks_max * 48u) return hipErrorInvalidValue;
    if (L.total > 160u * 1024u) return hipErrorInvalidValue;
    const int per_cu = L.total <= 80u * 1024u ? 2 : 1;
    uint64_t blocks = (uint64_t)num_cus * per_cu;
    if (blocks > a.A.n) blocks = a.A.n;
    if (blocks_used) *blocks_used = (int)blocks;
    hipLaunchKernelGGL(k_ct_mul_small, dim3((unsigned)blocks), dim3(kMulBlock), L.total, st, a, L);
    return hipGetLastError();
}

hipError_t launch_ct_add(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, int negate_b,
                         uint32_t max_layers, hipStream_t st) {
    if (!A.n) return hipSuccess;
    const size_t lds = ((size_t)max_layers * 4 + 15) & ~(size_t)15;
    if (lds > 120 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ct_add, dim3((unsigned)A.n), dim3(kAddBlock), lds, st, A, B, C, negate_b, max_layers);
    return hipGetLastError();
}

}  // namespace pvhip
