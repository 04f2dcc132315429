// k_mul_fresh.hip — batched ct_mul for fresh-shaped pairs (reference ops/arithmetic.hpp:47-106).
//
// Per pair C = A * B:
//   layers : C.L = A.L ++ B.L (PROD pa/pb += |A.L|) ++ |A.L||B.L| new PROD layers with caller
//            nonces and ztag = SHA-256 layer tag (crypto/matrix.hpp:254-264)
//   weights: for every (i in A.E, j in B.E): slot (la*LB+lb, (idx_i+idx_j) mod B), channel P
//            if ch_i == ch_j else M, acc += fp_mul(w_i, w_j)
//   order  : the reference iterates a std::unordered_map reserved for |A.E||B.E| keys.
//            libstdc++ links a new node first in its bucket when the bucket is non-empty and
//            at the list front when it is empty, so iteration order is (bucket first-insert
//            time DESC, key first-insert time DESC), where a key's first-insert time is
//            t = i*|B.E| + j of its first product. Reproduced exactly: per-key t via LDS
//            atomicMin, bucket chains via LDS atomicExch, a suffix scan over t, no hash table.
//   then guard_budget / compact_layers (ops/encrypt.hpp:73-111).
//
// Two launches:
//   k_mul_layers_fresh : one lane per pair writes the |C.L| layer records in identity
//                        placement, product-layer ztags included (one SHA-256 block each),
//                        so no SHA work sits on the aggregation kernel's critical path.
//   k_ct_mul_fresh     : one 256-thread workgroup per pair, persistent over the batch, ~72 KB
//                        LDS (two workgroups per CU). Sums are exact: every canonical product
//                        is split into 43/42/42-bit limbs accumulated with ds_add_u64 (order
//                        independent, no overflow below 2^21 addends). compact_layers is a
//                        wave-wide bitmask closure over LDS-resident parent masks; edges are
//                        staged in LDS at their emit positions and written out coalesced.
#include <cstdlib>

#include "common.hpp"
#include "sha256.hpp"

namespace pvhip {

namespace {

constexpr uint32_t kTInf = 0xFFFFFFFFu;
static_assert(kFreshLayersMax <= 64, "layer masks are u64");

// ---------------------------------------------------------------- layer records
constexpr int kLayBlock = 128;

__global__ __launch_bounds__(kLayBlock) void k_mul_layers_fresh(mul_fresh_args g) {
    const uint64_t pr = (uint64_t)blockIdx.x * kLayBlock + threadIdx.x;
    if (pr >= g.A.n || g.pair_class[pr] != PAIR_SMALL) return;
    const uint32_t LA = (uint32_t)g.A.l_cnt[pr], LB = (uint32_t)g.B.l_cnt[pr];
    const uint64_t alo = g.A.l_off[pr], blo = g.B.l_off[pr], clo = g.C.l_off[pr];
    for (uint32_t l = 0; l < LA; ++l) g.C.layers[clo + l] = g.A.layers[alo + l];
    for (uint32_t l = 0; l < LB; ++l) {
        pvac_layer y = g.B.layers[blo + l];
        if (y.rule == 1) { y.pa += LA; y.pb += LA; }
        g.C.layers[clo + LA + l] = y;
    }
    const uint32_t base = LA + LB, LP = LA * LB;
    for (uint32_t lp = 0; lp < LP; ++lp) {
        const uint64_t slot = clo + base + lp;
        pvac_layer y;
        y.rule = 1;
        y.pa = lp / LB;
        y.pb = LA + lp % LB;
        y.pad = 0;
        y.nonce_lo = g.nonces[2 * slot];
        y.nonce_hi = g.nonces[2 * slot + 1];
        y.ztag = layer_ztag(g.canon_tag, y.nonce_lo, y.nonce_hi);
        g.C.layers[slot] = y;
    }
}

// ---------------------------------------------------------------- aggregation + emit
struct fresh_layout {
    // byte offsets into dynamic LDS
    uint32_t acc, tkey, a_w, a_inf, b_w, b_inf, pm, remap, misc, total;
};

__host__ __device__ inline uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ inline fresh_layout fresh_lds(uint32_t ks, uint32_t na, uint32_t nb) {
    fresh_layout L;
    uint32_t o = 0;
    L.acc = o;   o = align16(o + ks * 48u);           // 2 channels x 3 u64 limbs per key slot
    L.tkey = o;  o = align16(o + ks * 4u);
    L.a_w = o;   o = align16(o + na * 16u);
    L.a_inf = o; o = align16(o + na * 4u);
    L.b_w = o;   o = align16(o + nb * 16u);
    L.b_inf = o; o = align16(o + nb * 4u);
    L.pm = o;    o = align16(o + kFreshLayersMax * 8u);   // parent masks of C's layers
    L.remap = o; o = align16(o + kFreshLayersMax * 4u);
    L.misc = o;  o = align16(o + 32u * 4u);
    L.total = o;
    return L;
}

// misc u32 word indices
enum : int { MF_PART = 0 /* <= 8 scan partials */, MF_INVALID = 8, MF_TOTAL = 9, MF_IDENT = 10,
             MF_KEEP = 12 /* u64 */, MF_WAVELP = 16 /* 8 x u64 */ };

__device__ __forceinline__ uint64_t wave_or_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t lo = __shfl_xor((uint32_t)v, d, 64);
        const uint32_t hi = __shfl_xor((uint32_t)(v >> 32), d, 64);
        v |= (uint64_t)lo | ((uint64_t)hi << 32);
    }
    return v;
}

// Per-pair header (workgroup-uniform). pr == kNoPair ends the persistent loop.
constexpr uint64_t kNoPair = ~0ull;
struct fresh_hdr {
    uint64_t pr;
    uint32_t LA, LB, nA, nB;
    uint64_t aeo, beo, alo, blo, clo, ceo;
};

__device__ __forceinline__ uint64_t next_small(const mul_fresh_args& g, uint64_t from) {
    for (uint64_t q = from; q < g.A.n; q += gridDim.x)
        if (g.pair_class[q] == PAIR_SMALL) return q;
    return kNoPair;
}

__device__ __forceinline__ fresh_hdr load_hdr(const mul_fresh_args& g, uint64_t pr) {
    fresh_hdr h{};
    h.pr = pr;
    if (pr != kNoPair) {
        h.LA = (uint32_t)g.A.l_cnt[pr]; h.LB = (uint32_t)g.B.l_cnt[pr];
        h.nA = (uint32_t)g.A.e_cnt[pr]; h.nB = (uint32_t)g.B.e_cnt[pr];
        h.aeo = g.A.e_off[pr]; h.beo = g.B.e_off[pr];
        h.alo = g.A.l_off[pr]; h.blo = g.B.l_off[pr];
        h.clo = g.C.l_off[pr]; h.ceo = g.C.e_off[pr];
    }
    return h;
}

// Next pair's inputs held in registers while the current pair is ordered and written:
// thread t owns A edge t, B edge t and C layer t (nA, nB <= 256 <= BS, Lc <= 64).
struct fresh_pref {
    uint64_t am, awl, awh, bm, bwl, bwh, pmv;
};

template <int BS>
__device__ __forceinline__ fresh_pref prefetch_pair(const mul_fresh_args& g, const fresh_hdr& h) {
    fresh_pref f{};
    const uint32_t t = threadIdx.x;
    if (h.pr == kNoPair) return f;
    if (t < h.nA) { f.am = g.A.meta[h.aeo + t]; f.awl = g.A.w_lo[h.aeo + t]; f.awh = g.A.w_hi[h.aeo + t]; }
    if (t < h.nB) { f.bm = g.B.meta[h.beo + t]; f.bwl = g.B.w_lo[h.beo + t]; f.bwh = g.B.w_hi[h.beo + t]; }
    const uint32_t base = h.LA + h.LB, Lc = base + h.LA * h.LB;
    if (t < base) {   // rule/pa/pb of the input layers (compact_layers parents)
        const pvac_layer& x = t < h.LA ? g.A.layers[h.alo + t] : g.B.layers[h.blo + (t - h.LA)];
        f.pmv = ((uint64_t)x.rule << 63) | ((uint64_t)x.pb << 32) | x.pa;
    } else if (t < Lc) {
        f.pmv = 0;
    }
    return f;
}

// registers -> LDS staging of one pair; flags invalid references in misc[MF_INVALID]
template <int BS>
__device__ __forceinline__ void stage_pair(const fresh_pref& f, const fresh_hdr& h, uint32_t Bm, ulonglong2* a_w,
                                           uint32_t* a_inf, ulonglong2* b_w, uint32_t* b_inf, uint64_t* pm,
                                           uint32_t* misc) {
    const uint32_t t = threadIdx.x;
    if (h.pr == kNoPair) return;
    if (t < h.nA) {
        const uint32_t la = meta_layer(f.am), idx = meta_idx(f.am), ch = meta_ch(f.am);
        if (la >= h.LA || idx >= Bm || ch > 1) misc[MF_INVALID] = 1;
        a_w[t] = make_ulonglong2(f.awl, f.awh);
        a_inf[t] = idx | ((la & 0x7FFFu) << 16) | (ch << 31);
    }
    if (t < h.nB) {
        const uint32_t lb = meta_layer(f.bm), idx = meta_idx(f.bm), ch = meta_ch(f.bm);
        if (lb >= h.LB || idx >= Bm || ch > 1) misc[MF_INVALID] = 1;
        b_w[t] = make_ulonglong2(f.bwl, f.bwh);
        b_inf[t] = idx | ((lb & 0x7FFFu) << 16) | (ch << 31);
    }
    const uint32_t base = h.LA + h.LB, Lc = base + h.LA * h.LB;
    if (t < Lc) {
        uint64_t m = 0;
        if (t < base) {
            if (f.pmv >> 63) {   // PROD: parents, B's shifted by |A.L| (arithmetic.hpp:54-57)
                const uint32_t off = t < h.LA ? 0u : h.LA;
                const uint32_t pa = (uint32_t)f.pmv + off, pb = (uint32_t)(f.pmv >> 32) + off;
                m = (pa < Lc ? 1ull << pa : 0ull) | (pb < Lc ? 1ull << pb : 0ull);
            }
        } else {
            const uint32_t lp = t - base;
            m = (1ull << (lp / h.LB)) | (1ull << (h.LA + lp % h.LB));
        }
        pm[t] = m;
    }
}

template <int BS, int MINW>
__global__ __launch_bounds__(BS, MINW) void k_ct_mul_fresh(mul_fresh_args g, fresh_layout Ls) {
    constexpr int FS = kFreshKeysMax / BS;               // key slots owned per thread
    constexpr int NW = BS / 64;
    static_assert(FS * BS == (int)kFreshKeysMax && BS >= (int)kFreshEdgesMax && NW <= 8, "fresh geometry");
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    unsigned long long* acc = (unsigned long long*)(lds + Ls.acc);
    uint32_t* accw = (uint32_t*)(lds + Ls.acc);           // u32 view: heads | G | nxt, then staging
    uint32_t* tkey = (uint32_t*)(lds + Ls.tkey);
    ulonglong2* a_w = (ulonglong2*)(lds + Ls.a_w);
    uint32_t* a_inf = (uint32_t*)(lds + Ls.a_inf);
    ulonglong2* b_w = (ulonglong2*)(lds + Ls.b_w);
    uint32_t* b_inf = (uint32_t*)(lds + Ls.b_inf);
    uint64_t* pm = (uint64_t*)(lds + Ls.pm);
    uint32_t* remap = (uint32_t*)(lds + Ls.remap);
    uint32_t* misc = (uint32_t*)(lds + Ls.misc);
    uint64_t* wave_lp = (uint64_t*)(misc + MF_WAVELP);     // per-wave OR of used product layers

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const uint32_t Bm = g.Bm;
    const uint32_t acc_vec = g.ks_max * 3u;               // 16-byte vectors in the accumulator region

    // one-time clear: accumulators 0, first-insert times INF
    for (uint32_t w = tid; w < acc_vec; w += BS) ((uint4*)accw)[w] = make_uint4(0, 0, 0, 0);
    for (uint32_t s = tid; s < g.ks_max; s += BS) tkey[s] = kTInf;
    if (tid < 32) misc[tid] = 0;
    __syncthreads();

    fresh_hdr cur = load_hdr(g, next_small(g, blockIdx.x));
    stage_pair<BS>(prefetch_pair<BS>(g, cur), cur, Bm, a_w, a_inf, b_w, b_inf, pm, misc);
    __syncthreads();

    while (cur.pr != kNoPair) {
        const fresh_hdr nxt = load_hdr(g, next_small(g, cur.pr + gridDim.x));
        const uint64_t pr = cur.pr;
        const uint32_t LA = cur.LA, LB = cur.LB, nA = cur.nA, nB = cur.nB;
        const uint32_t LP = LA * LB, KS = LP * Bm, n = nA * nB;
        const uint32_t base = LA + LB, Lc = base + LP;
        const uint32_t nbk = g.nb_table[n];
        const fastmod64 fm{nbk, g.nb_magic[n]};
        const uint64_t clo = cur.clo, ceo = cur.ceo;

        if (misc[MF_INVALID]) {   // invalid references: reject the pair (reference behaviour is UB)
            __syncthreads();
            if (tid == 0) {
                g.pair_status[pr] = 2;
                g.C.l_cnt[pr] = 0;
                g.C.e_cnt[pr] = 0;
                misc[MF_INVALID] = 0;
            }
            __syncthreads();
            stage_pair<BS>(prefetch_pair<BS>(g, nxt), nxt, Bm, a_w, a_inf, b_w, b_inf, pm, misc);
            __syncthreads();
            cur = nxt;
            continue;
        }

        // ---- S1: all |A.E||B.E| products into LDS limb accumulators + first-insert times.
        //      Thread (j, g0) keeps B edge j in registers and walks A edges g0, g0 + G, ...
        if (n) {
            const uint32_t groups = BS / nB;
            const uint32_t j = (uint32_t)tid % nB, g0 = (uint32_t)tid / nB;
            if (g0 < groups) {
                const uint32_t bj = b_inf[j];
                const ulonglong2 y = b_w[j];
                const fp yb{y.x, y.y};
                const uint32_t lb = (bj >> 16) & 0x7FFFu, ib = bj & 0xFFFFu;
                for (uint32_t i = g0; i < nA; i += groups) {
                    const uint32_t ai = a_inf[i];
                    const ulonglong2 x = a_w[i];
                    const uint32_t la = (ai >> 16) & 0x7FFFu;
                    uint32_t r = (ai & 0xFFFFu) + ib;
                    r = r >= Bm ? r - Bm : r;
                    const uint32_t s = (la * LB + lb) * Bm + r;
                    const uint32_t chn = (ai ^ bj) >> 31;   // 0 = P (same sign), 1 = M
                    const fp prod = fp_mul(fp{x.x, x.y}, yb);
                    uint64_t l0, l1, l2;
                    fp_split3(prod, l0, l1, l2);
                    unsigned long long* q = acc + (size_t)(s * 2 + chn) * 3;
                    atomicAdd(q + 0, (unsigned long long)l0);
                    atomicAdd(q + 1, (unsigned long long)l1);
                    atomicAdd(q + 2, (unsigned long long)l2);
                    atomicMin(&tkey[s], i * nB + j);
                }
            }
        }
        __syncthreads();
        // next pair's inputs: loads in flight across S2a..S5, staged after the copy-out
        const fresh_pref pf = prefetch_pair<BS>(g, nxt);

        // ---- S2a: fold owned slots into registers, clear their limbs, bucket of each key
        fp sumP[FS], sumM[FS];
        uint32_t tk[FS], eb[FS], bk[FS];
        uint64_t myor = 0;
#pragma unroll
        for (int k = 0; k < FS; ++k) {
            const uint32_t s = tid + k * BS;
            tk[k] = kTInf;
            eb[k] = 0;
            bk[k] = 0;
            sumP[k] = fp{0, 0};
            sumM[k] = fp{0, 0};
            if (s < KS) {
                tk[k] = tkey[s];
                if (tk[k] != kTInf) {
                    unsigned long long* q = acc + (size_t)s * 6;
                    sumP[k] = fp_fold3(q[0], q[1], q[2]);
                    sumM[k] = fp_fold3(q[3], q[4], q[5]);
                    eb[k] = (fp_nonzero(sumP[k]) ? 1u : 0u) | (fp_nonzero(sumM[k]) ? 2u : 0u);
                    q[0] = 0; q[1] = 0; q[2] = 0; q[3] = 0; q[4] = 0; q[5] = 0;
                    const uint32_t lp = s / Bm, idx = s - lp * Bm;
                    const uint64_t key = ((uint64_t)lp << 32) | idx;
                    bk[k] = (uint32_t)fmod64(key * kGolden, fm);   // std::hash -> bucket
                    if (eb[k]) myor |= 1ull << lp;
                }
            }
        }
        myor = wave_or_u64(myor);
        if (lane == 0) wave_lp[wave] = myor;
        __syncthreads();

        // ---- S2b: bucket chains over the (now all-zero) accumulator region
        uint32_t* heads = accw;
        uint32_t* G = heads + nbk;
        uint32_t* nxtl = G + n;
#pragma unroll
        for (int k = 0; k < FS; ++k) {
            if (tk[k] != kTInf) {
                const uint32_t s = tid + k * BS;
                const uint32_t prev = atomicExch(&heads[bk[k]], s + 1);
                nxtl[s] = prev | (eb[k] << 30);
            }
        }
        __syncthreads();

        // ---- S2c: walk chains -> bucket first-insert time, rank inside the bucket, group sizes;
        //      wave 0 then runs compact_layers (encrypt.hpp:73-104) as a bitmask closure
        uint32_t tb[FS], within[FS];
#pragma unroll
        for (int k = 0; k < FS; ++k) {
            tb[k] = 0;
            within[k] = 0;
            if (tk[k] != kTInf) {
                uint32_t q = heads[bk[k]], tmin = tk[k], w = 0, E = 0;
                while (q) {
                    const uint32_t s2 = q - 1;
                    const uint32_t t2 = tkey[s2];
                    const uint32_t nx = nxtl[s2];
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
        if (wave == 0) {
            const uint64_t all = Lc >= 64 ? ~0ull : ((1ull << Lc) - 1ull);
            uint64_t used_lp = 0;
#pragma unroll
            for (int w = 0; w < NW; ++w) used_lp |= wave_lp[w];
            uint64_t keep = (used_lp << base) & all;
            const uint64_t mypm = (uint32_t)lane < Lc ? pm[lane] : 0ull;
            for (;;) {   // transitive parents of used product layers; depth-bounded by Lc
                const uint64_t par = wave_or_u64(((keep >> lane) & 1ull) ? mypm : 0ull);
                const uint64_t nk = keep | par;
                if (nk == keep) break;
                keep = nk;
            }
            if ((uint32_t)lane < Lc)
                remap[lane] = ((keep >> lane) & 1ull) ? (uint32_t)__popcll(keep & ((1ull << lane) - 1ull)) : kTInf;
            if (lane == 0) {
                *(uint64_t*)(misc + MF_KEEP) = keep;
                misc[MF_IDENT] = keep == all;
            }
        }
        __syncthreads();

        // ---- S3: exclusive SUFFIX scan of G over t in [0, n): emit offset of each bucket group
        {
            const uint32_t per = (n + BS - 1) / BS;
            const uint32_t r0 = tid * per;   // reversed positions r in [r0, r0 + per), t = n-1-r
            uint32_t local = 0;
            for (uint32_t r = r0; r < r0 + per && r < n; ++r) local += G[n - 1 - r];
            uint32_t total;
            uint32_t run = block_exclusive_scan<BS>(local, misc + MF_PART, total);
            for (uint32_t r = r0; r < r0 + per && r < n; ++r) {
                const uint32_t t = n - 1 - r;
                const uint32_t v = G[t];
                G[t] = run;
                run += v;
            }
            if (tid == 0) misc[MF_TOTAL] = total;
        }
        __syncthreads();

        // ---- S4: emit positions into registers; reset first-insert times
        const uint32_t total = misc[MF_TOTAL];
        // guard_budget (encrypt.hpp:106-111): above edge_budget the reference runs compact_edges,
        // whose output is (layer, idx, P before M) order; product edges are already unique per
        // (layer, idx, ch) and nonzero, so it only re-orders them.
        const bool canonical = (g.flags & PVAC_MUL_ORDER_CANONICAL) != 0 || total > g.edge_budget;
        uint32_t pos[FS], hpos[FS];
        uint32_t rowbase = 0;
#pragma unroll
        for (int k = 0; k < FS; ++k) {
            hpos[k] = G[tb[k]] + within[k];
            if (canonical) {   // workgroup-uniform: slot order s = tid + k*BS
                uint32_t rowtot;
                pos[k] = rowbase + block_exclusive_scan<BS>(__popc(eb[k]), misc + MF_PART, rowtot);
                rowbase += rowtot;
            } else {
                pos[k] = hpos[k];
            }
            if (tk[k] != kTInf) tkey[tid + k * BS] = kTInf;
        }
        __syncthreads();

        // ---- S4b: stage edge records at their emit positions (over heads/G/nxt, now dead)
        uint64_t* st_meta = (uint64_t*)accw;
        uint64_t* st_lo = st_meta + total;
        uint64_t* st_hi = st_lo + total;
#pragma unroll
        for (int k = 0; k < FS; ++k) {
            if (eb[k]) {
                const uint32_t s = tid + k * BS;
                const uint32_t lp = s / Bm, idx = s - lp * Bm;
                const uint32_t lid = remap[base + lp];
                uint32_t p = pos[k];
                if (canonical && g.salt_pos) {   // salts are drawn in hash order (arithmetic.hpp:90-101)
                    g.salt_pos[ceo + p] = hpos[k];
                    if (eb[k] == 3u) g.salt_pos[ceo + p + 1] = hpos[k] + 1;
                }
                if (eb[k] & 1u) {
                    st_meta[p] = make_meta(lid, idx, 0);
                    st_lo[p] = sumP[k].lo;
                    st_hi[p] = sumP[k].hi;
                    ++p;
                }
                if (eb[k] & 2u) {
                    st_meta[p] = make_meta(lid, idx, 1);
                    st_lo[p] = sumM[k].lo;
                    st_hi[p] = sumM[k].hi;
                }
            }
        }
        __syncthreads();

        // ---- S5: coalesced copy-out, layer compaction fix-up, counts
        for (uint32_t t = tid; t < total; t += BS) {
            g.C.meta[ceo + t] = st_meta[t];
            g.C.w_lo[ceo + t] = st_lo[t];
            g.C.w_hi[ceo + t] = st_hi[t];
            if (g.salt_pos && !canonical) g.salt_pos[ceo + t] = t;
        }
        const uint64_t keep = *(const uint64_t*)(misc + MF_KEEP);
        if (!misc[MF_IDENT] && wave == 1) {
            // k_mul_layers_fresh wrote identity placement; compact in place (remap[l] <= l, and
            // every lane of this wave loads before any lane stores)
            const uint32_t l = lane;
            pvac_layer y{};
            if (l < Lc) y = g.C.layers[clo + l];
            if (l < Lc && ((keep >> l) & 1ull)) {
                if (y.rule == 1) {
                    y.pa = y.pa < Lc ? remap[y.pa] : kTInf;
                    y.pb = y.pb < Lc ? remap[y.pb] : kTInf;
                }
                g.C.layers[clo + remap[l]] = y;
            }
        }
        if (tid == 0) {
            g.C.e_cnt[pr] = total;
            g.C.l_cnt[pr] = (uint64_t)__popcll(keep);
            g.pair_status[pr] = canonical ? 1 : 0;
        }
        __syncthreads();
        // ---- clear what this pair dirtied (staging / chains), stage the next pair
        {
            const uint32_t words = max(6u * total, nbk + n + KS);
            const uint32_t vecs = (words + 3u) >> 2;
            for (uint32_t w = tid; w < vecs; w += BS) ((uint4*)accw)[w] = make_uint4(0, 0, 0, 0);
        }
        stage_pair<BS>(pf, nxt, Bm, a_w, a_inf, b_w, b_inf, pm, misc);
        __syncthreads();
        cur = nxt;
    }
}

}  // namespace

hipError_t launch_mul_layers_fresh(const mul_fresh_args& a, hipStream_t st) {
    if (!a.A.n) return hipSuccess;
    hipLaunchKernelGGL(k_mul_layers_fresh, dim3((unsigned)((a.A.n + kLayBlock - 1) / kLayBlock)), dim3(kLayBlock), 0,
                       st, a);
    return hipGetLastError();
}

hipError_t launch_ct_mul_fresh(const mul_fresh_args& a, int num_cus, hipStream_t st) {
    if (!a.A.n) return hipSuccess;
    if (a.ks_max > kFreshKeysMax || a.layers_max > kFreshLayersMax || a.na_max > kFreshEdgesMax ||
        a.nb_max > kFreshEdgesMax)
        return hipErrorInvalidValue;
    const fresh_layout L = fresh_lds(a.ks_max, a.na_max, a.nb_max);
    // chains (heads | G | nxt) and the staged edges must fit inside the accumulator region
    if ((uint64_t)(a.buckets_max + a.prod_max + a.ks_max) > (uint64_t)a.ks_max * 12u) return hipErrorInvalidValue;
    if (L.total > 160u * 1024u) return hipErrorInvalidValue;
    const int per_cu = L.total <= 80u * 1024u ? 2 : 1;
    uint64_t blocks = (uint64_t)num_cus * per_cu;
    if (blocks > a.A.n) blocks = a.A.n;
    static const int threads = [] {
        const char* e = std::getenv("PVAC_FRESH_THREADS");   // tuning knob; results are identical
        return e && std::atoi(e) == 256 ? 256 : 512;
    }();
    if (threads == 256)
        hipLaunchKernelGGL((k_ct_mul_fresh<256, 2>), dim3((unsigned)blocks), dim3(256), L.total, st, a, L);
    else
        hipLaunchKernelGGL((k_ct_mul_fresh<512, 4>), dim3((unsigned)blocks), dim3(512), L.total, st, a, L);
    return hipGetLastError();
}

}  // namespace pvhip
