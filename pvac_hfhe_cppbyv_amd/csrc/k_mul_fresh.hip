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
//   k_ct_mul_fresh3    : one 512-thread workgroup per pair, persistent over the batch, <= 53 KB
//                        LDS (three workgroups per CU). Emit positions are computed before the
//                        products; sums are exact (44/44/40-bit limbs added with ds_add_u64,
//                        order independent). compact_layers is a wave-wide bitmask closure over
//                        LDS-resident parent masks. See the phase list above the kernel.
#include <atomic>
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "common.hpp"
#include "sha256.hpp"

namespace pvhip {

// Diagnostic build only (make diag -> lib/libpvac_hip_diag.so): wave 0 of every workgroup
// accumulates s_memtime deltas per phase into a debug array; never touches kernel outputs.
#ifdef PVAC_CENSUS   // diagnostic build only: per-workgroup start / end s_memrealtime (100 MHz) + pairs done
__device__ unsigned long long g_census[4096 * 4];
extern "C" int pvac_hip_diag_census(unsigned long long* host, size_t n) {
    if (n > sizeof(g_census) / 8) n = sizeof(g_census) / 8;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_census), n * 8) == hipSuccess ? 0 : -5;
}
#endif
#ifdef PVAC_PHASE_STAMPS
constexpr int kStampPhases = 18;
__device__ unsigned long long g_fresh_stamps[4096 * kStampPhases];
#endif

namespace {

static_assert(kFreshLayersMax <= 64, "layer masks are u64");
static_assert(kFreshKeysMax <= 2048 && kFreshLayersMax <= 512, "writer entries pack slot, idx (11 bits each) and layer");

// ---------------------------------------------------------------- layer records
#ifndef PVAC_LAY_LANES   // A/B builds only
#define PVAC_LAY_LANES 4
#endif
constexpr int kLayBlock = 256;
constexpr int kLayLanes = PVAC_LAY_LANES;   // lanes per pair: output layers (and their SHA-256 ztags) split over them

__global__ __launch_bounds__(kLayBlock) void k_mul_layers_fresh(mul_fresh_args g) {
    const uint64_t pr = ((uint64_t)blockIdx.x * kLayBlock + threadIdx.x) / kLayLanes;
    const uint32_t sub = threadIdx.x % kLayLanes;
    if (pr >= g.A.n) return;
    fresh_rec rec{};
    if (g.pair_class[pr] != PAIR_SMALL) {   // nbk = 0: the aggregation kernel skips the pair
        if (sub == 0) g.recs[pr] = rec;
        return;
    }
    const uint32_t LA = (uint32_t)g.A.l_cnt[pr], LB = (uint32_t)g.B.l_cnt[pr];
    const uint64_t alo = g.A.l_off[pr], blo = g.B.l_off[pr], clo = g.C.l_off[pr];
    if (sub == 0) {
        const uint32_t nA = (uint32_t)g.A.e_cnt[pr], nB = (uint32_t)g.B.e_cnt[pr];
        rec.aeo = g.A.e_off[pr]; rec.beo = g.B.e_off[pr]; rec.ceo = g.C.e_off[pr];
        rec.alo = alo; rec.blo = blo; rec.clo = clo;
        rec.nb_magic = g.nb_magic[nA * nB];
        rec.shape = nA | (nB << 16);
        rec.nbk = (uint16_t)g.nb_table[nA * nB];
        rec.LA = (uint8_t)LA; rec.LB = (uint8_t)LB;
        g.recs[pr] = rec;
    }
    const uint32_t base = LA + LB, LP = LA * LB;
    for (uint32_t l = sub; l < base; l += kLayLanes) {
        if (l < LA) {
            g.C.layers[clo + l] = g.A.layers[alo + l];
        } else {
            pvac_layer y = g.B.layers[blo + (l - LA)];
            if (y.rule == 1) { y.pa += LA; y.pb += LA; }
            g.C.layers[clo + l] = y;
        }
    }
    for (uint32_t lp = sub; lp < LP; lp += kLayLanes) {
        const uint64_t slot = clo + base + lp;
        pvac_layer y;
        y.rule = 1;
        y.pa = lp / LB;
        y.pb = LA + lp % LB;
        y.pad = 0;
        y.nonce_lo = g.nonces[2 * slot];
        y.nonce_hi = g.nonces[2 * slot + 1];
#ifdef PVAC_EXP_NOZTAG   // timing experiment only: no SHA-256 (ztags wrong)
        y.ztag = y.nonce_lo ^ g.canon_tag;
#else
        y.ztag = layer_ztag(g.canon_tag, y.nonce_lo, y.nonce_hi);
#endif
        g.C.layers[slot] = y;
    }
}

// ---------------------------------------------------------------- aggregation + emit
// misc u32 word shared with stage_pair: invalid edge / layer references in the staged pair
// (and two words: the layers of A and of B that have edges, OR-ed by stage_pair; a product layer
// (la, lb) is used by compact_layers' closure exactly when both have edges, every product cell
// being assumed to emit, see P2. Fresh-shape pairs have |A.L| + |B.L| + |A.L||B.L| <= 64, so
// |A.L|, |B.L| <= 31)
enum : int { MF_INVALID = 16, MF_AMASK = 56, MF_BMASK = 57 };

__host__ __device__ inline uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

// Kernel arguments read through the constant address space: scalar loads (lgkmcnt only), so an
// argument read never waits on outstanding vector-memory loads.
using argp = const __attribute__((address_space(4))) mul_fresh_args*;

__device__ __forceinline__ argp launder(uint64_t v) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    asm volatile("" : "+s"(lo), "+s"(hi));
    return (argp)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ argp launder(argp p) { return launder((uint64_t)p); }


// Per-pair header (workgroup-uniform). pr == kNoPair ends the persistent loop.
constexpr uint64_t kNoPair = ~0ull;
// Only what every wave needs is decoded into registers (each decoded word costs one v_readlane
// per wave): the record's other words stay in LDS (misc[F3_HDR ..], written before the pair's
// prefetch), where prefetch_pair reads its four offsets; the rare users of clo / nb_magic read
// the record itself (scalar loads).
struct fresh_hdr {
    uint64_t pr;
    uint32_t LA, LB, nA, nB;
    uint64_t ceo;
    uint32_t nbk;        // libstdc++ bucket count after reserve(|A.E||B.E|)
};

// Header records are read through the constant address space: uniform-index reads become scalar
// loads (lgkmcnt), which never wait behind the vector-memory prefetch of the next pair.
using recp = const __attribute__((address_space(4))) fresh_rec*;

__device__ __forceinline__ uint64_t next_small(argp g, uint64_t from) {
    const recp R = (recp)g->recs;
    for (uint64_t q = from; q < g->A.n; q += gridDim.x)
        if (R[q].nbk) return q;
    return kNoPair;
}


// The next pair's header is loaded by VECTOR memory (lane l < 16 of every wave holds dword l of
// its record): its wait is vmcnt, so it never holds up an LDS wait the way a scalar load would
// (lgkmcnt counts both, and scalar loads return out of order).
__device__ __forceinline__ uint32_t hdr_issue(const fresh_rec* recs, uint64_t n_pairs, uint64_t q) {
    if (q >= n_pairs) return 0;
    return ((const uint32_t*)(recs + q))[threadIdx.x & 15u];
}

// header of pair q from its record's words (lane l & 15 holds dword l)
__device__ __forceinline__ fresh_hdr hdr_decode(uint32_t v, uint64_t q) {
    fresh_hdr h{};
    auto rd = [&](int k) { return (uint32_t)__builtin_amdgcn_readlane(v, k); };
    const uint32_t w15 = rd(15);
    h.pr = q;
    h.ceo = ((uint64_t)rd(5) << 32) | rd(4);
    const uint32_t shape = rd(14);
    h.nA = shape & 0xFFFFu;
    h.nB = shape >> 16;
    h.nbk = w15 & 0xFFFFu;
    h.LA = (w15 >> 16) & 0xFFu;
    h.LB = w15 >> 24;
    return h;
}

// The pair after q - gridDim.x: q itself when it is a fresh pair (its words v, from LDS), else the
// next fresh one, whose record every wave loads and the control wave copies into the LDS words
// (so a barrier must separate this call from the prefetch that reads them).
__device__ __forceinline__ fresh_hdr hdr_next(argp g, uint32_t v, uint64_t q, uint64_t n_pairs, uint32_t* hw) {
    fresh_hdr h{};
    h.pr = kNoPair;
    if (q >= n_pairs) return h;
    if (((uint32_t)__builtin_amdgcn_readlane(v, 15) & 0xFFFFu) != 0) return hdr_decode(v, q);
    const uint64_t q2 = next_small(g, q + gridDim.x);   // not a fresh pair (rare)
    if (q2 == kNoPair) return h;
    const uint32_t v2 = ((const uint32_t*)(g->recs + q2))[threadIdx.x & 15u];
    if ((threadIdx.x >> 6) == (blockDim.x >> 6) - 1 && (threadIdx.x & 63u) < 16) hw[threadIdx.x & 15u] = v2;
    return hdr_decode(v2, q2);
}
static_assert(offsetof(fresh_rec, nb_magic) == 48 && offsetof(fresh_rec, shape) == 56 && offsetof(fresh_rec, nbk) == 60 &&
                  offsetof(fresh_rec, LA) == 62 && offsetof(fresh_rec, LB) == 63,
              "hdr_next reads fresh_rec by dword");

// The next pair's raw inputs ride in registers while the current pair is ordered and written:
// thread t holds A edge t, B edge t and words 0..2 (rule, pa, pb) of input layer t. Nothing is
// computed from them until stage_pair, so no wait is placed on the loads before then.
struct fresh_pref {
    uint64_t am, al, ah, bm, bl, bh;
    uint32_t rule, pa, pb;
};

#ifndef PVAC_F3_PF_WAVES   // A/B builds: 0 = every wave prefetches (round 4)
#define PVAC_F3_PF_WAVES 1
#endif
__device__ __forceinline__ fresh_pref prefetch_pair(argp g, const fresh_hdr& h, const uint32_t* hw,
                                                    uint32_t t = threadIdx.x) {
    // every lane of a loading wave loads a valid address (a clamped index, or the argument block
    // itself when there is no pair / no edge), so the waitcnt pass never has to drain earlier loads
    // (or the previous pair's output stores) before issuing these; lanes past the counts ignore what
    // they loaded. Waves past the pair's edges and layers (wave-uniform: 7 of 8 for 40-edge
    // ciphers) load nothing.
    const bool live = h.pr != kNoPair;
#if PVAC_F3_PF_WAVES
    if ((t & ~63u) >= max(max(h.nA, h.nB), h.LA + h.LB)) return fresh_pref{};
#endif
    using gp64 = const __attribute__((address_space(1))) uint64_t*;   // global: never a flat load
    using gpl = const __attribute__((address_space(1))) uint32_t*;
    const gp64 dummy = (gp64)(uint64_t)g;
    const uint32_t v = hw[t & 15u];   // the pair's record words (only the loading waves decode them)
    auto rd = [&](int k) { return (uint64_t)(uint32_t)__builtin_amdgcn_readlane(v, k); };
    const uint64_t aeo = (rd(1) << 32) | rd(0), beo = (rd(3) << 32) | rd(2);
    const uint64_t alo = (rd(7) << 32) | rd(6), blo = (rd(9) << 32) | rd(8);
    const bool okA = live && h.nA, okB = live && h.nB;
    const uint64_t ea = okA ? aeo + min(t, h.nA - 1u) : 0ull;
    const uint64_t eb = okB ? beo + min(t, h.nB - 1u) : 0ull;
    const gp64 am = okA ? (gp64)g->A.meta : dummy;
    const gp64 al = okA ? (gp64)g->A.w_lo : dummy;
    const gp64 ah = okA ? (gp64)g->A.w_hi : dummy;
    const gp64 bm = okB ? (gp64)g->B.meta : dummy;
    const gp64 bl = okB ? (gp64)g->B.w_lo : dummy;
    const gp64 bh = okB ? (gp64)g->B.w_hi : dummy;
    const uint32_t nl = h.LA + h.LB;
    const uint32_t l = min(t, nl - 1u);
    const gpl rec = !(live && nl) ? (gpl)dummy
                    : l < h.LA    ? (gpl)(g->A.layers + alo + l)
                                  : (gpl)(g->B.layers + blo + (l - h.LA));
    fresh_pref f;
    f.am = am[ea]; f.al = al[ea]; f.ah = ah[ea];
    f.bm = bm[eb]; f.bl = bl[eb]; f.bh = bh[eb];
    f.rule = rec[0]; f.pa = rec[1]; f.pb = rec[2];
    return f;
}

// registers -> staged operands: validated, canonical weights (products depend only on w mod p;
// canonical operands let the lazy product skip a fold), packed (idx, layer, ch), and the
// compact_layers parent mask of every C layer. Flags invalid references in misc[MF_INVALID].
__device__ __forceinline__ void stage_pair(const fresh_pref& f, const fresh_hdr& h, uint32_t Bm, ulonglong2* a_w,
                                           uint32_t* a_inf, ulonglong2* b_w, uint32_t* b_inf, uint64_t* pm,
                                           uint32_t* misc, uint32_t t = threadIdx.x) {
    if (h.pr == kNoPair) return;
    uint32_t amask = 0, bmask = 0;
    if (t < h.nA) {
        const uint32_t la = meta_layer(f.am), idx = meta_idx(f.am), ch = meta_ch(f.am);
        if (la >= h.LA || idx >= Bm || ch > 1) misc[MF_INVALID] = 1;
        amask = la < 32u ? 1u << la : 0u;
        const fp w = fp_canon(f.al, f.ah);
        a_w[t] = make_ulonglong2(w.lo, w.hi);
        a_inf[t] = idx | ((la * h.LB * Bm) << 12) | (ch << 24);   // S1 adds A and B records (see there)
    }
    if (t < h.nB) {
        const uint32_t lb = meta_layer(f.bm), idx = meta_idx(f.bm), ch = meta_ch(f.bm);
        if (lb >= h.LB || idx >= Bm || ch > 1) misc[MF_INVALID] = 1;
        bmask = lb < 32u ? 1u << lb : 0u;
        const fp w = fp_canon(f.bl, f.bh);
        b_w[t] = make_ulonglong2(w.lo, w.hi);
        b_inf[t] = idx | ((lb * Bm) << 12) | (ch << 24);
    }
    // layer masks: one OR per wave that holds edges (wave-uniform test, so every lane takes part in
    // the reduction), one LDS atomic per mask and wave
    if ((t & ~63u) < max(h.nA, h.nB)) {
        amask = wave_or_u32(amask);
        bmask = wave_or_u32(bmask);
        if ((t & 63u) == 0) {
            if (amask) atomicOr(misc + MF_AMASK, amask);
            if (bmask) atomicOr(misc + MF_BMASK, bmask);
        }
    }
    const uint32_t base = h.LA + h.LB, Lc = base + h.LA * h.LB;
    uint32_t rule = f.rule;
    asm volatile("" : "+v"(rule));   // keep the compare here: hoisted, it waits on the prefetch
    if (t < Lc) {
        uint64_t m = 0;
        if (t < base) {
            if (rule == 1u) {   // PROD: parents, B's shifted by |A.L| (arithmetic.hpp:54-57)
                const uint32_t off = t < h.LA ? 0u : h.LA;
                const uint32_t pa = f.pa + off, pb = f.pb + off;
                m = (pa < Lc ? 1ull << pa : 0ull) | (pb < Lc ? 1ull << pb : 0ull);
            }
        } else {
            const uint32_t lp = t - base;   // < 64: lp / LB by multiply-shift (exact for lp < 2^16 / LB)
            const uint32_t la = (lp * ((65536u + h.LB - 1u) / h.LB)) >> 16;
            m = (1ull << la) | (1ull << (h.LA + lp - la * h.LB));
        }
        pm[t] = m;
    }
}


// ================================================================ k_ct_mul_fresh3
// Positions before products. Three workgroups per CU (<= 53 KB LDS, <= 80 VGPRs):
//   P1 key times : every product t = i|B.E| + j lands in cell 2 s + ch (s = key slot, ch = P/M);
//                  one ds_min_u32 per product gives each cell's first-insert time (no multiply)
//   P2 order     : slot owners read their two cells and the cells of their bucket's other slots:
//                  key time, bucket first-insert time, rank in the bucket, bucket edge count
//                  G[t_bkt]. A cell with products is assumed to emit (its sum is != 0).
//                  Slots are dealt to threads sorted by the size of their bucket (static per
//                  bucket count), so a wave loops only over as many bucket mates as it needs.
//   P3 scan      : every wave suffix-scans one 256-time segment of G; wave 0 then runs
//                  compact_layers
//   P4 positions : each emitting cell gets its hash-order emit position p (segment offset added
//                  from the segment totals); p goes into the cell word, the cell id into limb 2 of p
//   P5 products  : fp_mul of every product, 44/44/40-bit limbs added into position p's
//                  accumulators (3 ds_add_u64)
//   P6 writer    : positions p = tid, tid + 448, ... fold their limbs (coalesced LDS reads), write
//                  the edge records coalesced, clear. A folded sum of 0 (a cancelling key, or a
//                  zero weight) means the optimistic emit in P2 was wrong, and guard_budget /
//                  ORDER_CANONICAL want another order: such pairs are flagged (pair_status 3,
//                  redo list) and the host re-runs them on the general path.
// LDS word of cell c (tkey[c], u32): low half = first-insert time (0xFFFF none), then the emit
// position; high half, indexed by product time t instead: G[t], then its in-segment suffix offset.
// misc words of k_ct_mul_fresh3 (F3_INVALID is stage_pair's MF_INVALID)
enum : int { F3_PART = 0 /* 16 scan segment totals / block-scan partials */, F3_INVALID = MF_INVALID,
             F3_BIGOVF = 17, F3_IDENT = 18, F3_ZERO = 19, F3_KEEP = 20 /* u64 */,
             F3_CLS = 24 /* 8 class counters while rebuilding */, F3_WAVELP = 24 /* 8 x u64 */,
             F3_HDR = 40 /* 16: next pair's header record */, F3_AMASK = MF_AMASK, F3_BMASK = MF_BMASK,
             F3_WORDS = 60 };
static_assert(F3_AMASK == 56 && F3_BMASK == 57, "stage_pair ORs the layer masks into misc[56], misc[57]");
static_assert(F3_INVALID == 16, "stage_pair flags misc[F3_INVALID]");
constexpr uint32_t kBigCap = 256;   // LDS entries for the slots of buckets with more than 4 slots

struct fresh3_layout {
    uint32_t tkey, lim, members, a_w, a_inf, b_w, b_inf, pm, remap, misc, total;
    uint32_t tk_words, pmax, boff;
};

__host__ __device__ inline fresh3_layout fresh3_lds(uint32_t ks, uint32_t prod, uint32_t na, uint32_t nb, uint32_t nbk,
                                                   uint32_t nl) {
    fresh3_layout L;
    uint32_t o = 0;
    const uint32_t cells = 2u * ks;
    L.tk_words = ((cells + 2u > prod ? cells + 2u : prod) + 3u) & ~3u;   // b128 scan chunks; a dummy slot
    L.pmax = ((prod < cells ? prod : cells) + 1u) & ~1u;
    L.tkey = o;    o = align16(o + L.tk_words * 4u);
    L.lim = o;     o = align16(o + L.pmax * 24u);   // 3 u64 limbs per emit position, interleaved
    L.members = o; o = align16(o + kBigCap * 2u);   // slots of buckets with more than 4 slots
    L.a_w = o;     o = align16(o + na * 16u);
    L.a_inf = o;   o = align16(o + na * 4u);
    L.b_w = o;     o = align16(o + nb * 16u);
    L.b_inf = o;   o = align16(o + nb * 4u);
    L.pm = o;      o = align16(o + nl * 8u);   // parent masks and remap of C's layers (nl <= 64)
    L.remap = o;   o = align16(o + nl * 4u);
    L.misc = o;    o = align16(o + F3_WORDS * 4u);
    // bucket-group rebuild scratch: nbk u32 CSR offsets, 2 ks u32 slot records, ks u16 CSR
    // members; in the limb arrays when they fit (zero between pairs, zeroed again after a
    // rebuild), else at the end
    const uint32_t scratch = (2u * nbk + 2u * ks) * 4u + ks * 2u;
    if (scratch <= L.pmax * 24u) {
        L.boff = L.lim;
    } else {
        L.boff = o;
        o = align16(o + scratch);
    }
    L.total = o;
    return L;
}

#ifndef PVAC_U5
#define PVAC_U5 2
#endif
#ifndef PVAC_REP_P1   // experiment builds repeat a phase (idempotent) to measure its cost
#define PVAC_REP_P1 1
#endif
#ifndef PVAC_REP_P2
#define PVAC_REP_P2 1
#endif
#ifndef PVAC_REP_P4
#define PVAC_REP_P4 1
#endif

#ifdef PVAC_PHASE_STAMPS
#define STAMP3(ph)                                                        \
    do {                                                                  \
        if (threadIdx.x == 0) {                                           \
            const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
            st3_acc[ph] += now_ - st3_last;                               \
            st3_last = now_;                                              \
        }                                                                 \
    } while (0)
#define STAMP3_SYNC(ph)                                    \
    do {                                                   \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
        STAMP3(ph);                                        \
    } while (0)
#else
#define STAMP3(ph) do {} while (0)
#define STAMP3_SYNC(ph) do {} while (0)
#endif
#ifdef PVAC_ASM_MARKS
#define M3(ph) asm volatile("; PVAC_MARK " #ph ::: "memory")
#else
#define M3(ph) do {} while (0)
#endif

// a value the compiler cannot see through: per-phase thread ids built from it keep per-thread LDS
// addresses from being hoisted out of the pair loop (and spilled) at 80 VGPRs
__device__ __forceinline__ uint32_t opaque(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}

#ifndef PVAC_F3_BS   // A/B builds only: workgroup size of k_ct_mul_fresh3
#define PVAC_F3_BS 512
#endif
#ifndef PVAC_F3_WPE   // A/B builds only: waves per SIMD the kernel is compiled for (6: <= 80 VGPRs)
#define PVAC_F3_WPE 6
#endif
#ifndef PVAC_F3_U     // A/B builds only: product rounds per thread kept in registers from P1 to P5
#define PVAC_F3_U 4
#endif
constexpr uint32_t kF3Threads = PVAC_F3_BS;
template <int BS>
__global__ __launch_bounds__(BS, PVAC_F3_WPE) void k_ct_mul_fresh3(const mul_fresh_args* __restrict__ gp, fresh3_layout Ls) {
    constexpr int KI = (kFreshKeysMax + BS - 1) / BS;    // key slots per thread (rebuild)
    // bins per thread: a bin holds 2 or 3 slots except when size-2 buckets are left without a
    // size-1 partner, so there are at most kFreshKeysMax / 2 bins
    constexpr int KR = (kFreshKeysMax / 2 + BS - 1) / BS;
    constexpr int NW = BS / 64;
    constexpr int U = PVAC_F3_U;                         // product rounds per pass
    constexpr uint32_t kT16 = 0xFFFFu;                   // no first-insert time
    static_assert(BS % 64 == 0 && BS >= (int)kFreshEdgesMax && NW <= 16, "fresh geometry");
    static_assert(kFreshProdMax <= 16u * 256u, "16 scan segments of 256 product times");
    argp gq = launder((uint64_t)gp);
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint32_t* tkey = (uint32_t*)(lds + Ls.tkey);
    uint16_t* tk16 = (uint16_t*)(lds + Ls.tkey);         // [2 c] = low half of cell c, [2 t + 1] = G[t]
    const uint64_t* tk64 = (const uint64_t*)(lds + Ls.tkey);   // [s] = cells 2 s, 2 s + 1
    unsigned long long* lim = (unsigned long long*)(lds + Ls.lim);   // [3 p + l] limb l of position p
    uint32_t* boff = (uint32_t*)(lds + Ls.boff);
    uint16_t* members = (uint16_t*)(lds + Ls.members);
    ulonglong2* a_w = (ulonglong2*)(lds + Ls.a_w);
    uint32_t* a_inf = (uint32_t*)(lds + Ls.a_inf);
    ulonglong2* b_w = (ulonglong2*)(lds + Ls.b_w);
    uint32_t* b_inf = (uint32_t*)(lds + Ls.b_inf);
    uint64_t* pm = (uint64_t*)(lds + Ls.pm);
    uint32_t* remap = (uint32_t*)(lds + Ls.remap);
    uint32_t* misc = (uint32_t*)(lds + Ls.misc);

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t Bm = gq->Bm;
    const uint32_t bdiv = (uint32_t)(0x100000000ull / Bm) + 1u;   // s / Bm = mulhi(s, bdiv) for s < 2^16
    const uint32_t dummy = gq->ks_max;   // a slot whose two cell words are never set (tk_words > 2 ks_max + 1)
    // Owned slots (static per bucket count and B): rec0 = slot | mates << 11 | m0 << 16,
    // rec1 = m1 | m2 << 16, the other slots of its libstdc++ bucket (unused: dummy). mates = 7:
    // the bucket has more than 3 others; then m0 = CSR start into `members`, rec1 = their number.
    // Slot k of a thread has rank tid + k*BS in mate-count order (descending), so lane 0 of a wave
    // holds that wave's largest count for row k (cmax, wave-uniform).
    uint32_t rec0[KR], rec1[KR], cmax[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        rec0[k] = dummy | (dummy << 16);
        rec1[k] = dummy | (dummy << 16);
        cmax[k] = 0;
    }
    uint32_t nbk_c = 0, nB_c = 0, mdiv = 0;

    {   // one-time clear: cell words empty, limbs zero
        const uint32_t tid = threadIdx.x;
        for (uint32_t w = tid; w < Ls.tk_words; w += BS) tkey[w] = kT16;
        for (uint32_t w = tid; w < 3u * Ls.pmax; w += BS) lim[w] = 0;
        if (tid < F3_WORDS) misc[tid] = 0;
    }
    __syncthreads();

#ifdef PVAC_PHASE_STAMPS
    // diagnostic build: phase times of thread 0 accumulated in LDS (registers would cost occupancy)
    __shared__ unsigned long long st3_acc[kStampPhases];
    if (threadIdx.x < kStampPhases) st3_acc[threadIdx.x] = 0;
    unsigned long long st3_last = __builtin_amdgcn_s_memtime();
#endif
#ifdef PVAC_CENSUS
    const unsigned long long cen_t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long cen_pairs = 0;
#endif
    const fresh_rec* const recs = gq->recs;
    const uint64_t n_pairs = gq->A.n;
    fresh_hdr cur{};
    cur.pr = kNoPair;
    {   // the first pair's record words into LDS (the control wave), then decoded by every wave
        const uint64_t q0 = next_small(gq, blockIdx.x);
        if (q0 != kNoPair) {
            const uint32_t v0 = ((const uint32_t*)(recs + q0))[threadIdx.x & 15u];
            if (wave == NW - 1 && lane < 16) misc[F3_HDR + lane] = v0;
            cur = hdr_decode(v0, q0);
        }
    }
    __syncthreads();
    stage_pair(prefetch_pair(gq, cur, misc + F3_HDR), cur, Bm, a_w, a_inf, b_w, b_inf, pm, misc);
    __syncthreads();

    while (cur.pr != kNoPair) {
        gq = launder(gq);
        const uint64_t qn = cur.pr + gridDim.x;
        const uint32_t hv = wave == NW - 1 ? hdr_issue(recs, n_pairs, qn) : 0u;
        const uint64_t pr = cur.pr;
        const uint32_t LA = cur.LA, LB = cur.LB, nA = cur.nA, nB = cur.nB;
        const uint32_t LP = LA * LB, KS = LP * Bm, n = nA * nB;
        const uint32_t base = LA + LB, Lc = base + LP;
        const uint32_t nbk = cur.nbk;

        if (misc[F3_INVALID]) {   // invalid references: reject the pair (reference behaviour is UB)
            __syncthreads();
            if (threadIdx.x == 0) {
                gq->pair_status[pr] = 2;
                gq->C.l_cnt[pr] = 0;
                gq->C.e_cnt[pr] = 0;
                misc[F3_INVALID] = 0;
                misc[F3_AMASK] = 0;
                misc[F3_BMASK] = 0;
            }
            if (wave == NW - 1 && lane < 16) misc[F3_HDR + lane] = hv;
            __syncthreads();
            const fresh_hdr nx = hdr_next(gq, misc[F3_HDR + (lane & 15)], qn, n_pairs, misc + F3_HDR);
            __syncthreads();   // (hdr_next may have replaced the LDS words)
            stage_pair(prefetch_pair(gq, nx, misc + F3_HDR), nx, Bm, a_w, a_inf, b_w, b_inf, pm, misc);
            __syncthreads();
            cur = nx;
            continue;
        }
        if (nB != nB_c) {   // i = ((t << 8) * mdiv) >> 32, exact for t < 2^12
            nB_c = nB;
            mdiv = (1u << 24) / max(nB, 1u) + 1u;
        }

        // ---- static slot records for a new bucket count: bucket of every slot, the buckets as a
        //      CSR (counting sort), each slot's mates, then the slots dealt to threads in
        //      descending mate-count order. Scratch in the (zero) limb arrays, zeroed afterwards.
        if (nbk != nbk_c) {
            const uint32_t tid = opaque(threadIdx.x);
            const uint32_t ksa = gq->ks_max;
            uint32_t* rnk = boff + nbk;                  // [nbk] rank of a bucket inside its size class
            uint32_t* drec = rnk + nbk;                  // [2 ksa] bin records
            uint16_t* csr = (uint16_t*)(drec + 2u * ksa);   // [ksa] slots in bucket order
            const fastmod64 fm{nbk, ((recp)gq->recs + pr)->nb_magic};
            uint32_t bk[KI];
#pragma unroll
            for (int k = 0; k < KI; ++k) {
                const uint32_t s = tid + (uint32_t)k * BS;
                const uint32_t lp = __umulhi(s, bdiv);
                bk[k] = (uint32_t)fmod64((((uint64_t)lp << 32) | (s - lp * Bm)) * kGolden, fm);
            }
            for (uint32_t w = tid; w < nbk; w += BS) boff[w] = 0;
            if (tid < 8) misc[F3_CLS + tid] = 0;   // size classes 0 (big), 1, 2, 3; [7] = big-member allocation
            if (tid == 0) misc[F3_BIGOVF] = 0;
            __syncthreads();
#pragma unroll
            for (int k = 0; k < KI; ++k)
                if (tid + (uint32_t)k * BS < ksa) atomicAdd(&boff[bk[k]], 1u);
            __syncthreads();
            {
                const uint32_t per = (nbk + BS - 1) / BS, b0 = tid * per;
                uint32_t local = 0;
                for (uint32_t b = b0; b < b0 + per && b < nbk; ++b) local += boff[b];
                uint32_t tot;
                uint32_t run = block_exclusive_scan<BS>(local, misc + F3_PART, tot);
                for (uint32_t b = b0; b < b0 + per && b < nbk; ++b) {
                    const uint32_t v = boff[b];
                    boff[b] = run;
                    run += v;
                }
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < KI; ++k) {
                const uint32_t s = tid + (uint32_t)k * BS;
                if (s < ksa) csr[atomicAdd(&boff[bk[k]], 1u)] = (uint16_t)s;
            }
            __syncthreads();   // boff[b] is now the END of bucket b's slots
            // Buckets packed into bins of at most 3 slots (a bucket never splits): every size-3
            // bucket alone, each size-2 bucket with one size-1 bucket while they last, the other
            // size-1 buckets by three; a bucket of more than 3 slots gets a bin of its own and
            // its slots go to `members`. Bin record: rec0 = m0 | m1 << 16, rec1 = m2 | flags << 16
            // (flags: bit 0 m0~m1 share a bucket, bit 1 m0~m2, bit 2 m1~m2, bit 3 big); unused
            // slots are the dummy. Bin q belongs to thread q % BS, row q / BS.
            const uint32_t nbr = (nbk + BS - 1) / BS;
            for (uint32_t j = 0; j < nbr; ++j) {   // pass 1: rank inside the size class
                const uint32_t b = tid + j * BS;
                if (b >= nbk) break;
                const uint32_t z = boff[b] - (b ? boff[b - 1] : 0u);
                if (z) rnk[b] = atomicAdd(&misc[F3_CLS + (z > 3 ? 0u : z)], 1u);
            }
            for (uint32_t q = tid; q < 2u * ksa; q += BS) drec[q] = q & 1u ? dummy : dummy | (dummy << 16);
            __syncthreads();
            const uint32_t nbig = misc[F3_CLS + 0], n1 = misc[F3_CLS + 1], n2 = misc[F3_CLS + 2], n3 = misc[F3_CLS + 3];
            const uint32_t pair1 = min(n1, n2);                    // size-1 buckets that join a size-2 one
            const uint32_t b3 = nbig, b2 = b3 + n3, b1 = b2 + n2;  // first bin of each kind
            const uint32_t nbins = b1 + (n1 - pair1 + 2u) / 3u;
            uint16_t* dh = (uint16_t*)drec;                        // [4 q + f]: field f of bin q
            for (uint32_t j = 0; j < nbr; ++j) {   // pass 2: slots into bins
                const uint32_t b = tid + j * BS;
                if (b >= nbk) break;
                const uint32_t end = boff[b], start = b ? boff[b - 1] : 0u, z = end - start;
                if (z == 0) continue;
                const uint32_t r = rnk[b];
                if (z == 3) {
                    const uint32_t q = b3 + r;
                    dh[4u * q] = csr[start];
                    dh[4u * q + 1u] = csr[start + 1];
                    dh[4u * q + 2u] = csr[start + 2];
                    dh[4u * q + 3u] = 7u;
                } else if (z == 2) {
                    const uint32_t q = b2 + r;
                    dh[4u * q] = csr[start];
                    dh[4u * q + 1u] = csr[start + 1];
                    dh[4u * q + 3u] = 1u;
                } else if (z == 1) {
                    if (r < pair1) {
                        dh[4u * (b2 + r) + 2u] = csr[start];
                    } else {
                        const uint32_t x = r - pair1;
                        dh[4u * (b1 + x / 3u) + x % 3u] = csr[start];
                    }
                } else {   // more than 3 slots
                    const uint32_t q = r;
                    uint32_t at = atomicAdd(&misc[F3_CLS + 7], z);
                    uint32_t zz = z;
                    if (at + z <= kBigCap) {
                        for (uint32_t x = 0; x < z; ++x) members[at + x] = csr[start + x];
                    } else {   // pairs of this bucket count go to the general path
                        at = 0;
                        zz = 1;
                        misc[F3_BIGOVF] = 1u;
                    }
                    dh[4u * q] = (uint16_t)at;
                    dh[4u * q + 1u] = (uint16_t)zz;
                    dh[4u * q + 3u] = 8u;
                }
            }
            __syncthreads();
            if (tid == 0 && nbins > (uint32_t)(KR * BS)) misc[F3_BIGOVF] = 1u;   // cannot happen (see KR)
#pragma unroll
            for (int k = 0; k < KR; ++k) {
                const uint32_t q = tid + (uint32_t)k * BS;
                rec0[k] = q < nbins ? drec[2u * q] : dummy | (dummy << 16);
                rec1[k] = q < nbins ? drec[2u * q + 1u] : dummy;
                cmax[k] = __builtin_amdgcn_readfirstlane(q < nbins ? 1u : 0u);   // row has bins in this wave
            }
            nbk_c = nbk;
            __syncthreads();
            for (uint32_t w = tid; w < 2u * nbk + 2u * ksa + (ksa + 1u) / 2u; w += BS) boff[w] = 0;
            __syncthreads();
        }

        // cell of a staged (A record + B record) sum: 2 * slot + (ch_i != ch_j)
        auto cell_of = [&](uint32_t sum) {
            uint32_t r = sum & 0xFFFu;
            r = min(r, r - Bm);
            return ((((sum >> 12) & 0xFFFu) + r) << 1) | ((sum >> 24) & 1u);
        };
        M3(1);
        // ---- P1: first-insert time of every cell. The first pass's products stay in registers
        //      for P5: i | j << 8 | cell << 16 (i, j < 256, cell < 4096); t >= n: ~0
        uint32_t prod[U];
#pragma unroll
        for (int u = 0; u < U; ++u) prod[u] = ~0u;
        for (int rep_ = 0; rep_ < PVAC_REP_P1; ++rep_) {   // experiment builds only (tools/exp_fresh3.py)
        {
            const uint32_t tid = opaque(threadIdx.x);
            for (uint32_t t0 = tid; t0 < n; t0 += U * BS) {
                uint32_t sum[U], ij[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t t = min(t0 + (uint32_t)u * BS, n - 1u);
                    const uint32_t i = __umulhi(t << 8, mdiv);
                    const uint32_t j = t - i * nB;
                    ij[u] = i | (j << 8);
                    sum[u] = a_inf[i] + b_inf[j];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t t = t0 + (uint32_t)u * BS;
                    const uint32_t c = cell_of(sum[u]);
                    if (t < n) atomicMin(&tkey[c], t);
                    if (t0 == tid) prod[u] = t < n ? ij[u] | (c << 16) : ~0u;
                }
            }
        }
        }
        STAMP3_SYNC(1);
        if (wave == NW - 1 && lane < 16) misc[F3_HDR + lane] = hv;   // its load has had P1 to land
        __syncthreads();
        STAMP3(2);
        gq = launder(gq);
        __builtin_amdgcn_s_setprio(1);
        const fresh_hdr nxt = hdr_next(gq, misc[F3_HDR + (lane & 15)], qn, n_pairs, misc + F3_HDR);

        M3(2);
        // ---- P2: per bin (up to 3 slots whose buckets lie wholly in the bin): key time and emit
        //      bits of each slot, its bucket's first-insert time t_bkt, its rank in the bucket
        //      (edges of later keys) and the bucket's edge count G[t_bkt]
        uint32_t ordA[KR], ordB[KR];   // t_bkt of slots 0, 1 | t_bkt of slot 2, rank 3 bits x 3, emit 2 bits x 3
#if PVAC_REP_P2 == 0   // experiment builds: no P2 (no emits, every bucket time "none")
#pragma unroll
        for (int k = 0; k < KR; ++k) {
            ordA[k] = kT16 | (kT16 << 16);
            ordB[k] = kT16;
        }
#endif
        for (int rep_ = 0; rep_ < PVAC_REP_P2; ++rep_) {   // experiment builds only (tools/exp_fresh3.py)
        {
            auto cells = [&](uint64_t x, uint32_t& t, uint32_t& e) {
                const uint32_t x0 = (uint32_t)x & kT16, x1 = (uint32_t)(x >> 32) & kT16;
                t = min(x0, x1);
                e = (x0 != kT16 ? 1u : 0u) | (x1 != kT16 ? 2u : 0u);
            };
#pragma unroll
            for (int k = 0; k < KR; ++k) {
                ordA[k] = kT16 | (kT16 << 16);
                ordB[k] = kT16;
                if (cmax[k] == 0u) continue;   // wave-uniform: no bin in this row
                const uint32_t fl = rec1[k] >> 16;
                const bool big = (fl & 8u) != 0;
                const uint32_t m0 = big ? dummy : rec0[k] & 0xFFFFu, m1 = big ? dummy : rec0[k] >> 16;
                const uint32_t m2 = rec1[k] & 0xFFFFu;
                uint32_t t0, t1, t2, e0, e1, e2;
                cells(tk64[m0], t0, e0);
                cells(tk64[m1], t1, e1);
                cells(tk64[m2], t2, e2);
                const uint32_t p0 = __popc(e0), p1 = __popc(e1), p2 = __popc(e2);
                const bool f01 = fl & 1u, f02 = fl & 2u, f12 = fl & 4u;
                // times are distinct when present; an absent slot has no edges (p = 0)
                const uint32_t wi0 = (f01 && t1 > t0 ? p1 : 0u) + (f02 && t2 > t0 ? p2 : 0u);
                const uint32_t wi1 = (f01 && t0 > t1 ? p0 : 0u) + (f12 && t2 > t1 ? p2 : 0u);
                const uint32_t wi2 = (f02 && t0 > t2 ? p0 : 0u) + (f12 && t1 > t2 ? p1 : 0u);
                uint32_t tb0 = min(t0, min(f01 ? t1 : kT16, f02 ? t2 : kT16));
                const uint32_t tb1 = min(t1, min(f01 ? t0 : kT16, f12 ? t2 : kT16));
                const uint32_t tb2 = min(t2, min(f02 ? t0 : kT16, f12 ? t1 : kT16));
                uint32_t cE0 = p0 + (f01 ? p1 : 0u) + (f02 ? p2 : 0u);
                const uint32_t cE1 = p1 + (f01 ? p0 : 0u) + (f12 ? p2 : 0u);
                const uint32_t cE2 = p2 + (f02 ? p0 : 0u) + (f12 ? p1 : 0u);
                if (big) {   // a bucket of more than 3 slots (rare): t_bkt and edges from `members`
                    const uint32_t q0 = rec0[k] & 0xFFFFu, g = rec0[k] >> 16;
                    for (uint32_t q = q0; q < q0 + g; ++q) {
                        const uint32_t m = members[q];
                        uint32_t t, e;
                        cells(tk64[m], t, e);
                        tb0 = min(tb0, t);
                        cE0 += __popc(e);
                    }
                }
                // G[t_bkt] from the bucket's leader (duplicates of one bucket write the same value)
                if (tb0 != kT16 && tb0 == t0) tk16[2u * tb0 + 1u] = (uint16_t)cE0;
                if (tb1 != kT16 && tb1 == t1) tk16[2u * tb1 + 1u] = (uint16_t)cE1;
                if (tb2 != kT16 && tb2 == t2) tk16[2u * tb2 + 1u] = (uint16_t)cE2;
                if (big && tb0 != kT16) tk16[2u * tb0 + 1u] = (uint16_t)cE0;
                ordA[k] = tb0 | (tb1 << 16);
                ordB[k] = tb2 | (wi0 << 16) | (wi1 << 19) | (wi2 << 22) | (e0 << 25) | (e1 << 27) | (e2 << 29);
            }
        }
        }
        STAMP3_SYNC(3);
        __syncthreads();
        STAMP3(4);
        gq = launder(gq);

        M3(3);
        // ---- P3: every wave suffix-scans 256-time segments of G (in place, in-segment offsets;
        //      segment totals into misc[F3_PART + g]); then wave 0 runs compact_layers
        {
            const uint32_t nseg = (n + 255u) >> 8;
            uint4* gv = (uint4*)tkey;
            for (uint32_t g = (uint32_t)wave; g < nseg; g += NW) {
                const uint32_t q = g * 64u + (uint32_t)lane;   // b128 chunk: times 4q .. 4q + 3
                const bool live = 4u * q < n;
                const uint4 x = live ? gv[q] : make_uint4(0, 0, 0, 0);
                const uint32_t local = (x.x >> 16) + (x.y >> 16) + (x.z >> 16) + (x.w >> 16);
                const uint32_t incl = wave_incl_scan_u32(local);
                const uint32_t tot = __builtin_amdgcn_readlane(incl, 63);
                uint32_t run = tot - incl;   // later chunks of the segment
                uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int h = 3; h >= 0; --h) {
                    const uint32_t gcur = w[h] >> 16;
                    w[h] = (w[h] & 0xFFFFu) | (run << 16);
                    run += gcur;
                }
                if (live) gv[q] = make_uint4(w[0], w[1], w[2], w[3]);
                if (lane == 0) misc[F3_PART + g] = tot;
            }
        }
        // compact_layers: when every product layer has an edge, every input layer is a direct
        // parent of one, so nothing is removed (ident); only otherwise does wave 0 run the closure
        // product layers with cells: (la, lb) with edges in A's layer la and in B's layer lb
        uint64_t used_lp = 0;
        {
            uint32_t a = __builtin_amdgcn_readfirstlane(misc[F3_AMASK]);
            const uint64_t b = __builtin_amdgcn_readfirstlane(misc[F3_BMASK]);
            while (a) {   // scalar: LA * LB <= 64, so every shift is < 64
                const uint32_t la = (uint32_t)__builtin_ctz(a);
                a &= a - 1;
                used_lp |= b << (la * LB);
            }
        }
        const bool all_lp = used_lp == (LP >= 64 ? ~0ull : ((1ull << LP) - 1ull));
        if (wave == 0 && !all_lp) {
            __builtin_amdgcn_s_setprio(3);
            const uint64_t all = Lc >= 64 ? ~0ull : ((1ull << Lc) - 1ull);
            uint64_t keep = (used_lp << base) & all;
            const uint64_t mypm = (uint32_t)lane < Lc ? pm[lane] : 0ull;
            for (;;) {
                const uint64_t par = wave_or_u64(((keep >> lane) & 1ull) ? mypm : 0ull);
                const uint64_t nk = keep | par;
                if (nk == keep) break;
                keep = nk;
            }
            if ((uint32_t)lane < Lc)
                remap[lane] = ((keep >> lane) & 1ull)
                                  ? __builtin_amdgcn_mbcnt_hi((uint32_t)(keep >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)keep, 0u))
                                  : 0xFFFFFFFFu;
            if (lane == 0) {
                *(uint64_t*)(misc + F3_KEEP) = keep;
                misc[F3_IDENT] = keep == all;
            }
            __builtin_amdgcn_s_setprio(1);
        }
        STAMP3_SYNC(5);
        __syncthreads();
        STAMP3(6);
        gq = launder(gq);

        M3(4);
        // ---- P4: segment offsets (suffix over the segment totals, lane g holds segment g's),
        //      then emit positions into the cell words and cell ids into limb 2
        const uint32_t nseg = (n + 255u) >> 8;
        uint32_t segsuf, total;
        {
            const uint32_t tl = (uint32_t)lane < nseg ? misc[F3_PART + lane] : 0u;
            const uint32_t incl = wave_incl_scan_u32(tl);
            total = __builtin_amdgcn_readlane(incl, 63);
            segsuf = total - incl;   // segments after lane's
        }
        // guard_budget (encrypt.hpp:106-111) and ORDER_CANONICAL want (layer, idx, P<M) order: the
        // general path produces it (redo); this kernel emits the reference hash order only
        const bool canonical = (gq->flags & PVAC_MUL_ORDER_CANONICAL) != 0 || total > gq->edge_budget;
        const uint64_t ceo = cur.ceo;
        for (int rep_ = 0; rep_ < PVAC_REP_P4; ++rep_) {   // experiment builds only (tools/exp_fresh3.py)
        {
            // 32-bit LDS byte offsets (no 64-bit address arithmetic): a cell word's low half, limb 2
            // of a position
            // (LDS pointers: 32-bit address arithmetic, no 64-bit mad per store)
            typedef __attribute__((address_space(3))) uint8_t lds8;
            lds8* const L3 = (lds8*)lds;
            const uint32_t tkb = Ls.tkey, lmb = Ls.lim + 20u;   // limb 2's HIGH dword of position 0
            // slot m's cells at p (P), p + (P present) (M). Limb 2 of a position holds the cell id at
            // bit 52: only its high dword is written (cell << 20), the limbs being zero between pairs
            auto emit = [&](uint32_t m, uint32_t e, uint32_t p) {
                const uint32_t ca = tkb + 8u * m, la = lmb + 24u * p;
                if (e & 1u) {
                    *(__attribute__((address_space(3))) uint16_t*)(L3 + ca) = (uint16_t)p;
                    *(__attribute__((address_space(3))) uint32_t*)(L3 + la) = m << 21;
                }
                if (e & 2u) {
                    const uint32_t pp = e & 1u;
                    *(__attribute__((address_space(3))) uint16_t*)(L3 + ca + 4u) = (uint16_t)(p + pp);
                    *(__attribute__((address_space(3))) uint32_t*)(L3 + la + 24u * pp) = (m << 21) | (1u << 20);
                }
            };
            // emit offset of bucket time tb: in-segment suffix offset + segment offset (from lane
            // tb >> 8 by ds_bpermute, in which every lane takes part)
            auto offset = [&](uint32_t tb) {
                const bool has = tb != kT16;
                const uint32_t so = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((has ? tb >> 8 : 0u) << 2), (int)segsuf);
                const uint32_t tv = tkey[has ? tb : 0u];   // unconditional: no exec-masked branch
                return has ? (tv >> 16) + so : 0u;
            };
#pragma unroll
            for (int k = 0; k < KR; ++k) {
                if (cmax[k] == 0u) continue;   // wave-uniform
                const uint32_t fl = rec1[k] >> 16;
                const bool big = (fl & 8u) != 0;
                const uint32_t tb0 = ordA[k] & kT16, tb1 = ordA[k] >> 16, tb2 = ordB[k] & kT16;
                const uint32_t o0 = offset(tb0), o1 = offset(tb1), o2 = offset(tb2);
                if (!big) {
                    emit(rec0[k] & 0xFFFFu, (ordB[k] >> 25) & 3u, o0 + ((ordB[k] >> 16) & 7u));
                    emit(rec0[k] >> 16, (ordB[k] >> 27) & 3u, o1 + ((ordB[k] >> 19) & 7u));
                    emit(rec1[k] & 0xFFFFu, (ordB[k] >> 29) & 3u, o2 + ((ordB[k] >> 22) & 7u));
                } else if (tb0 != kT16) {   // big bucket: each slot's rank from the others' times (O(z^2), rare)
                    // Two passes: every member's rank is computed from the UNMODIFIED first-insert
                    // times while only the positions' limb words record the cell; the cell words
                    // get their positions afterwards (an emit inside the rank loop would overwrite
                    // times that later members still compare against)
                    const uint32_t q0 = rec0[k] & 0xFFFFu, g = rec0[k] >> 16;
                    uint32_t cnt = 0;
                    for (uint32_t q = q0; q < q0 + g; ++q) {
                        const uint32_t m = members[q];
                        const uint64_t x = tk64[m];
                        const uint32_t x0 = (uint32_t)x & kT16, x1 = (uint32_t)(x >> 32) & kT16;
                        const uint32_t t = min(x0, x1);
                        const uint32_t e = (x0 != kT16 ? 1u : 0u) | (x1 != kT16 ? 2u : 0u);
                        if (!e) continue;
                        uint32_t within = 0;
                        for (uint32_t r = q0; r < q0 + g; ++r) {
                            const uint64_t y = tk64[members[r]];
                            const uint32_t y0 = (uint32_t)y & kT16, y1 = (uint32_t)(y >> 32) & kT16;
                            const uint32_t t2 = min(y0, y1);
                            within += t2 != kT16 && t2 > t ? (y0 != kT16 ? 1u : 0u) + (y1 != kT16 ? 1u : 0u) : 0u;
                        }
                        uint32_t p = o0 + within;
                        if (e & 1u) lim[3u * p++ + 2u] = (unsigned long long)(2u * m) << 52;
                        if (e & 2u) lim[3u * p + 2u] = (unsigned long long)(2u * m + 1u) << 52;
                        cnt += __popc(e);
                    }
                    for (uint32_t p = o0; p < o0 + cnt; ++p) tk16[2u * (uint32_t)(lim[3u * p + 2u] >> 52)] = (uint16_t)p;
                }
            }
        }
        }
        const uint64_t keep = all_lp ? (Lc >= 64 ? ~0ull : ((1ull << Lc) - 1ull)) : *(const uint64_t*)(misc + F3_KEEP);
        const bool ident = all_lp || misc[F3_IDENT] != 0;
        if (!ident && wave == 1) {   // compact the identity-placed layer records in place
            const uint32_t l = lane;
            const uint64_t clo = ((recp)gq->recs + pr)->clo;
            pvac_layer y{};
            if (l < Lc) y = gq->C.layers[clo + l];
            if (l < Lc && ((keep >> l) & 1ull)) {
                if (y.rule == 1) {
                    y.pa = y.pa < Lc ? remap[y.pa] : 0xFFFFFFFFu;
                    y.pb = y.pb < Lc ? remap[y.pb] : 0xFFFFFFFFu;
                }
                gq->C.layers[clo + remap[l]] = y;
            }
        }
        if (threadIdx.x == 0) {
            gq->C.e_cnt[pr] = total;
            gq->C.l_cnt[pr] = (uint64_t)__popcll(keep);
            gq->pair_status[pr] = 0;
            // every thread read the layer masks in P3 (a barrier ago); stage_pair ORs the next
            // pair's into them after P5's barrier
            misc[F3_AMASK] = 0;
            misc[F3_BMASK] = 0;
        }
        // next pair's raw inputs: in flight through P5 and the writer, staged after them
        const fresh_pref pf = prefetch_pair(gq, nxt, misc + F3_HDR, opaque(threadIdx.x));
        STAMP3_SYNC(7);
        __syncthreads();
        STAMP3(8);
        gq = launder(gq);
        __builtin_amdgcn_s_setprio(0);

        M3(5);
        // ---- P5: products into the limb accumulators of their emit positions
#ifndef PVAC_EXP_SKIP_P5   // experiment builds only: no products (outputs wrong; the phase's cost)
        {
            const uint32_t tid = opaque(threadIdx.x);
            auto accumulate = [&](const ulonglong2& x, const ulonglong2& y, uint32_t p) {
                uint64_t x0, x1, l0, l1, l2;
#ifdef PVAC_EXP_NOMUL3
                x0 = x.x ^ y.x;
                x1 = (x.y ^ y.y) & 0x7FFFFFFFFFFFFFFFull;
#else
                fp_mul_fold1(fp{x.x, x.y}, fp{y.x, y.y}, x0, x1);
#endif
                fp_split3_44(x0, x1, l0, l1, l2);
                unsigned long long* q = lim + 3u * p;
                atomicAdd(q, (unsigned long long)l0);
                atomicAdd(q + 1, (unsigned long long)l1);
                atomicAdd(q + 2, (unsigned long long)l2);
            };
            // first pass from the registers of P1, two products at a time
#pragma unroll
            for (int u0 = 0; u0 < U; u0 += 2) {
                if (__builtin_amdgcn_ballot_w64(prod[u0] != ~0u) == 0) continue;   // none in this wave's rounds
                ulonglong2 x[2], y[2];
                uint32_t p[2];
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    if (u0 + v >= U) break;   // odd U (A/B builds)
                    const uint32_t pk = prod[u0 + v] == ~0u ? 0u : prod[u0 + v];
                    x[v] = a_w[pk & 0xFFu];
                    y[v] = b_w[(pk >> 8) & 0xFFu];
                    p[v] = tk16[2u * (pk >> 16)];
                }
#pragma unroll
                for (int v = 0; v < 2; ++v)
                    if (u0 + v < U && prod[u0 + v] != ~0u) accumulate(x[v], y[v], p[v]);
            }
            // further passes (n > U * BS): recompute
            for (uint32_t t = tid + U * BS; t < n; t += BS) {
                const uint32_t i = __umulhi(t << 8, mdiv);
                const uint32_t j = t - i * nB;
                const ulonglong2 x = a_w[i], y = b_w[j];
                const uint32_t p = tk16[2u * cell_of(a_inf[i] + b_inf[j])];
                accumulate(x, y, p);
            }
        }
#endif
        STAMP3_SYNC(9);
        __syncthreads();
        STAMP3(10);
        gq = launder(gq);

        M3(7);
        // ---- P6: stage the next pair first (its loads were issued before P5; a wait after the
        //      writer's stores would have to wait for those too: vmcnt counts both in order), then
        //      the coalesced writer over emit positions (not the control wave: its vector-memory
        //      queue stays free of stores), then clear the cell words
        stage_pair(pf, nxt, Bm, a_w, a_inf, b_w, b_inf, pm, misc, opaque(threadIdx.x));
        {
            const uint32_t tid = opaque(threadIdx.x);
            uint64_t* cm = gq->C.meta + ceo;
            uint64_t* cl = gq->C.w_lo + ceo;
            uint64_t* chh = gq->C.w_hi + ceo;
            uint32_t* sp = gq->salt_pos ? gq->salt_pos + ceo : nullptr;
            const bool zero0 = canonical || misc[F3_BIGOVF];
            uint64_t zmask = 0;   // lanes that folded a 0 sum (a ballot per position round: SGPRs, no VALU)
            // one zero register pair for the three limb clears (else rematerialised per position)
            uint64_t z64 = 0;
            asm volatile("" : "+v"(z64));
            // buffer stores: one 32-bit offset for the three arrays (SGPR bases) instead of three
            // 64-bit address computations per position (round 4: -1.7%, A/B)
            typedef unsigned int u2v __attribute__((ext_vector_type(2)));
            const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(cm, 0, 0x7FFFFFF8, 0x00020000);
            const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(cl, 0, 0x7FFFFFF8, 0x00020000);
            const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(chh, 0, 0x7FFFFFF8, 0x00020000);
#ifdef PVAC_EXP_SKIP_W   // experiment builds only: no writer (outputs wrong; the phase's cost)
            for (uint32_t p = tid; p < 0u; p += BS - 64) {
#else
            for (uint32_t p = tid; p < total && wave != NW - 1; p += BS - 64) {
#endif
                unsigned long long* q = lim + 3u * p;
                const uint64_t l0 = q[0], l1 = q[1], l2c = q[2];
                q[0] = z64;
                q[1] = z64;
                q[2] = z64;
                const uint32_t cell = (uint32_t)(l2c >> 52);
                const fp w = fp_fold3_44(l0, l1, l2c & ((1ull << 52) - 1ull));
                zmask |= __builtin_amdgcn_ballot_w64(!fp_nonzero(w));
                const uint32_t s = cell >> 1;
                const uint32_t lp = __umulhi(s, bdiv);
                const uint32_t r = s - lp * Bm;
                const uint32_t lid = ident ? base + lp : remap[base + lp];
                // streaming stores: the output is not read again by this kernel (-1%, A/B)
                const uint64_t mv = make_meta(lid, r, cell & 1u);
                const uint32_t bo = p * 8u;   // < 2^31: a pair has <= 2 x 4096 edges
                __builtin_amdgcn_raw_buffer_store_b64(u2v{(uint32_t)mv, (uint32_t)(mv >> 32)}, rm, bo, 0, 2);
                __builtin_amdgcn_raw_buffer_store_b64(u2v{(uint32_t)w.lo, (uint32_t)(w.lo >> 32)}, rl, bo, 0, 2);
                __builtin_amdgcn_raw_buffer_store_b64(u2v{(uint32_t)w.hi, (uint32_t)(w.hi >> 32)}, rh, bo, 0, 2);
                if (sp) sp[p] = p;   // hash order == emit order here
            }
            if (zero0 || zmask) misc[F3_ZERO] = 1u;
            STAMP3_SYNC(11);
            const uint32_t used = (max(2u * KS, n) + 3u) >> 2;   // b128 words of this pair's cells and G
            uint4* tv = (uint4*)tkey;
            for (uint32_t q = tid; q < used; q += BS) tv[q] = make_uint4(kT16, kT16, kT16, kT16);
        }
        M3(8);
        STAMP3_SYNC(12);
        __syncthreads();
        STAMP3(13);
        if (threadIdx.x == 0 && misc[F3_ZERO]) {   // the general path redoes the pair
            gq->pair_status[pr] = kPairRedo;
            gq->redo_ids[atomicAdd(gq->redo_cnt, 1u)] = pr;
            misc[F3_ZERO] = 0;
        }
        cur = nxt;
        STAMP3(0);
#ifdef PVAC_CENSUS
        ++cen_pairs;
#endif
    }
#ifdef PVAC_CENSUS
    if (threadIdx.x == 0 && blockIdx.x < 4096) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        g_census[4 * blockIdx.x] = cen_t0;
        g_census[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        g_census[4 * blockIdx.x + 2] = cen_pairs;
        g_census[4 * blockIdx.x + 3] = hw;
    }
#endif
#ifdef PVAC_PHASE_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < 4096)
        for (int p = 0; p < kStampPhases; ++p) g_fresh_stamps[blockIdx.x * kStampPhases + p] = st3_acc[p];
#endif
}

}  // namespace

#ifdef PVAC_PHASE_STAMPS
extern "C" int pvac_hip_diag_fresh_stamps(unsigned long long* host, size_t n) {
    if (n > sizeof(g_fresh_stamps) / 8) n = sizeof(g_fresh_stamps) / 8;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fresh_stamps), n * 8) == hipSuccess ? 0 : -5;
}
#endif

hipError_t launch_mul_layers_fresh(const mul_fresh_args& a, hipStream_t st) {
    if (!a.A.n) return hipSuccess;
    hipLaunchKernelGGL(k_mul_layers_fresh, dim3((unsigned)((a.A.n * kLayLanes + kLayBlock - 1) / kLayBlock)), dim3(kLayBlock), 0,
                       st, a);
    return hipGetLastError();
}

hipError_t launch_ct_mul_fresh(const mul_fresh_args& a, const mul_fresh_args* args_dev, int num_cus, hipStream_t st) {
    if (!a.A.n) return hipSuccess;
    if (a.ks_max > kFreshKeysMax || a.layers_max > kFreshLayersMax || a.na_max > kFreshEdgesMax ||
        a.nb_max > kFreshEdgesMax)
        return hipErrorInvalidValue;
    // 12-bit product times and cell ids, 16-bit positions (see k_ct_mul_fresh3)
    if (a.prod_max > kFreshProdMax || 2u * a.ks_max > 4096u) return hipErrorInvalidValue;
    const fresh3_layout L = fresh3_lds(a.ks_max, a.prod_max, a.na_max, a.nb_max, a.buckets_max, a.layers_max);
    if (L.total > 160u * 1024u) return hipErrorInvalidValue;
    // resident workgroups per CU as the runtime counts them (LDS granules, registers): the
    // grid is persistent, so a workgroup that is not resident would run after the others
    // (cache keyed by the LDS size, shared by every context and thread: one atomic word
    // {LDS bytes << 8 | blocks}, so a reader never sees half an update)
    static std::atomic<uint64_t> occ_cache{0};
    uint64_t oc = occ_cache.load(std::memory_order_relaxed);
    if ((oc >> 8) != (uint64_t)L.total + 1u) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_ct_mul_fresh3<kF3Threads>, kF3Threads,
                                                          L.total) != hipSuccess || nb < 1)
            nb = 1;
        oc = (((uint64_t)L.total + 1u) << 8) | (uint64_t)std::min(nb, 255);
        occ_cache.store(oc, std::memory_order_relaxed);
        if (std::getenv("PVAC_DEBUG_OCC"))
            std::fprintf(stderr, "[pvac] k_ct_mul_fresh3: %u B LDS per workgroup, %d resident per CU\n", L.total, nb);
    }
    const int occ_blocks = (int)(oc & 0xFFu);
    // the API counts LDS in 128-byte steps; measured residency (tools/res_probe.hip) follows
    // 2 KiB granules: 53,248 B gives 3 workgroups per CU, 53,888 B only 2
    const int lds_fit = (int)((160u * 1024u) / ((L.total + 2047u) & ~2047u));
    int per_cu = std::min(std::min(occ_blocks, lds_fit), 3);
#ifdef PVAC_FRESH_PER_CU   // probe builds only (tools/percu_probe.sh): fewer resident workgroups per CU
    per_cu = std::max(1, std::min(per_cu, (int)PVAC_FRESH_PER_CU));
#endif
    uint64_t blocks = (uint64_t)num_cus * per_cu;
    if (blocks > a.A.n) blocks = a.A.n;
    hipLaunchKernelGGL((k_ct_mul_fresh3<kF3Threads>), dim3((unsigned)blocks), dim3(kF3Threads), L.total, st,
                       args_dev, L);
    return hipGetLastError();
}

}  // namespace pvhip
