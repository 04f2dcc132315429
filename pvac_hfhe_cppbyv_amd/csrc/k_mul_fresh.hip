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
#include "common.hpp"
#include "sha256.hpp"

namespace pvhip {

// Diagnostic build only (make diag -> lib/libpvac_hip_diag.so): wave 0 of every workgroup
// accumulates s_memtime deltas per phase into a debug array; never touches kernel outputs.
#ifdef PVAC_PHASE_STAMPS
constexpr int kStampPhases = 18;
__device__ unsigned long long g_fresh_stamps[4096 * kStampPhases];
#define PHASE_STAMP(ph)                                                  \
    do {                                                                 \
        if (threadIdx.x == 0) {                                          \
            const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
            st_acc_[ph] += now_ - st_last_;                              \
            st_last_ = now_;                                             \
        }                                                                \
    } while (0)
// sub-phase stamp after this wave's LDS traffic has completed (diagnostic build only)
#define PHASE_STAMP_SYNC(ph)                                   \
    do {                                                       \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     \
        PHASE_STAMP(ph);                                       \
    } while (0)
#elif defined(PVAC_ASM_MARKS)   // static instruction counts per phase (tools/asm_phases.py)
#define PHASE_STAMP(ph) asm volatile("; PVAC_MARK " #ph ::: "memory")
#define PHASE_STAMP_SYNC(ph) PHASE_STAMP(ph)
#else
#define PHASE_STAMP(ph) \
    do {                \
    } while (0)
#define PHASE_STAMP_SYNC(ph) \
    do {                     \
    } while (0)
#endif

namespace {

constexpr uint32_t kTInf = 0xFFFFFFFFu;
static_assert(kFreshLayersMax <= 64, "layer masks are u64");
static_assert(kFreshKeysMax <= 2048 && kFreshLayersMax <= 512, "writer entries pack slot, idx (11 bits each) and layer");

// ---------------------------------------------------------------- layer records
constexpr int kLayBlock = 256;
constexpr int kLayLanes = 4;   // lanes per pair: output layers (and their SHA-256 ztags) split over them

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
        y.ztag = layer_ztag(g.canon_tag, y.nonce_lo, y.nonce_hi);
        g.C.layers[slot] = y;
    }
}

// ---------------------------------------------------------------- aggregation + emit
struct fresh_layout {
    // byte offsets into dynamic LDS; ks = slots per accumulator array
    uint32_t acc, boff, members, tkey, a_w, a_inf, b_w, b_inf, pm, remap, misc, total, ks;
};

// misc u32 word indices
enum : int { MF_PART = 0 /* <= 16 scan partials */, MF_INVALID = 16, MF_TOTAL = 17, MF_IDENT = 18,
             MF_KEEP = 20 /* u64 */, MF_WAVELP = 24 /* 16 x u64 */,
             MF_HDR = 56 /* 16: next pair's header record */, MF_WORDS = 72 };

__host__ __device__ inline uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

// Accumulators: six u64 arrays X0..X5 of ks slots (structure of arrays: a slot's u64 words sit
// 8 bytes apart across lanes, so random-slot atomics spread over 32 bank pairs and owner reads are
// contiguous). S1: X0..X2 = P limbs, X3..X5 = M limbs. From S2 on: P sum (X0 lo, X1 hi), M sum
// (X2, X3), X4 = G (u16 per product time), X5 = the writer map inv (u32 per emit position), both
// zero outside their use. boff / members: the slots of every libstdc++ bucket as a CSR (bucket
// offsets u32, slot ids u16), rebuilt when the bucket count changes (see k_ct_mul_fresh).
__host__ __device__ inline fresh_layout fresh_lds(uint32_t ks, uint32_t na, uint32_t nb, uint32_t nbk) {
    fresh_layout L;
    uint32_t o = 0;
    L.ks = ks;
    L.acc = o;   o = align16(o + ks * 48u);           // 2 channels x 3 u64 limbs per key slot
    L.boff = o;  o = align16(o + nbk * 4u);
    L.members = o; o = align16(o + ks * 2u);
    L.tkey = o;  o = align16(o + ks * 4u);
    L.a_w = o;   o = align16(o + na * 16u);
    L.a_inf = o; o = align16(o + na * 4u);
    L.b_w = o;   o = align16(o + nb * 16u);
    L.b_inf = o; o = align16(o + nb * 4u);
    L.pm = o;    o = align16(o + kFreshLayersMax * 8u);   // parent masks of C's layers
    L.remap = o; o = align16(o + kFreshLayersMax * 4u);
    L.misc = o;  o = align16(o + MF_WORDS * 4u);
    L.total = o;
    return L;
}


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
struct fresh_hdr {
    uint64_t pr;
    uint32_t LA, LB, nA, nB;
    uint64_t aeo, beo, alo, blo, clo, ceo;
    uint32_t nbk;        // libstdc++ bucket count after reserve(|A.E||B.E|)
    uint64_t nb_magic;   // its fastmod64 multiplier
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

__device__ __forceinline__ fresh_hdr load_hdr(argp g, uint64_t pr) {
    fresh_hdr h{};
    h.pr = pr;
    if (pr != kNoPair) {
        const recp r = (recp)g->recs + pr;
        h.LA = r->LA; h.LB = r->LB;
        h.nA = r->shape & 0xFFFFu; h.nB = r->shape >> 16;
        h.aeo = r->aeo; h.beo = r->beo; h.ceo = r->ceo;
        h.alo = r->alo; h.blo = r->blo; h.clo = r->clo;
        h.nbk = r->nbk;
        h.nb_magic = r->nb_magic;
    }
    return h;
}

// The next pair's header is loaded by VECTOR memory (lane l < 16 of every wave holds dword l of
// its record): its wait is vmcnt, so it never holds up an LDS wait the way a scalar load would
// (lgkmcnt counts both, and scalar loads return out of order).
__device__ __forceinline__ uint32_t hdr_issue(const fresh_rec* recs, uint64_t n_pairs, uint64_t q) {
    if (q >= n_pairs) return 0;
    return ((const uint32_t*)(recs + q))[threadIdx.x & 15u];
}

__device__ __forceinline__ fresh_hdr hdr_next(argp g, uint32_t v, uint64_t q, uint64_t n_pairs) {
    fresh_hdr h{};
    h.pr = kNoPair;
    if (q >= n_pairs) return h;
    auto rd = [&](int k) { return (uint32_t)__builtin_amdgcn_readlane(v, k); };
    const uint32_t w15 = rd(15);
    if ((w15 & 0xFFFFu) == 0) return load_hdr(g, next_small(g, q + gridDim.x));   // not a fresh pair
    h.pr = q;
    h.aeo = ((uint64_t)rd(1) << 32) | rd(0);
    h.beo = ((uint64_t)rd(3) << 32) | rd(2);
    h.ceo = ((uint64_t)rd(5) << 32) | rd(4);
    h.alo = ((uint64_t)rd(7) << 32) | rd(6);
    h.blo = ((uint64_t)rd(9) << 32) | rd(8);
    h.clo = ((uint64_t)rd(11) << 32) | rd(10);
    h.nb_magic = ((uint64_t)rd(13) << 32) | rd(12);
    const uint32_t shape = rd(14);
    h.nA = shape & 0xFFFFu;
    h.nB = shape >> 16;
    h.nbk = w15 & 0xFFFFu;
    h.LA = (w15 >> 16) & 0xFFu;
    h.LB = w15 >> 24;
    return h;
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

__device__ __forceinline__ fresh_pref prefetch_pair(argp g, const fresh_hdr& h) {
    // branch-free and unconditional: every lane loads a valid address (a clamped index, or the
    // argument block itself when there is no pair / no edge), so the waitcnt pass never has to
    // drain earlier loads (or the previous pair's output stores) before issuing these; lanes past
    // the counts ignore what they loaded
    const uint32_t t = threadIdx.x;
    const bool live = h.pr != kNoPair;
    using gp64 = const __attribute__((address_space(1))) uint64_t*;   // global: never a flat load
    using gpl = const __attribute__((address_space(1))) uint32_t*;
    const gp64 dummy = (gp64)(uint64_t)g;
    const bool okA = live && h.nA, okB = live && h.nB;
    const uint64_t ea = okA ? h.aeo + min(t, h.nA - 1u) : 0ull;
    const uint64_t eb = okB ? h.beo + min(t, h.nB - 1u) : 0ull;
    const gp64 am = okA ? (gp64)g->A.meta : dummy;
    const gp64 al = okA ? (gp64)g->A.w_lo : dummy;
    const gp64 ah = okA ? (gp64)g->A.w_hi : dummy;
    const gp64 bm = okB ? (gp64)g->B.meta : dummy;
    const gp64 bl = okB ? (gp64)g->B.w_lo : dummy;
    const gp64 bh = okB ? (gp64)g->B.w_hi : dummy;
    const uint32_t nl = h.LA + h.LB;
    const uint32_t l = min(t, nl - 1u);
    const gpl rec = !(live && nl) ? (gpl)dummy
                    : l < h.LA    ? (gpl)(g->A.layers + h.alo + l)
                                  : (gpl)(g->B.layers + h.blo + (l - h.LA));
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
                                           uint32_t* misc) {
    const uint32_t t = threadIdx.x;
    if (h.pr == kNoPair) return;
    if (t < h.nA) {
        const uint32_t la = meta_layer(f.am), idx = meta_idx(f.am), ch = meta_ch(f.am);
        if (la >= h.LA || idx >= Bm || ch > 1) misc[MF_INVALID] = 1;
        const fp w = fp_canon(f.al, f.ah);
        a_w[t] = make_ulonglong2(w.lo, w.hi);
        a_inf[t] = idx | ((la * h.LB * Bm) << 12) | (ch << 24);   // S1 adds A and B records (see there)
    }
    if (t < h.nB) {
        const uint32_t lb = meta_layer(f.bm), idx = meta_idx(f.bm), ch = meta_ch(f.bm);
        if (lb >= h.LB || idx >= Bm || ch > 1) misc[MF_INVALID] = 1;
        const fp w = fp_canon(f.bl, f.bh);
        b_w[t] = make_ulonglong2(w.lo, w.hi);
        b_inf[t] = idx | ((lb * Bm) << 12) | (ch << 24);
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
            const uint32_t lp = t - base;   // < 64: float quotient is exact after floor
            const uint32_t la = (uint32_t)__float2uint_rd(((float)lp + 0.5f) / (float)h.LB);
            m = (1ull << la) | (1ull << (h.LA + lp - la * h.LB));
        }
        pm[t] = m;
    }
}

template <int BS, int MINW>
__global__ __launch_bounds__(BS, MINW) void k_ct_mul_fresh(const mul_fresh_args* __restrict__ gp, fresh_layout Ls) {
    constexpr int KI = (kFreshKeysMax + BS - 1) / BS;    // key slots owned per thread: s = tid + k*BS
    constexpr int NW = BS / 64;
    constexpr int U = 4;                                 // unrolled product rounds per thread in S1
    static_assert(BS == (int)kFreshThreads && BS >= (int)kFreshEdgesMax && NW <= 16, "fresh geometry");
    // Arguments live in a device buffer; the pointer is laundered after every barrier so the
    // compiler re-reads fields from the scalar cache on use instead of pinning ~60 SGPRs of
    // pointers for the whole loop (which spilled into VGPRs and scratch).
    argp gq = launder((uint64_t)gp);
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    unsigned long long* acc = (unsigned long long*)(lds + Ls.acc);
    const uint32_t KSM = Ls.ks;                           // accumulator array stride (slots)
    unsigned long long* X4 = acc + 4u * KSM;
    unsigned long long* X5 = acc + 5u * KSM;
    uint32_t* boff = (uint32_t*)(lds + Ls.boff);
    uint16_t* members = (uint16_t*)(lds + Ls.members);
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
    const uint32_t Bm = gq->Bm;
    // The slots a thread owns (s = tid + k*BS) are the same for every pair: their (lp, r) split
    // is computed once, and their libstdc++ buckets once per distinct bucket count. Packed per
    // slot: bucket (15 bits) | r << 15 (11 bits) | lp << 26 (6 bits; only slots < KS are used,
    // where lp < |C.L| <= 64).
    uint32_t sinfo[KI];
    uint32_t nbk_c = 0;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
        const uint32_t s = tid + (uint32_t)k * BS;
        const uint32_t lp = s / Bm;
        sinfo[k] = ((s - lp * Bm) << 15) | (min(lp, 63u) << 26);
    }
    // The other slots of each owned slot's bucket (a static property of the bucket count and B):
    // up to 4 cached as packed u16 pairs; gcnt = their number | CSR start << 16 (more than 4 are
    // read from `members`).
    uint32_t gmem[KI][2], gcnt[KI];
#pragma unroll
    for (int k = 0; k < KI; ++k) { gmem[k][0] = gmem[k][1] = 0; gcnt[k] = 0; }
#define SLOT_LP(k) (sinfo[k] >> 26)
#define SLOT_R(k) ((sinfo[k] >> 15) & 0x7FFu)
#define SLOT_BK(k) (sinfo[k] & 0x7FFFu)

    // one-time clear: accumulators 0, first-insert times INF
    for (uint32_t w = tid; w < (Ls.tkey - Ls.acc) / 16u; w += BS) ((uint4*)lds)[Ls.acc / 16u + w] = make_uint4(0, 0, 0, 0);
    for (uint32_t s = tid; s < gq->ks_max; s += BS) tkey[s] = kTInf;
    if (tid < MF_WORDS) misc[tid] = 0;
    __syncthreads();

#ifdef PVAC_PHASE_STAMPS
    unsigned long long st_acc_[kStampPhases] = {};
    unsigned long long st_last_ = __builtin_amdgcn_s_memtime();
#endif
    const fresh_rec* const recs = gq->recs;
    const uint64_t n_pairs = gq->A.n;
    fresh_hdr cur = load_hdr(gq, next_small(gq, blockIdx.x));
    stage_pair(prefetch_pair(gq, cur), cur, Bm, a_w, a_inf, b_w, b_inf, pm, misc);
    __syncthreads();
    PHASE_STAMP(0);

    while (cur.pr != kNoPair) {
        gq = launder(gq);
        const uint64_t qn = cur.pr + gridDim.x;
        // The last wave is the control wave: it issues no global stores (it skips the S5 writer),
        // so waiting for its header load never waits for output stores (vmcnt counts both, in
        // order). It loads the next pair's record now and relays it through LDS after S1.
        const uint32_t hv = wave == NW - 1 ? hdr_issue(recs, n_pairs, qn) : 0u;
        auto hdr_publish = [&]() {
            if (wave == NW - 1 && lane < 16) misc[MF_HDR + lane] = hv;
        };
        const uint64_t pr = cur.pr;
        const uint32_t LA = cur.LA, LB = cur.LB, nA = cur.nA, nB = cur.nB;
        const uint32_t LP = LA * LB, KS = LP * Bm, n = nA * nB;
        const uint32_t base = LA + LB, Lc = base + LP;
        const uint32_t nbk = cur.nbk;
        // G[t] and inv[p] in the slot tails (see fresh_lds)
        auto G_at = [&](uint32_t t) { return (uint16_t*)X4 + t; };
        auto inv_at = [&](uint32_t q) { return (uint32_t*)X5 + q; };

        if (misc[MF_INVALID]) {   // invalid references: reject the pair (reference behaviour is UB)
            __syncthreads();
            if (tid == 0) {
                gq->pair_status[pr] = 2;
                gq->C.l_cnt[pr] = 0;
                gq->C.e_cnt[pr] = 0;
                misc[MF_INVALID] = 0;
            }
            hdr_publish();
            __syncthreads();
            const fresh_hdr nx = hdr_next(gq, misc[MF_HDR + (lane & 15)], qn, n_pairs);
            stage_pair(prefetch_pair(gq, nx), nx, Bm, a_w, a_inf, b_w, b_inf, pm, misc);
            __syncthreads();
            cur = nx;
            continue;
        }

        // ---- bucket groups: on a new reserve() size (workgroup-uniform), hash every slot
        //      s < ks_max to its libstdc++ bucket and group the slots by bucket (counting sort in
        //      LDS). Each thread caches the other slots of its own slots' buckets, so S2c reads their
        //      keys directly instead of discovering them through per-pair bucket chains.
        if (nbk != nbk_c) {
            const uint32_t ksa = gq->ks_max;
            const fastmod64 fm{nbk, cur.nb_magic};
#pragma unroll
            for (int k = 0; k < KI; ++k) {
                const uint32_t b = (uint32_t)fmod64((((uint64_t)SLOT_LP(k) << 32) | SLOT_R(k)) * kGolden, fm);
                sinfo[k] = (sinfo[k] & ~0x7FFFu) | b;   // std::hash -> bucket
            }
            for (uint32_t w = tid; w < nbk; w += BS) boff[w] = 0;
            __syncthreads();
#pragma unroll
            for (int k = 0; k < KI; ++k)
                if (tid + (uint32_t)k * BS < ksa) atomicAdd(&boff[SLOT_BK(k)], 1u);
            __syncthreads();
            {   // exclusive scan of the bucket sizes in place
                const uint32_t per = (nbk + BS - 1) / BS, b0 = tid * per;
                uint32_t local = 0;
                for (uint32_t b = b0; b < b0 + per && b < nbk; ++b) local += boff[b];
                uint32_t tot;
                uint32_t run = block_exclusive_scan<BS>(local, misc + MF_PART, tot);
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
                if (s < ksa) members[atomicAdd(&boff[SLOT_BK(k)], 1u)] = (uint16_t)s;
            }
            __syncthreads();   // boff[b] is now the END of bucket b's slots
#pragma unroll
            for (int k = 0; k < KI; ++k) {
                const uint32_t s = tid + (uint32_t)k * BS;
                const uint32_t b = SLOT_BK(k);
                uint32_t g0 = 0, g1 = 0, c = 0, start = 0;
                if (s < ksa) {
                    const uint32_t end = boff[b];
                    start = b ? boff[b - 1] : 0u;
                    for (uint32_t q = start; q < end; ++q) {
                        const uint32_t m = members[q];
                        if (m == s) continue;
                        g0 |= c == 0 ? m : (c == 1 ? m << 16 : 0u);
                        g1 |= c == 2 ? m : (c == 3 ? m << 16 : 0u);
                        ++c;
                    }
                }
                gmem[k][0] = g0;
                gmem[k][1] = g1;
                gcnt[k] = c | (start << 16);
            }
            nbk_c = nbk;
            __syncthreads();   // boff is rebuilt in place by the next change
        }

        // ---- S1: all |A.E||B.E| products into LDS limb accumulators + first-insert times.
        //      Product t = i*|B.E| + j (the reference's loop order) is taken by thread t mod BS,
        //      so every wave but the first runs ceil(n/BS) - 1 or ceil(n/BS) rounds. Staged
        //      records: idx | layer-slot base << 12 | ch << 24, so one add of an A and a B record
        //      gives idx_i + idx_j, the product layer's slot base and ch_i + ch_j (bit 24 = P/M).
        if (n) {
            const uint32_t mdiv = (1u << 24) / nB + 1u;   // i = ((t << 8) * mdiv) >> 32, exact for t < 2^12
            for (uint32_t t0 = (uint32_t)tid; t0 < n; t0 += U * BS) {   // one pass for n <= U*BS
                // all operand reads first (clamped in-range indices), so their latency is paid once
                ulonglong2 x[U], y[U];
                uint32_t sum[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t t = min(t0 + (uint32_t)u * BS, n - 1u);
                    const uint32_t i = __umulhi(t << 8, mdiv);
                    const uint32_t j = t - i * nB;
                    x[u] = a_w[i];
                    y[u] = b_w[j];
                    sum[u] = a_inf[i] + b_inf[j];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t t = t0 + (uint32_t)u * BS;
                    if (t < n) {
                        uint32_t r = sum[u] & 0xFFFu;
                        r = min(r, r - Bm);   // (idx_i + idx_j) mod B: r - B wraps when r < B
                        const uint32_t s = ((sum[u] >> 12) & 0xFFFu) + r;
                        const uint32_t chn = (sum[u] >> 24) & 1u;   // 0 = P (same sign), 1 = M
                        uint64_t x0, x1, l0, l1, l2;
#ifdef PVAC_EXP_NOMUL
                        x0 = x[u].x ^ y[u].x; x1 = (x[u].y ^ y[u].y) & 0x7FFFFFFFFFFFFFFFull;
#else
                        fp_mul_fold1(fp{x[u].x, x[u].y}, fp{y[u].x, y[u].y}, x0, x1);
#endif
                        fp_split3_128(x0, x1, l0, l1, l2);
                        unsigned long long* q = acc + chn * (3u * KSM) + s;
                        atomicAdd(q, (unsigned long long)l0);
                        atomicAdd(q + KSM, (unsigned long long)l1);
                        atomicAdd(q + 2u * KSM, (unsigned long long)l2);
                        atomicMin(&tkey[s], t);
                    }
                }
            }
        }
        PHASE_STAMP_SYNC(11);
        hdr_publish();   // its load has had S1 to land
        PHASE_STAMP(10);
        __syncthreads();
        gq = launder(gq);
        PHASE_STAMP(1);
        // S2a..S4 are chains of short dependent steps; S1 (products) and S5 (stores) are bulk work:
        // the workgroup in its ordering phases is served first by the arbiter of a shared SIMD
        __builtin_amdgcn_s_setprio(1);
        // next pair's header (from the control wave) and raw inputs: the data loads stay in
        // flight until stage_pair in S3
        const fresh_hdr nxt = hdr_next(gq, misc[MF_HDR + (lane & 15)], qn, n_pairs);
        const fresh_pref pf = prefetch_pair(gq, nxt);

        // ---- S2a: every thread owns key slots s = tid + k*BS: fold the limbs, clear them, hash
        //      the key to its libstdc++ bucket
        fp sumP[KI], sumM[KI];
        uint32_t kt[KI], eb[KI];
        uint64_t myor = 0;
        // all reads first (the stores below would otherwise pin every later read behind them: same
        // LDS array), then the arithmetic, then the exchanges and in-place stores
        uint64_t lim[KI][6];
#pragma unroll
        for (int k = 0; k < KI; ++k) {
            const uint32_t s = tid + (uint32_t)k * BS;
            kt[k] = s < KS ? tkey[s] : kTInf;
        }
#pragma unroll
        for (int k = 0; k < KI; ++k) {
            const uint32_t s = tid + (uint32_t)k * BS;
            const unsigned long long* q = acc + min(s, KS - 1u);
#pragma unroll
            for (int c = 0; c < 6; ++c) lim[k][c] = q[c * KSM];
        }
        PHASE_STAMP_SYNC(12);
        // branch-free: empty slots hold zero limbs (slots past KS are masked by kt), so the six
        // folds form one block the scheduler interleaves (their carry chains hide each other's
        // VALU hazards)
#pragma unroll
        for (int k = 0; k < KI; ++k) {
#ifdef PVAC_EXP_NOFOLD
            sumP[k] = fp{lim[k][0] ^ lim[k][2], lim[k][1] & 0x7FFFFFFFFFFFFFFFull};
            sumM[k] = fp{lim[k][3] ^ lim[k][5], lim[k][4] & 0x7FFFFFFFFFFFFFFFull};
#else
            sumP[k] = fp_fold3_lazy(lim[k][0], lim[k][1], lim[k][2]);
            sumM[k] = fp_fold3_lazy(lim[k][3], lim[k][4], lim[k][5]);
#endif
        }
#pragma unroll
        for (int k = 0; k < KI; ++k) {
            const uint32_t e = (fp_nonzero(sumP[k]) ? 1u : 0u) | (fp_nonzero(sumM[k]) ? 2u : 0u);
            eb[k] = kt[k] != kTInf ? e : 0u;
            myor |= eb[k] ? 1ull << SLOT_LP(k) : 0ull;
        }
        PHASE_STAMP(13);
        // key sums in place over the slot's own limbs (a zero sum is the zero unit), tail zeroed
#pragma unroll
        for (int k = 0; k < KI; ++k) {
            const uint32_t s = tid + (uint32_t)k * BS;
            if (kt[k] != kTInf) {
                unsigned long long* q = acc + s;
                q[0] = sumP[k].lo; q[KSM] = sumP[k].hi;
                q[2u * KSM] = sumM[k].lo; q[3u * KSM] = sumM[k].hi;
                q[4u * KSM] = 0; q[5u * KSM] = 0;
            }
        }
        myor = wave_or_u64(myor);
        if (lane == 0) wave_lp[wave] = myor;
        // key entry: first-insert time (12 bits) | channels present << 23 (empty slots keep INF)
#pragma unroll
        for (int k = 0; k < KI; ++k)
            if (kt[k] != kTInf) tkey[tid + (uint32_t)k * BS] = kt[k] | (eb[k] << 23);
        PHASE_STAMP_SYNC(14);
        __syncthreads();
        gq = launder(gq);
        PHASE_STAMP(2);

        // ---- S2c: bucket first-insert time, rank inside the bucket and bucket edge count from the
        //      keys of the other slots of the bucket (one LDS round trip: their entries are read
        //      together); wave 0 then runs compact_layers (encrypt.hpp:73-104) as a bitmask closure
        uint32_t tb[KI], within[KI], cE[KI];
        {
            auto take = [&](int k, uint32_t x) {   // another slot's key entry (INF: empty slot)
                if (x != kTInf) {
                    const uint32_t t2 = x & 0xFFFu, e2 = __popc(x >> 23);
                    tb[k] = t2 < tb[k] ? t2 : tb[k];
                    within[k] += t2 > kt[k] ? e2 : 0u;
                    cE[k] += e2;
                }
            };
            uint32_t v[KI][4];
#pragma unroll
            for (int k = 0; k < KI; ++k) {
                tb[k] = kt[k];
                within[k] = 0;
                cE[k] = __popc(eb[k]);
                const uint32_t g = gcnt[k] & 0xFFFFu;
                const uint32_t c = (kt[k] != kTInf && g <= 4u) ? g : 0u;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t m = (gmem[k][j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                    v[k][j] = (uint32_t)j < c ? tkey[m] : kTInf;
                }
            }
#pragma unroll
            for (int k = 0; k < KI; ++k)
#pragma unroll
                for (int j = 0; j < 4; ++j) take(k, v[k][j]);
#pragma unroll
            for (int k = 0; k < KI; ++k) {   // buckets of more than five slots: the whole group from LDS
                const uint32_t g = gcnt[k] & 0xFFFFu;
                if (kt[k] != kTInf && g > 4u) {
                    const uint32_t s = tid + (uint32_t)k * BS, q0 = gcnt[k] >> 16;
                    for (uint32_t q = q0; q <= q0 + g; ++q) {
                        const uint32_t m = members[q];
                        if (m != s) take(k, tkey[m]);
                    }
                }
            }
        }
        PHASE_STAMP(15);
#pragma unroll
        for (int k = 0; k < KI; ++k)
            if (kt[k] != kTInf && tb[k] == kt[k]) *G_at(tb[k]) = (uint16_t)cE[k];
        if (wave == 0) {
            __builtin_amdgcn_s_setprio(3);   // the closure holds up the barrier below
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
                remap[lane] = ((keep >> lane) & 1ull)   // popcount of the kept layers below this one
                                  ? __builtin_amdgcn_mbcnt_hi((uint32_t)(keep >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)keep, 0u))
                                  : kTInf;
            if (lane == 0) {
                *(uint64_t*)(misc + MF_KEEP) = keep;
                misc[MF_IDENT] = keep == all;
            }
            __builtin_amdgcn_s_setprio(1);
        }
        __syncthreads();
        gq = launder(gq);
        PHASE_STAMP(4);

        // ---- S3: exclusive SUFFIX scan of G over t in [0, n): emit offset of each bucket group.
        //      One wave (the last: it holds no input records, edges <= 256) scans with no barrier:
        //      lane l owns the aligned t-chunk [(63 - l) c, (64 - l) c) (c a multiple of 8; only
        //      8-groups that start below n are touched, and their entries at t >= n - which lie in
        //      G's zero tail or the zero writer map - stay zero), so lane order is suffix order. Meanwhile the
        //      other waves stage the next pair: a_w/a_inf/b_w/b_inf were last read in S1 and pm in
        //      the S2c closure, and the prefetched loads have had S2a and S2c to land.
        if (wave == NW - 1) {
            __builtin_amdgcn_s_setprio(3);   // the scan is the phase's critical path
            const uint32_t c8 = (n + 511u) / 512u;   // b128 chunks (8 times) per lane
            uint4* gv = (uint4*)X4;
            const uint32_t q0 = (63u - (uint32_t)lane) * c8;
            uint32_t local = 0;
            const uint32_t qn = min(c8, ((n + 7u) >> 3) > q0 ? ((n + 7u) >> 3) - q0 : 0u);   // chunks with t < n
            for (uint32_t q = 0; q < qn; ++q) {
                const uint4 v = gv[q0 + q];
                local += (v.x & 0xFFFFu) + (v.x >> 16) + (v.y & 0xFFFFu) + (v.y >> 16) + (v.z & 0xFFFFu) +
                         (v.z >> 16) + (v.w & 0xFFFFu) + (v.w >> 16);
            }
            const uint32_t incl = wave_incl_scan_u32(local);
            uint32_t run = incl - local;
            for (uint32_t q = qn; q-- > 0;) {   // t descending inside the chunk
                const uint4 v = gv[q0 + q];
                uint32_t w[4] = {v.x, v.y, v.z, v.w};
                const uint32_t tq = (q0 + q) * 8u;
#pragma unroll
                for (int h = 3; h >= 0; --h) {
                    const uint32_t hi = w[h] >> 16, lo = w[h] & 0xFFFFu;
                    const uint32_t ohi = run;
                    run += hi;
                    const uint32_t olo = run;
                    run += lo;
                    const uint32_t t = tq + 2u * (uint32_t)h;
                    w[h] = (t < n ? olo : 0u) | ((t + 1u < n ? ohi : 0u) << 16);
                }
                gv[q0 + q] = make_uint4(w[0], w[1], w[2], w[3]);
            }
            if (lane == 63) misc[MF_TOTAL] = run;   // lane 63 owns t = 0: its running sum is the total
            __builtin_amdgcn_s_setprio(1);
        }
        stage_pair(pf, nxt, Bm, a_w, a_inf, b_w, b_inf, pm, misc);
        __syncthreads();
        gq = launder(gq);
        PHASE_STAMP(5);

        // ---- S4: emit positions
        const uint32_t total = misc[MF_TOTAL];
        // guard_budget (encrypt.hpp:106-111): above edge_budget the reference runs compact_edges,
        // whose output is (layer, idx, P before M) order; product edges are already unique per
        // (layer, idx, ch) and nonzero, so it only re-orders them.
        const bool canonical = (gq->flags & PVAC_MUL_ORDER_CANONICAL) != 0 || total > gq->edge_budget;
        // reference (hash) order: owners publish their edges' positions (inv[p]) and a writer pass
        // stores positions p = tid, tid + BS, ... contiguously (total <= 2 KS: inv always fits).
        // Canonical order stores from the owners instead.
        const bool gather = !canonical;
        const uint64_t ceo = cur.ceo;
        const bool ident = misc[MF_IDENT] != 0;
        if (gather) {
            // writer entry: slot (11 bits) | channel << 11 | idx << 12 | output layer << 23
#pragma unroll
            for (int k = 0; k < KI; ++k) {
                const uint32_t s = tid + (uint32_t)k * BS;
                if (kt[k] != kTInf) {
                    tkey[s] = kTInf;
                    uint32_t p = *G_at(tb[k]) + within[k];
                    if (eb[k]) {
                        const uint32_t lid = ident ? base + SLOT_LP(k) : remap[base + SLOT_LP(k)];
                        const uint32_t e = s | (SLOT_R(k) << 12) | (lid << 23);
                        if (eb[k] & 1u) *inv_at(p++) = e;
                        if (eb[k] & 2u) *inv_at(p) = e | (1u << 11);
                    }
                }
            }
        } else {
            uint32_t rowbase = 0;
#pragma unroll
            for (int k = 0; k < KI; ++k) {
                const uint32_t s = tid + (uint32_t)k * BS;
                const bool own = kt[k] != kTInf;
                const uint32_t hp = own ? *G_at(tb[k]) + within[k] : 0u;
                uint32_t p = hp;
                if (canonical) {   // workgroup-uniform: row k = slots k*BS.., i.e. slot order
                    uint32_t rowtot;
                    p = rowbase + block_exclusive_scan<BS>(__popc(eb[k]), misc + MF_PART, rowtot);
                    rowbase += rowtot;
                }
                if (own) tkey[s] = kTInf;
                if (eb[k]) {
                    const uint32_t idx = SLOT_R(k);
                    const uint32_t lid = ident ? base + SLOT_LP(k) : remap[base + SLOT_LP(k)];
                    uint32_t* sp = gq->salt_pos;
                    if (eb[k] & 1u) {
                        const ulonglong2 w = make_ulonglong2(acc[s], acc[KSM + s]);
                        gq->C.meta[ceo + p] = make_meta(lid, idx, 0);
                        gq->C.w_lo[ceo + p] = w.x;
                        gq->C.w_hi[ceo + p] = w.y;
                        if (sp) sp[ceo + p] = hp;   // salts are drawn in hash order (arithmetic.hpp:90-101)
                        ++p;
                    }
                    if (eb[k] & 2u) {
                        const ulonglong2 w = make_ulonglong2(acc[2u * KSM + s], acc[3u * KSM + s]);
                        gq->C.meta[ceo + p] = make_meta(lid, idx, 1);
                        gq->C.w_lo[ceo + p] = w.x;
                        gq->C.w_hi[ceo + p] = w.y;
                        if (sp) sp[ceo + p] = hp + (eb[k] & 1u);
                    }
                }
                if (own) {
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[c * KSM + s] = 0;
                }
            }
        }
        const uint64_t keep = *(const uint64_t*)(misc + MF_KEEP);
        if (!misc[MF_IDENT] && wave == 1) {
            // k_mul_layers_fresh wrote identity placement; compact in place (remap[l] <= l, and
            // every lane of this wave loads before any lane stores)
            const uint32_t l = lane;
            const uint64_t clo = cur.clo;
            pvac_layer y{};
            if (l < Lc) y = gq->C.layers[clo + l];
            if (l < Lc && ((keep >> l) & 1ull)) {
                if (y.rule == 1) {
                    y.pa = y.pa < Lc ? remap[y.pa] : kTInf;
                    y.pb = y.pb < Lc ? remap[y.pb] : kTInf;
                }
                gq->C.layers[clo + remap[l]] = y;
            }
        }
        if (tid == 0) {
            gq->C.e_cnt[pr] = total;
            gq->C.l_cnt[pr] = (uint64_t)__popcll(keep);
            gq->pair_status[pr] = canonical ? 1 : 0;
        }
        __syncthreads();
        gq = launder(gq);
        PHASE_STAMP(6);
        __builtin_amdgcn_s_setprio(0);

        // ---- S5 (reference order): coalesced writer over emit positions; clears what it read
        if (gather) {
            uint32_t* sp = gq->salt_pos;
            // waves 0..NW-2 only: the control wave keeps its vector-memory queue free of stores
            for (uint32_t p = tid; p < total && wave != NW - 1; p += BS - 64) {
                uint32_t* ip = inv_at(p);
                const uint32_t e = *ip;
                const uint32_t s = e & 0x7FFu, ch = (e >> 11) & 1u, idx = (e >> 12) & 0x7FFu, lid = e >> 23;
                unsigned long long* q = acc + (2u * ch) * KSM + s;
                const ulonglong2 w = make_ulonglong2(q[0], q[KSM]);
                *ip = 0;
                q[0] = 0;
                q[KSM] = 0;
#ifndef PVAC_EXP_NOWRITE
                gq->C.meta[ceo + p] = make_meta(lid, idx, ch);
                gq->C.w_lo[ceo + p] = w.x;
                gq->C.w_hi[ceo + p] = w.y;
                if (sp) sp[ceo + p] = p;   // hash order == emit order here
#else
                if (w.x == 0x1234567 && lid == 77) gq->C.w_hi[ceo + p] = w.y + idx;
#endif
            }
        }
        PHASE_STAMP(8);

        // ---- clear G for the next pair (the rest was cleared by its readers)
        for (uint32_t q = tid; q < (n + 3u) / 4u; q += BS) X4[q] = 0;   // G
        PHASE_STAMP(7);
        __syncthreads();
        PHASE_STAMP(9);
        cur = nxt;
    }
#undef SLOT_LP
#undef SLOT_R
#undef SLOT_BK
#ifdef PVAC_PHASE_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < 4096)
        for (int p = 0; p < kStampPhases; ++p) g_fresh_stamps[blockIdx.x * kStampPhases + p] = st_acc_[p];
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
    const fresh_layout L = fresh_lds(a.ks_max, a.na_max, a.nb_max, a.buckets_max);
    // G (one u16 per product time) lives in the slot tails: 4 per slot (the plan keeps |A.E||B.E|
    // <= 3 |A.L||B.L|B for fresh-path pairs)
    if ((uint64_t)a.prod_max > 4ull * a.ks_max) return hipErrorInvalidValue;
    if (L.total > 160u * 1024u) return hipErrorInvalidValue;
    const int per_cu = L.total <= 80u * 1024u ? 2 : 1;
    uint64_t blocks = (uint64_t)num_cus * per_cu;
    if (blocks > a.A.n) blocks = a.A.n;
    hipLaunchKernelGGL((k_ct_mul_fresh<kFreshThreads, 4>), dim3((unsigned)blocks), dim3(kFreshThreads), L.total, st,
                       args_dev, L);
    return hipGetLastError();
}

}  // namespace pvhip
