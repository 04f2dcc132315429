// k_sigma.hip — sigma_from_H (crypto/matrix.hpp:267-303) and gen_H (matrix.hpp:191-251)
// on CDNA4.
//
// sigma = XOR of x_col_wt columns of the public sparse matrix H, then err_wt noise-bit
// flips. Column / row choices come from prg_choose_k (matrix.hpp:15-92): a SHA-256
// counter-mode stream over (label || le64 words... || le64 ctr), four little-endian u64
// draws per digest, rejection-bounded to [0, N), and the FIRST k DISTINCT values in draw
// order.
//
// Mapping: one wavefront per edge. Lanes 0..31 run the "pvac.dom.x_seed" stream and lanes
// 32..63 the "pvac.dom.noise" stream, each lane one counter per pass (4 draws). The first
// 64-byte block of both messages does not depend on the counter, so it is compressed once
// per edge (midstate) and each pass costs one compression per lane. Exact "first k
// distinct in draw order" is restored per pass: a draw is new if its value was selected by
// no earlier pass (LDS bitmap) and by no earlier position of this pass (wave shuffles);
// ranks come from a 32-lane prefix count. Selected columns are expanded through the sparse
// H rows with LDS atomic XOR into a 1 KiB sigma image, written out as one 16-byte store per
// lane.
#include <algorithm>
#include <vector>
#include <cstdlib>
#include <cstring>
#include <string>

#include "common.hpp"
#include "sha256.hpp"
#include "sigma.hpp"

namespace pvhip {

namespace {

constexpr int kSigBlock = 256;   // 4 waves, one edge each at a time
constexpr uint32_t kMaxPasses = 4096;   // >> the ~2-3 passes a random stream needs

template <int N>
struct cstr { char c[N]; };

// Pack message byte `b` at absolute position `pos` of a message into block `blk` words.
__device__ __forceinline__ void put(uint32_t (&w)[16], int blk, int pos, uint32_t b) {
    const int p = pos - 64 * blk;
    if (p >= 0 && p < 64) w[p >> 2] |= (b & 0xFFu) << (24 - 8 * (p & 3));
}

// Block `blk` of SHA-256 padding of the message  label(LL) || le64 words[NW] || le64 ctr.
template <int LL, int NW>
__device__ __forceinline__ void build_block(uint32_t (&w)[16], int blk, const char* label, const uint64_t* words,
                                            uint64_t ctr) {
    constexpr int T = LL + 8 * NW + 8;
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = 0;
#pragma unroll
    for (int i = 0; i < LL; ++i) put(w, blk, i, (uint32_t)label[i]);
#pragma unroll
    for (int k = 0; k < NW; ++k)
#pragma unroll
        for (int i = 0; i < 8; ++i) put(w, blk, LL + 8 * k + i, (uint32_t)(words[k] >> (8 * i)));
#pragma unroll
    for (int i = 0; i < 8; ++i) put(w, blk, LL + 8 * NW + i, (uint32_t)(ctr >> (8 * i)));
    put(w, blk, T, 0x80u);
    // big-endian bit length in the last 8 bytes of the final block
    constexpr int nblk = (T + 9 + 63) / 64;
    if (blk == nblk - 1) {
        const uint64_t bits = (uint64_t)T * 8;
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
    }
}

__device__ constexpr char kLabX[] = "pvac.dom.x_seed";   // 15
__device__ constexpr char kLabN[] = "pvac.dom.noise";    // 14
__device__ constexpr char kLabH[] = "pvac.dom.h_gen";    // 14

// One pass of "first K distinct in draw order" over a group of GS lanes (GS = 32 or 64,
// groups aligned). Each lane holds 4 consecutive draws (positions 4*li+q of this pass).
// `bm` is the group's LDS bitmap of already-selected values. Returns, per q, the rank
// (0-based, over the whole selection) of a newly selected value, or -1.
template <int GS>
__device__ __forceinline__ void select_pass(const uint32_t (&val)[4], uint32_t* bm, uint32_t K, uint32_t& have,
                                            int (&rank)[4]) {
    const int lane = threadIdx.x & 63;
    const int li = lane & (GS - 1);
    const int gbase = lane & ~(GS - 1);
    bool isnew[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t v = val[q];
        isnew[q] = v != 0xFFFFFFFFu && !((bm[v >> 5] >> (v & 31)) & 1u);
    }
    // earlier positions of this pass with the same value
    for (int s = 0; s < GS; ++s) {
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
            const uint32_t o = __shfl(val[q2], gbase + s, 64);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool earlier = s < li || (s == li && q2 < q);
                if (earlier && o == val[q]) isnew[q] = false;
            }
        }
    }
    const uint32_t mine = (uint32_t)isnew[0] + isnew[1] + isnew[2] + isnew[3];
    // inclusive prefix over the group
    uint32_t x = mine;
#pragma unroll
    for (int d = 1; d < GS; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, GS);
        if (li >= d) x += y;
    }
    const uint32_t group_total = __shfl(x, gbase + GS - 1, 64);
    uint32_t r = have + x - mine;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        rank[q] = -1;
        if (isnew[q]) {
            if (r < K) {
                rank[q] = (int)r;
                atomicOr(&bm[val[q] >> 5], 1u << (val[q] & 31));
            }
            ++r;
        }
    }
    have = have + group_total < K ? have + group_total : K;
}

// The same selection for two 32-lane groups (X and noise streams of one edge), without the
// O(GS^2) shuffle scan. Each draw first reads the bitmap of values selected by EARLIER passes,
// then sets its bit with a returning atomic OR: a bit found already set marks an equal value
// elsewhere in THIS pass (LDS ops of a wave execute in issue order, so the reads see the
// pre-pass bitmap). Every duplicated value has at least one marked draw; a wave-uniform loop
// over the marked values finds all draws of each with four ballots and keeps only the first in
// draw order (position 4*lane + q). Bits of draws ranked >= K are set too, but K is then reached
// and the stream is finished. Selected set == select_pass<32>.
__device__ __forceinline__ void select_pass2x32(const uint32_t (&val)[4], uint32_t* bm, uint32_t K, uint32_t& have,
                                                int (&rank)[4]) {
    const int lane = threadIdx.x & 63;
    const uint64_t gmask = lane < 32 ? 0x00000000FFFFFFFFull : 0xFFFFFFFF00000000ull;
    bool isnew[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t v = val[q];
        isnew[q] = v != 0xFFFFFFFFu && !((bm[v >> 5] >> (v & 31)) & 1u);
    }
    uint32_t flagged = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (isnew[q]) {
            const uint32_t bit = 1u << (val[q] & 31);
            if (atomicOr(&bm[val[q] >> 5], bit) & bit) flagged |= 1u << q;
        }
    }
    uint64_t fl = __ballot(flagged != 0);
    while (fl) {   // wave-uniform; typically 0-2 iterations
        const int L = __ffsll((unsigned long long)fl) - 1;
        fl &= fl - 1;
        uint32_t fq = __builtin_amdgcn_readlane(flagged, L);
        const uint64_t lg = L < 32 ? 0x00000000FFFFFFFFull : 0xFFFFFFFF00000000ull;
        while (fq) {
            const int q0 = __ffs(fq) - 1;
            fq &= fq - 1;
            const uint32_t mine = q0 == 0 ? val[0] : q0 == 1 ? val[1] : q0 == 2 ? val[2] : val[3];
            const uint32_t v = __builtin_amdgcn_readlane(mine, L);
            uint64_t m[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) m[q] = __ballot(val[q] == v) & lg;
            const int f = __ffsll((unsigned long long)(m[0] | m[1] | m[2] | m[3])) - 1;   // first lane
            const int qf = ((m[0] >> f) & 1) ? 0 : ((m[1] >> f) & 1) ? 1 : ((m[2] >> f) & 1) ? 2 : 3;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (((m[q] >> lane) & 1) && !(lane == f && q == qf)) isnew[q] = false;
        }
    }
    (void)gmask;
    const uint32_t cnt = (uint32_t)isnew[0] + isnew[1] + isnew[2] + isnew[3];
    uint32_t x = wave_incl_scan_u32(cnt);
    const uint32_t lowtot = __builtin_amdgcn_readlane(x, 31);
    const uint32_t alltot = __builtin_amdgcn_readlane(x, 63);
    if (lane >= 32) x -= lowtot;
    const uint32_t group_total = lane < 32 ? lowtot : alltot - lowtot;
    uint32_t r = have + x - cnt;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        rank[q] = -1;
        if (isnew[q]) {
            if (r < K) rank[q] = (int)r;
            ++r;
        }
    }
    have = have + group_total < K ? have + group_total : K;
}

struct sig_args {
    pvac_ct_batch X;
    const uint64_t* salts;
    const uint32_t* salt_pos;
    const uint16_t* rows;
    const uint16_t* rows_fast;   // bank-sorted encoded rows (sigma_tables::rows_fast) or null
    const uint8_t* rows_delta;   // byte-delta rows (sigma_tables::rows_delta) or null
    const uint32_t* counts;
    uint32_t width;
    uint32_t full;   // every column has exactly width rows
    uint64_t canon;
    uint32_t n_bits, m_bits, x_col_wt, err_wt;
    uint32_t sub_blocks;
};

// per-wave LDS: sigma [m_bits/32] | bmX [n_bits/32] | bmN [m_bits/32] | cols [x_col_wt] u16 |
// noise rows [2 kNoiseWords] u16 | midstates [32 edges][2 streams][8] u32
// 6 blocks per CU (6 waves per SIMD): the compiler keeps the pass loop within 80 VGPRs without
// spills instead of hoisting the whole SHA-256 message schedule (149 VGPRs, 3 waves per SIMD)
#ifdef PVAC_EXP_SIG_MID16   // experiment builds only: 16-edge midstate batches, 7 workgroups per CU
constexpr uint32_t kMidBatch = 16;
constexpr int kSigMinBlocks = 7;
#elif defined(PVAC_EXP_SIG_MINB5)   // experiment builds only: 5 workgroups per CU (96 VGPRs, no spills)
constexpr uint32_t kMidBatch = 32;
constexpr int kSigMinBlocks = 5;
#else
constexpr uint32_t kMidBatch = 32;   // edges whose block-0 midstates one compression per lane covers
constexpr int kSigMinBlocks = 6;
#endif
// The delta path flips into four bank-interleaved copies of the image (word W of copy k at dword
// 4 W + k of the 1024 words sigma | bmX | bmN, dead after the selection), copy k = lane & 3: the 8
// lanes of a 32-lane ds_xor group that share a copy meet on 8 banks, instead of 32 lanes on 32
// (expected busiest bank 2.3 instead of 3.5 addresses per instruction), for one more VALU per flip
// (round 4: 35.2 -> 30.5 ms per 5.05 M edges, A/B in one process). The noise rows wait in
// kNoiseWords after the columns and are flipped with them; the output word is the XOR of its copies.
constexpr uint32_t kNoiseWords = 64;
#ifdef PVAC_EXP_SIG_COPY8   // experiment builds only: eight image copies (copy = lane & 7)
constexpr uint32_t kSigCopies = 8;
#else
constexpr uint32_t kSigCopies = 4;
#endif
// words of the image region (sigma | bmX | bmN, and the delta path's copies)
__host__ __device__ constexpr uint32_t sigma_img_words(uint32_t m_bits, uint32_t n_bits) {
    return m_bits / 32 + n_bits / 32 + m_bits / 32 > kSigCopies * (m_bits / 32) ? m_bits / 32 + n_bits / 32 + m_bits / 32
                                                                                  : kSigCopies * (m_bits / 32);
}
__host__ __device__ constexpr uint32_t sigma_wave_words(uint32_t m_bits, uint32_t n_bits, uint32_t x_col_wt) {
    return ((sigma_img_words(m_bits, n_bits) + (x_col_wt + 1) / 2 + kNoiseWords + 3) & ~3u) + kMidBatch * 2 * 8;
}

// Fast column expansion (default Params: m_bits 8192, n_bits 16384, x_col_wt <= 128, full
// columns). Wave WV's sigma image sits at a compile-time LDS address, and rows_fast encodes a row
// r as (r & 31) | (r >> 5) << 7, so a flip is one bit-field extract (or shift) for the byte
// offset, folded into the ds_xor's immediate base, and one shift for the bit: two VALU per flip.
// (The fallback when rows_delta is unavailable; bank-sorted row orders with bank-matched column
// assignment, lane-rotated chunk orders and deeper load batches were measured and rejected.)
constexpr uint32_t kFastWaveWords = sigma_wave_words(8192, 16384, 128);
// LDS atomic XOR at an absolute LDS byte address (the dynamic LDS of k_sigma starts at 0: it has
// no static __shared__ data; the kernel checks this before taking the fast path)
using lds_u32 = __attribute__((address_space(3))) uint32_t;
__device__ __forceinline__ void lds_xor(uint32_t byte_addr, uint32_t v) {
    __hip_atomic_fetch_xor((lds_u32*)(size_t)byte_addr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <int WV>
__device__ __forceinline__ void flip_cols_fast(const uint16_t* rows_fast, uint32_t W, uint32_t c0, uint32_t c1,
                                               uint32_t ncols, int lane) {
    constexpr uint32_t img = WV * kFastWaveWords * 4u;   // byte address of wave WV's image
    const uint32_t nch = W / 8u;   // 16-byte chunks (8 rows) per column
    auto flip2 = [&](uint32_t x) {   // rows x & 0xFFFF and x >> 16
        lds_xor(img + __builtin_amdgcn_ubfe(x, 5, 10), 1u << (x & 31u));
        lds_xor(img + (x >> 21), 1u << ((x >> 16) & 31u));
    };
#pragma unroll 1
    for (uint32_t cc = 0; cc < 2; ++cc) {
        if ((uint32_t)lane + 64u * cc >= ncols) break;
        const uint4* rp = (const uint4*)(rows_fast + (size_t)(cc ? c1 : c0) * W);
        constexpr uint32_t kB = 8;
        for (uint32_t q8 = 0; q8 < nch; q8 += kB) {
            uint4 v[kB];
#pragma unroll
            for (uint32_t b = 0; b < kB; ++b) {
                v[b] = q8 + b < nch ? rp[q8 + b] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (uint32_t b = 0; b < kB; ++b) {
                if (q8 + b >= nch) break;
                flip2(v[b].x); flip2(v[b].y); flip2(v[b].z); flip2(v[b].w);
            }
        }
    }
}

// Byte-delta column expansion (default Params): a row r is the key R = (r >> 5) | (r & 31) << 8,
// i.e. its image word in byte 0 and its bit in byte 1. A column is its 192 keys in ascending order
// as kDeltaBytes byte increments (R starts at 0; each byte advances R and flips R). A gap of 256 or
// more is bridged by an increment of 255 followed by one of 0 (the same bit flipped twice), and the
// column is padded with 0 increments (an even number: the last bit flipped twice more). Per flip:
// one byte-select add, one byte-select shift for the LDS address, one for the bit. The table is
// 3.4 MB (16384 x 208 B) against 6.3 MB of u16 rows, so it mostly stays in each XCD's 4 MB L2:
// the u16 expansion was bound by these gathers (about 26 of 42 ms), not by the flips.
constexpr uint32_t kDeltaBytes = 208;   // 13 chunks of 16 increments; <= 8 bridges per column
template <int WV>
__device__ __forceinline__ void flip_cols_delta(const uint8_t* tab, uint32_t c0, uint32_t c1) {
    constexpr uint32_t img = WV * kFastWaveWords * 4u;   // byte address of wave WV's image
    uint32_t two = kSigCopies == 8 ? 5u : 4u, one = 1u;   // word W of copy k at byte 4 (copies W + k)
    const uint32_t kofs = (threadIdx.x & (kSigCopies - 1u)) << 2;
    asm volatile("" : "+v"(two), "+v"(one));   // VGPR operands for the SDWA shifts
    auto word4 = [&](uint32_t& R, uint32_t w) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            R += (w >> (8 * k)) & 255u;
            // byte 0 of R << 2 (the word's LDS offset) and 1 << byte 1 of R, one SDWA shift each
            uint32_t off, bit;
            asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
                : "=v"(off) : "v"(two), "v"(R));
            asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
                : "=v"(bit) : "v"(R), "v"(one));
            off |= kofs;
            __builtin_assume(off < 1024u * kSigCopies);
            lds_xor(img + off, bit);
        }
    };
#pragma unroll 1
    for (uint32_t cc = 0; cc < 2; ++cc) {
        const uint4* rp = (const uint4*)(tab + (size_t)(cc ? c1 : c0) * kDeltaBytes);
        uint32_t R = 0;
        {
            uint4 v[8];
#ifdef PVAC_EXP_SIG_DNOLOAD   // timing experiment: synthetic increments, no table reads (sigma wrong)
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const uint32_t h = ((cc ? c1 : c0) * 0x9E3779B1u + b * 0x85EBCA77u);
                v[b] = make_uint4(h & 0x3F3F3F3Fu, (h * 0xC2B2AE3Du) & 0x3F3F3F3Fu, (h * 0x27D4EB2Fu) & 0x3F3F3F3Fu,
                                  (h * 0x165667B1u) & 0x3F3F3F3Fu);
            }
#else
#pragma unroll
            for (int b = 0; b < 8; ++b) v[b] = rp[b];
#endif
#pragma unroll
            for (int b = 0; b < 8; ++b) { word4(R, v[b].x); word4(R, v[b].y); word4(R, v[b].z); word4(R, v[b].w); }
        }
        {
            uint4 v[5];
#ifdef PVAC_EXP_SIG_DNOLOAD
#pragma unroll
            for (int b = 0; b < 5; ++b) {
                const uint32_t h = ((cc ? c1 : c0) * 0x9E3779B1u + (b + 8) * 0x85EBCA77u);
                v[b] = make_uint4(h & 0x3F3F3F3Fu, (h * 0xC2B2AE3Du) & 0x3F3F3F3Fu, (h * 0x27D4EB2Fu) & 0x3F3F3F3Fu,
                                  (h * 0x165667B1u) & 0x3F3F3F3Fu);
            }
#else
#pragma unroll
            for (int b = 0; b < 5; ++b) v[b] = rp[8 + b];
#endif
#pragma unroll
            for (int b = 0; b < 5; ++b) { word4(R, v[b].x); word4(R, v[b].y); word4(R, v[b].z); word4(R, v[b].w); }
        }
    }
}

// POW2: n_bits and m_bits are powers of two (default Params), so the rejection bound is
// 2^64 - N and x mod N is a mask instead of a 64-bit software division per draw
template <bool POW2>
__global__ __launch_bounds__(kSigBlock, kSigMinBlocks) void k_sigma(sig_args a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t slds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t sw32 = a.m_bits / 32, bx32 = a.n_bits / 32, bn32 = a.m_bits / 32;
    const uint32_t imgw = sigma_img_words(a.m_bits, a.n_bits);
    const uint32_t per_wave = imgw + (a.x_col_wt + 1) / 2 + kNoiseWords;
    uint32_t* sig = slds + (size_t)wave * sigma_wave_words(a.m_bits, a.n_bits, a.x_col_wt);
    uint32_t* bmX = sig + sw32;
    uint32_t* bmN = bmX + bx32;
    uint16_t* cols = (uint16_t*)(sig + imgw);
    uint32_t* mids = sig + ((per_wave + 3) & ~3u);   // [edge j][stream][8]
    for (uint32_t w = lane; w < imgw; w += 64) sig[w] = 0;

    const bool isX = lane < 32;
    const uint32_t Nmod = isX ? a.n_bits : a.m_bits;
    const uint32_t K = isX ? a.x_col_wt : a.err_wt;
    const uint64_t lim = ~0ULL - (~0ULL % (uint64_t)Nmod);
    uint32_t* bm = isX ? bmX : bmN;
    const uint64_t words_per_sigma = a.X.sigma_words;
    const uint32_t sub = blockIdx.y * 4 + wave, nsub = a.sub_blocks * 4;
    const bool lds_at0 = (uint32_t)(size_t)(lds_u32*)slds == 0u;   // flip_cols_fast's absolute addresses
    const bool icopy = a.rows_delta && lds_at0;
    uint16_t* nrows = cols + a.x_col_wt;   // kNoiseWords: err_wt <= 128 rows (host-checked)

    // the salt-independent words of an edge (salt last: it is the only word in both blocks)
    auto edge_words = [&](uint64_t eo, uint64_t lo, uint64_t nl, uint64_t e, uint64_t (&words)[7]) {
        const uint64_t m = a.X.meta[e];
        const uint32_t lid = meta_layer(m);
        pvac_layer L{};
        if (lid < nl) L = a.X.layers[lo + lid];
        const uint64_t salt = a.salt_pos ? a.salts[eo + a.salt_pos[e]] : a.salts[e];
        words[0] = a.canon; words[1] = L.ztag; words[2] = L.nonce_lo; words[3] = L.nonce_hi;
        words[4] = (uint64_t)meta_idx(m); words[5] = (uint64_t)meta_ch(m); words[6] = salt;
    };
    for (uint64_t ci = blockIdx.x; ci < a.X.n; ci += gridDim.x) {
        const uint64_t eo = a.X.e_off[ci], ne = a.X.e_cnt[ci], lo = a.X.l_off[ci], nl = a.X.l_cnt[ci];
        for (uint64_t kb = sub; kb < ne; kb += (uint64_t)kMidBatch * nsub) {
          // block-0 midstates of the wave's next kMidBatch edges: lane j computes edge j's X-stream
          // midstate, lane 32 + j its noise-stream midstate (block 0 holds the label, the first six
          // words and the salt's low byte(s); it does not depend on the counter)
          // The same lane then draws counter 32 of its edge and stream (the first block of pass 1):
          // pass 0's 128 draws hold K = 128 distinct values only when there is no repeat, so most
          // edges need a few more draws, and these four (kept in registers, read by the edge's
          // turn with readlane) usually suffice instead of a whole second pass.
          uint32_t pre[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
          {
            const uint64_t kk = kb + (uint64_t)(lane & 31) * nsub;
            if (kk < ne && (uint32_t)(lane & 31) < kMidBatch) {
                uint64_t words[7];
                edge_words(eo, lo, nl, eo + kk, words);
                uint32_t b0[16], b1[16];
                if (isX) { build_block<15, 7>(b0, 0, kLabX, words, 0); build_block<15, 7>(b1, 1, kLabX, words, 32); }
                else { build_block<14, 7>(b0, 0, kLabN, words, 0); build_block<14, 7>(b1, 1, kLabN, words, 32); }
                sha_state ms;
                sha_init(ms);
                sha_compress(ms, b0);
                uint32_t* dst = mids + ((lane & 31) * 2 + (isX ? 0 : 1)) * 8;
#pragma unroll
                for (int i = 0; i < 8; ++i) dst[i] = ms.h[i];
                sha_compress(ms, b1);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint64_t x = (uint64_t)bswap32(ms.h[2 * q]) | ((uint64_t)bswap32(ms.h[2 * q + 1]) << 32);
                    pre[q] = x <= lim ? (uint32_t)(POW2 ? (x & (uint64_t)(Nmod - 1u)) : x % Nmod) : 0xFFFFFFFFu;
                }
            }
            __builtin_amdgcn_wave_barrier();
          }
          for (uint32_t jb = 0; jb < kMidBatch; ++jb) {
            const uint64_t k = kb + (uint64_t)jb * nsub;
            if (k >= ne) break;
            const uint64_t e = eo + k;
            uint64_t words[7];
            edge_words(eo, lo, nl, e, words);
            uint32_t tm[16];
            sha_state mid;
            {
                const uint32_t* src = mids + (jb * 2 + (isX ? 0 : 1)) * 8;
#pragma unroll
                for (int i = 0; i < 8; ++i) mid.h[i] = src[i];
                // block 1 template (counter 0); each pass ORs its counter in below
                uint32_t bx[16], bn[16];
                build_block<15, 7>(bx, 1, kLabX, words, 0);
                build_block<14, 7>(bn, 1, kLabN, words, 0);
#pragma unroll
                for (int i = 0; i < 16; ++i) tm[i] = isX ? bx[i] : bn[i];
            }
            // the le64 counter sits at block-1 byte offset 7 (X: 15-byte label) or 6 (noise: 14):
            // as a big-endian 96-bit window over words 1..3 that is bswap64(ctr) << 8 or << 16
            const uint32_t csh = isX ? 8u : 16u;
            uint32_t have = 0;
            // step 0: pass 0; step 1: counter 32 alone (precomputed above, lanes 0 and 32); step
            // s >= 2: pass s - 1, whose counter-32 block was consumed by step 1 (draw order kept)
            const uint32_t jl = (uint32_t)jb;
            __builtin_amdgcn_s_setprio(1);   // selection (SHA-256 + bitmap) above the next edge's midstates
            for (uint32_t step = 0; step < kMaxPasses; ++step) {   // bounded: never hang the GPU
                uint32_t val[4];
                if (step == 1) {   // wave-uniform
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t vx = __builtin_amdgcn_readlane(pre[q], jl);
                        const uint32_t vn = __builtin_amdgcn_readlane(pre[q], 32 + jl);
                        val[q] = (have < K && (lane & 31) == 0) ? (isX ? vx : vn) : 0xFFFFFFFFu;
                    }
                } else {
                const uint32_t pass = step == 0 ? 0u : step - 1u;
                const uint64_t ctr = (uint64_t)pass * 32 + (lane & 31);
                const uint64_t bs = ((uint64_t)bswap32((uint32_t)ctr) << 32) | bswap32((uint32_t)(ctr >> 32));
                uint32_t blk[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) blk[i] = tm[i];
                blk[1] |= (uint32_t)(bs >> (64u - csh));
                blk[2] |= (uint32_t)((bs << csh) >> 32);
                blk[3] |= (uint32_t)(bs << csh);
                sha_state s = mid;
                sha_compress(s, blk);
                const bool used = pass == 1 && (lane & 31) == 0;   // counter 32: taken in step 1
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint64_t x = (uint64_t)bswap32(s.h[2 * q]) | ((uint64_t)bswap32(s.h[2 * q + 1]) << 32);
                    val[q] = (have < K && x <= lim && !used) ? (uint32_t)(POW2 ? (x & (uint64_t)(Nmod - 1u)) : x % Nmod)
                                                             : 0xFFFFFFFFu;
                }
                }
                int rank[4];
                select_pass2x32(val, bm, K, have, rank);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (rank[q] >= 0) {
                        if (isX) cols[rank[q]] = (uint16_t)val[q];
                        else if (icopy) nrows[rank[q]] = (uint16_t)val[q];   // flipped with the columns
                        else atomicXor(&sig[val[q] >> 5], 1u << (val[q] & 31));   // noise bit
                    }
                }
                const bool doneX = __shfl(have, 0, 64) >= a.x_col_wt;
                const bool doneN = __shfl(have, 32, 64) >= a.err_wt;
                if (doneX && doneN) break;
            }
            // XOR the selected H columns: every lane takes whole columns and reads their row lists
            // with 16-byte loads (width is a multiple of 8), flipping bits with LDS atomic XOR. The
            // selection bitmaps are dead now and sit right after the sigma image, so each 16-lane
            // group flips into its own copy of the image (group g: words sig[256 g + (w + 16 g) mod
            // 256]; the skew puts the groups' equal word indices on different banks): lanes of
            // different groups never contend for a word. Copy 0 already holds the noise bits.
            const uint32_t W = a.width;
            if (a.rows_delta && lds_at0) {   // host-checked: default Params, kFastWaveWords per wave
#if defined(PVAC_EXP_SIG_PRIO0)
                __builtin_amdgcn_s_setprio(0);
#elif defined(PVAC_EXP_SIG_PRIO1)
                __builtin_amdgcn_s_setprio(1);
#elif defined(PVAC_EXP_SIG_PRIO3)
                __builtin_amdgcn_s_setprio(3);
#else
                __builtin_amdgcn_s_setprio(2);   // LDS-atomic phase ahead of other waves' SHA-256
#endif
                const uint32_t c0 = cols[lane], c1 = cols[lane + 64];   // x_col_wt == 128
                for (uint32_t w4 = lane; w4 < (bx32 + bn32) / 4u; w4 += 64) ((uint4*)bmX)[w4] = make_uint4(0, 0, 0, 0);
#ifdef PVAC_EXP_SIG_NOEXP   // timing experiment: no column expansion (sigma wrong)
                if (a.width == 0x7FFFFFFFu)
#endif
                switch (__builtin_amdgcn_readfirstlane(wave)) {
                    case 0: flip_cols_delta<0>(a.rows_delta, c0, c1); break;
                    case 1: flip_cols_delta<1>(a.rows_delta, c0, c1); break;
                    case 2: flip_cols_delta<2>(a.rows_delta, c0, c1); break;
                    default: flip_cols_delta<3>(a.rows_delta, c0, c1); break;
                }
                {   // the noise rows, into the lane's copy like the columns
                    const uint32_t kofs = ((uint32_t)lane & (kSigCopies - 1u)) << 2;
                    for (uint32_t q = (uint32_t)lane; q < a.err_wt; q += 64) {
                        const uint32_t r = nrows[q];
                        atomicXor((uint32_t*)((uint8_t*)sig + (((r >> 5) << (kSigCopies == 8 ? 5 : 4)) | kofs)),
                                  1u << (r & 31u));
                    }
                }
                __builtin_amdgcn_wave_barrier();
                uint64_t* out = a.X.sigma + e * words_per_sigma;
                {
                    // output words 4 lane .. 4 lane + 3: each the XOR of its four copies (one b128 read)
                    constexpr int kQ = (int)kSigCopies;   // b128 reads per lane (4 words x copies / 4)
                    uint4* s4 = (uint4*)sig + kQ * lane;
                    uint32_t o[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        uint32_t x = 0;
#pragma unroll
                        for (int h = 0; h < kQ / 4; ++h) {
                            const uint4 v = s4[q * (kQ / 4) + h];
                            x ^= v.x ^ v.y ^ v.z ^ v.w;
                        }
                        o[q] = x;
                    }
                    ((ulonglong2*)out)[lane] = make_ulonglong2((uint64_t)o[0] | ((uint64_t)o[1] << 32),
                                                               (uint64_t)o[2] | ((uint64_t)o[3] << 32));
#pragma unroll
                    for (int q = 0; q < kQ; ++q) s4[q] = make_uint4(0, 0, 0, 0);
                }
                __builtin_amdgcn_s_setprio(0);
                continue;
            }
            if (a.rows_fast && lds_at0) {   // host-checked: default Params, full columns, kFastWaveWords per wave
                __builtin_amdgcn_s_setprio(2);   // LDS-atomic phase ahead of other waves' SHA-256
                const uint32_t c0 = (uint32_t)lane < a.x_col_wt ? cols[lane] : 0u;
                const uint32_t c1 = (uint32_t)lane + 64u < a.x_col_wt ? cols[lane + 64] : 0u;
                for (uint32_t w4 = lane; w4 < (bx32 + bn32) / 4u; w4 += 64) ((uint4*)bmX)[w4] = make_uint4(0, 0, 0, 0);
#ifdef PVAC_EXP_SIG_NOEXP   // timing experiment: no column expansion (sigma wrong)
                if (a.width == 0x7FFFFFFFu)
#endif
                switch (__builtin_amdgcn_readfirstlane(wave)) {
                    case 0: flip_cols_fast<0>(a.rows_fast, W, c0, c1, a.x_col_wt, lane); break;
                    case 1: flip_cols_fast<1>(a.rows_fast, W, c0, c1, a.x_col_wt, lane); break;
                    case 2: flip_cols_fast<2>(a.rows_fast, W, c0, c1, a.x_col_wt, lane); break;
                    default: flip_cols_fast<3>(a.rows_fast, W, c0, c1, a.x_col_wt, lane); break;
                }
                __builtin_amdgcn_wave_barrier();
                uint64_t* out = a.X.sigma + e * words_per_sigma;
                {
                    uint4* s4 = (uint4*)sig + lane;   // 256 words: one 16-byte store per lane
                    const uint4 v = *s4;
                    ((ulonglong2*)out)[lane] = make_ulonglong2((uint64_t)v.x | ((uint64_t)v.y << 32),
                                                               (uint64_t)v.z | ((uint64_t)v.w << 32));
                    *s4 = make_uint4(0, 0, 0, 0);
                }
                __builtin_amdgcn_s_setprio(0);
                continue;
            }
            const bool split = sw32 == 256u && bx32 + bn32 >= 768u;   // default Params: 4 copies fit
            // Full row lists (every column exactly W rows, as gen_H makes them): no per-row guard,
            // the copies sit 272 words apart (bank offset 16 g without a modular wrap), and a flip
            // is one bit-field extract, one address add and one shift from the packed row pair.
            // Copy 3 reaches into the column list, so both column ids are read first.
            const bool fast = split && a.full && a.x_col_wt <= 128u && per_wave >= 1072u;
            if (fast) {
                __builtin_amdgcn_s_setprio(2);   // LDS-atomic phase ahead of other waves' SHA-256
                const uint32_t c0 = (uint32_t)lane < a.x_col_wt ? cols[lane] : 0u;
                const uint32_t c1 = (uint32_t)lane + 64u < a.x_col_wt ? cols[lane + 64] : 0u;
                __builtin_amdgcn_wave_barrier();
                for (uint32_t w4 = lane; w4 < (1072u - 256u) / 4u; w4 += 64) ((uint4*)(sig + 256))[w4] = make_uint4(0, 0, 0, 0);
                __builtin_amdgcn_wave_barrier();
                uint32_t* img = sig + 272u * ((uint32_t)lane >> 4);
                auto flip2 = [&](uint32_t x) {   // rows x & 0xFFFF and x >> 16
                    atomicXor(&img[__builtin_amdgcn_ubfe(x, 5, 11)], 1u << (x & 31u));
                    atomicXor(&img[__builtin_amdgcn_ubfe(x, 21, 11)], 1u << __builtin_amdgcn_ubfe(x, 16, 5));
                };
#pragma unroll 1
                for (uint32_t cc = 0; cc < 2; ++cc) {
                    if ((uint32_t)lane + 64u * cc >= a.x_col_wt) break;
                    const uint4* rp = (const uint4*)(a.rows + (size_t)(cc ? c1 : c0) * W);
                    constexpr uint32_t kB = 8;
                    for (uint32_t q8 = 0; q8 < W / 8u; q8 += kB) {
                        uint4 v[kB];
#pragma unroll
                        for (uint32_t b = 0; b < kB; ++b) v[b] = q8 + b < W / 8u ? rp[q8 + b] : make_uint4(0, 0, 0, 0);
#pragma unroll
                        for (uint32_t b = 0; b < kB; ++b) {
                            if (q8 + b >= W / 8u) break;
                            flip2(v[b].x); flip2(v[b].y); flip2(v[b].z); flip2(v[b].w);
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
                uint64_t* out = a.X.sigma + e * words_per_sigma;
                for (uint32_t w4 = lane; w4 < 64u; w4 += 64) {
                    uint4 v = *(const uint4*)(sig + w4 * 4);
#pragma unroll
                    for (uint32_t g = 1; g < 4; ++g) {
                        const uint4 u = *(const uint4*)(sig + 272u * g + w4 * 4);
                        v.x ^= u.x; v.y ^= u.y; v.z ^= u.z; v.w ^= u.w;
                    }
                    ((ulonglong2*)out)[w4] = make_ulonglong2((uint64_t)v.x | ((uint64_t)v.y << 32),
                                                             (uint64_t)v.z | ((uint64_t)v.w << 32));
                }
                for (uint32_t w = lane; w < 1072u; w += 64) sig[w] = 0;
                __builtin_amdgcn_s_setprio(0);
                continue;
            }
            if (split) {
                for (uint32_t w4 = lane; w4 < 192u; w4 += 64) ((uint4*)(sig + 256))[w4] = make_uint4(0, 0, 0, 0);
                __builtin_amdgcn_wave_barrier();
            }
            const uint32_t grp = split ? (uint32_t)lane >> 4 : 0u;
            uint32_t* img = sig + 256u * grp;
            const uint32_t skew = 16u * grp;
#ifdef PVAC_EXP_SIG_NOXOR
            if (a.width == 0x7FFFFFFFu)   // timing experiment: no column expansion at all
#endif
            for (uint32_t c = lane; c < a.x_col_wt; c += 64) {
                const uint32_t col = cols[c];
                const uint32_t cnt = a.counts[col];
                const uint4* rp = (const uint4*)(a.rows + (size_t)col * W);
                // eight 16-byte row loads in flight per lane, then their 64 flips: the row lists live
                // in L2/MALL, so one load at a time would expose ~24 load latencies per column
                constexpr uint32_t kB = 8;
                for (uint32_t k8 = 0; k8 < cnt; k8 += 8 * kB) {
                    uint4 v[kB];
#pragma unroll
                    for (uint32_t b = 0; b < kB; ++b)
                        v[b] = k8 + 8 * b < cnt ? rp[(k8 >> 3) + b] : make_uint4(0, 0, 0, 0);
#pragma unroll
                    for (uint32_t b = 0; b < kB; ++b) {
                        const uint32_t kb = k8 + 8 * b;
                        const uint32_t rr[8] = {v[b].x & 0xFFFFu, v[b].x >> 16, v[b].y & 0xFFFFu, v[b].y >> 16,
                                                v[b].z & 0xFFFFu, v[b].z >> 16, v[b].w & 0xFFFFu, v[b].w >> 16};
#ifdef PVAC_EXP_SIG_NOLDSXOR
                        // timing experiment: rows read, no LDS atomics
                        if ((rr[0] ^ rr[3] ^ rr[7]) == 0xFFFFFFFFu) sig[0] = rr[1];
#else
#pragma unroll
                        for (int j = 0; j < 8; ++j)
                            if (kb + j < cnt)
                                atomicXor(&img[split ? ((rr[j] >> 5) + skew) & 255u : rr[j] >> 5], 1u << (rr[j] & 31));
#endif
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            // write 8192 bits: one 16-byte store per lane (the XOR of the copies), then clear the
            // wave's LDS
            uint64_t* out = a.X.sigma + e * words_per_sigma;
            for (uint32_t w4 = lane; w4 * 4 < sw32; w4 += 64) {
                uint4 v = *(const uint4*)(sig + w4 * 4);
                if (split) {
#pragma unroll
                    for (uint32_t g = 1; g < 4; ++g) {
                        const uint4 u = *(const uint4*)(sig + 256u * g + ((w4 * 4 + 16u * g) & 255u));
                        v.x ^= u.x; v.y ^= u.y; v.z ^= u.z; v.w ^= u.w;
                    }
                }
                ((ulonglong2*)out)[w4] = make_ulonglong2((uint64_t)v.x | ((uint64_t)v.y << 32),
                                                         (uint64_t)v.z | ((uint64_t)v.w << 32));
            }
            for (uint32_t w = lane; w < imgw; w += 64) sig[w] = 0;
          }
        }
    }
}

// gen_H: one wave per column; 64 lanes x 4 draws per pass ("pvac.dom.h_gen", 5 words)
__global__ __launch_bounds__(256) void k_gen_H(uint16_t* rows, uint32_t* counts, uint32_t width, uint32_t m_bits,
                                               uint32_t n_bits, uint32_t wt, uint64_t canon) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hlds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t bw = m_bits / 32;
    uint32_t* bm = hlds + (size_t)wave * bw;
    const uint64_t lim = ~0ULL - (~0ULL % (uint64_t)m_bits);
    for (uint32_t c = blockIdx.x * 4 + wave; c < n_bits; c += gridDim.x * 4) {
        for (uint32_t w = lane; w < bw; w += 64) bm[w] = 0;
        const uint64_t words[5] = {m_bits, n_bits, wt, c, canon};
        uint32_t have = 0;
        for (uint32_t pass = 0; have < wt && pass < kMaxPasses; ++pass) {
            const uint64_t ctr = (uint64_t)pass * 64 + lane;
            uint32_t blk[16];
            sha_state s;
            sha_init(s);
            build_block<14, 5>(blk, 0, kLabH, words, ctr);
            sha_compress(s, blk);
            build_block<14, 5>(blk, 1, kLabH, words, ctr);
            sha_compress(s, blk);
            uint32_t val[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint64_t x = (uint64_t)bswap32(s.h[2 * q]) | ((uint64_t)bswap32(s.h[2 * q + 1]) << 32);
                val[q] = x <= lim ? (uint32_t)(x % m_bits) : 0xFFFFFFFFu;
            }
            int rank[4];
            select_pass<64>(val, bm, wt, have, rank);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (rank[q] >= 0) rows[(size_t)c * width + rank[q]] = (uint16_t)val[q];
        }
        if (lane == 0) counts[c] = wt;
    }
}

// rows_fast from rows (one thread per column): encode (r & 31) | (r >> 5) << 7, draw order kept
__global__ __launch_bounds__(256) void k_encode_fast(const uint16_t* rows, uint16_t* out, uint32_t W, uint32_t n_cols) {
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;
    if (c >= n_cols) return;
    const uint16_t* r = rows + (size_t)c * W;
    uint16_t* o = out + (size_t)c * W;
    for (uint32_t i = 0; i < W; ++i) o[i] = (uint16_t)((r[i] & 31u) | ((r[i] >> 5) << 7));
}

// rows_delta from rows (one thread per column): keys R = (r >> 5) | (r & 31) << 8 in ascending
// order as byte increments with bridges and even 0-padding (see flip_cols_delta); *ovf is set when
// a column needs more than kDeltaBytes increments
__global__ __launch_bounds__(256) void k_encode_delta(const uint16_t* rows, uint8_t* out, uint32_t W, uint32_t n_cols,
                                                      uint32_t* ovf) {
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;
    if (c >= n_cols) return;
    const uint16_t* r = rows + (size_t)c * W;
    uint8_t* o = out + (size_t)c * kDeltaBytes;
    uint32_t k = 0, prev = 0;
    auto put = [&](uint32_t d) {
        if (k < kDeltaBytes) o[k] = (uint8_t)d;
        ++k;
    };
    for (uint32_t b = 0; b < 32; ++b) {   // byte 1 of R: the bit
        uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // image words holding a row with this bit
        for (uint32_t i = 0; i < W; ++i)
            if ((r[i] & 31u) == b) m[r[i] >> 10] |= 1u << ((r[i] >> 5) & 31u);
        for (uint32_t j = 0; j < 8; ++j)
            while (m[j]) {
                const uint32_t R = (j * 32u + (uint32_t)__builtin_ctz(m[j])) | (b << 8);
                m[j] &= m[j] - 1u;
                while (R - prev > 255u) { put(255u); put(0u); prev += 255u; }
                put(R - prev);
                prev = R;
            }
    }
    if (k > kDeltaBytes || (k & 1u)) atomicOr(ovf, 1u);
    while (k < kDeltaBytes) put(0u);
}

}  // namespace

// rows_delta for the default geometry (see flip_cols_delta); synchronous; left null when a column
// does not fit kDeltaBytes (the u16 expansion is used then)
static hipError_t build_delta_rows(sigma_tables& T, const pvac_hip_params& prm, hipStream_t st) {
    if (T.rows_delta) { hipFree(T.rows_delta); T.rows_delta = nullptr; }
    if (!(prm.m_bits == 8192 && prm.x_col_wt == 128 && T.full && T.rows &&
          sigma_wave_words(prm.m_bits, prm.n_bits, prm.x_col_wt) == kFastWaveWords))
        return hipSuccess;
    uint32_t* ovf = nullptr;
    hipError_t e = hipMalloc(&T.rows_delta, (size_t)T.n_cols * kDeltaBytes);
    if (e == hipSuccess) e = hipMalloc(&ovf, 4);
    if (e == hipSuccess) e = hipMemsetAsync(ovf, 0, 4, st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_encode_delta, dim3((T.n_cols + 255) / 256), dim3(256), 0, st, T.rows, T.rows_delta, T.width,
                           T.n_cols, ovf);
        e = hipGetLastError();
    }
    uint32_t h = 1;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, ovf, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    hipFree(ovf);
    if (e != hipSuccess || h) { hipFree(T.rows_delta); T.rows_delta = nullptr; }
    return e;
}

// rows_fast for the default geometry (see flip_cols_fast); other geometries keep rows only
static hipError_t build_fast_rows(sigma_tables& T, const pvac_hip_params& prm, hipStream_t st) {
    if (T.rows_fast) { hipFree(T.rows_fast); T.rows_fast = nullptr; }
    if (!(prm.m_bits == 8192 && prm.x_col_wt == 128 && T.full && T.width % 8 == 0 && T.width >= 8 &&
          sigma_wave_words(prm.m_bits, prm.n_bits, prm.x_col_wt) == kFastWaveWords))
        return hipSuccess;
    hipError_t e = hipMalloc(&T.rows_fast, (size_t)T.n_cols * T.width * 2);
    if (e != hipSuccess) { T.rows_fast = nullptr; return e; }
    hipLaunchKernelGGL(k_encode_fast, dim3((T.n_cols + 255) / 256), dim3(256), 0, st, T.rows, T.rows_fast, T.width,
                       T.n_cols);
    return hipGetLastError();
}

// host SHA-256 over a contiguous buffer
void sha256_host(const uint8_t* p, size_t n, uint8_t out[32]) {
    sha_state s;
    sha_init(s);
    size_t off = 0;
    uint32_t w[16];
    auto load = [&](const uint8_t* b) {
        for (int i = 0; i < 16; ++i)
            w[i] = (uint32_t)b[4 * i] << 24 | (uint32_t)b[4 * i + 1] << 16 | (uint32_t)b[4 * i + 2] << 8 | b[4 * i + 3];
    };
    for (; off + 64 <= n; off += 64) { load(p + off); sha_compress(s, w); }
    uint8_t tail[128] = {0};
    const size_t r = n - off;
    std::memcpy(tail, p + off, r);
    tail[r] = 0x80;
    const size_t tl = (r + 9 <= 64) ? 64 : 128;
    const uint64_t bits = (uint64_t)n * 8;
    for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    for (size_t b = 0; b < tl; b += 64) { load(tail + b); sha_compress(s, w); }
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(s.h[i] >> 24); out[4 * i + 1] = (uint8_t)(s.h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(s.h[i] >> 8); out[4 * i + 3] = (uint8_t)s.h[i];
    }
}


void sigma_tables_free(sigma_tables& T) {
    hipFree(T.rows);
    hipFree(T.counts);
    hipFree(T.rows_fast);
    hipFree(T.rows_delta);
    T = sigma_tables{};
}

// A copy of src's device tables for a context on dst_dev (same or another device: peer copies
// over xGMI); synchronous on st, which must belong to dst_dev.
hipError_t sigma_tables_clone(sigma_tables& dst, const sigma_tables& src, int dst_dev, int src_dev, hipStream_t st) {
    sigma_tables_free(dst);
    if (!src.ready) return hipSuccess;
    const size_t nr = (size_t)src.n_cols * src.width * 2, nc = (size_t)src.n_cols * 4,
                 nd = (size_t)src.n_cols * kDeltaBytes;
    auto one = [&](void** d, const void* s, size_t bytes) -> hipError_t {
        if (!s) return hipSuccess;
        hipError_t e = hipMalloc(d, bytes);
        if (e == hipSuccess) e = hipMemcpyPeerAsync(*d, dst_dev, s, src_dev, bytes, st);
        return e;
    };
    hipError_t e = one((void**)&dst.rows, src.rows, nr);
    if (e == hipSuccess) e = one((void**)&dst.counts, src.counts, nc);
    if (e == hipSuccess) e = one((void**)&dst.rows_fast, src.rows_fast, nr);
    if (e == hipSuccess) e = one((void**)&dst.rows_delta, src.rows_delta, nd);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        sigma_tables_free(dst);
        return e;
    }
    dst.width = src.width;
    dst.n_cols = src.n_cols;
    dst.full = src.full;
    dst.ready = true;
    return hipSuccess;
}

static hipError_t alloc_tables(sigma_tables& T, uint32_t n_cols, uint32_t width) {
    sigma_tables_free(T);
    hipError_t e = hipMalloc(&T.rows, (size_t)n_cols * width * 2);
    if (e == hipSuccess) e = hipMalloc(&T.counts, (size_t)n_cols * 4);
    if (e != hipSuccess) { sigma_tables_free(T); return e; }
    T.width = width;
    T.n_cols = n_cols;
    return hipSuccess;
}

hipError_t sigma_tables_from_dense(sigma_tables& T, const pvac_hip_params& prm, const uint64_t* H, hipStream_t st) {
    const uint32_t wpc = (prm.m_bits + 63) / 64;
    uint32_t width = 0;
    std::vector<uint32_t> cnt(prm.n_bits);
    for (uint32_t c = 0; c < prm.n_bits; ++c) {
        uint32_t k = 0;
        for (uint32_t w = 0; w < wpc; ++w) k += (uint32_t)__builtin_popcountll(H[(size_t)c * wpc + w]);
        cnt[c] = k;
        width = k > width ? k : width;
    }
    width = (width + 7) & ~7u;   // row lists padded to 16-byte multiples (k_sigma reads uint4)
    if (width == 0) width = 8;
    std::vector<uint16_t> rows((size_t)prm.n_bits * width, 0);
    for (uint32_t c = 0; c < prm.n_bits; ++c) {
        uint32_t k = 0;
        for (uint32_t w = 0; w < wpc; ++w) {
            uint64_t x = H[(size_t)c * wpc + w];
            while (x) {
                const int b = __builtin_ctzll(x);
                rows[(size_t)c * width + k++] = (uint16_t)(w * 64 + b);
                x &= x - 1;
            }
        }
    }
    hipError_t e = alloc_tables(T, prm.n_bits, width);
    T.full = std::all_of(cnt.begin(), cnt.end(), [&](uint32_t k) { return k == width; });
    if (e == hipSuccess) e = hipMemcpyAsync(T.rows, rows.data(), rows.size() * 2, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(T.counts, cnt.data(), cnt.size() * 4, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = build_fast_rows(T, prm, st);
    if (e == hipSuccess) e = build_delta_rows(T, prm, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    T.ready = e == hipSuccess;
    return e;
}

hipError_t sigma_tables_generate(sigma_tables& T, const pvac_hip_params& prm, uint8_t digest[32], hipStream_t st) {
    if (prm.h_col_wt == 0 || prm.h_col_wt > prm.m_bits || prm.m_bits % 32 || prm.m_bits > 65536)
        return hipErrorInvalidValue;
    // row lists padded to 16-byte multiples (k_sigma reads uint4); counts bound every reader
    hipError_t e = alloc_tables(T, prm.n_bits, (prm.h_col_wt + 7) & ~7u);
    if (e != hipSuccess) return e;
    T.full = T.width == prm.h_col_wt;   // gen_H draws exactly h_col_wt distinct rows per column
    const size_t lds = (size_t)4 * (prm.m_bits / 32) * 4;
    hipLaunchKernelGGL(k_gen_H, dim3(2048), dim3(256), lds, st, T.rows, T.counts, T.width, prm.m_bits, prm.n_bits,
                       prm.h_col_wt, prm.canon_tag);
    e = hipGetLastError();
    if (e == hipSuccess) e = build_fast_rows(T, prm, st);
    if (e == hipSuccess) e = build_delta_rows(T, prm, st);
    if (e != hipSuccess) return e;
    if (digest) {
        std::vector<uint16_t> rows((size_t)prm.n_bits * T.width);
        e = hipMemcpyAsync(rows.data(), T.rows, rows.size() * 2, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return e;
        // H_digest = SHA-256("H|v2" || le64 m || le64 n || le64 wt || column bytes) (matrix.hpp:218-250)
        const size_t colbytes = (prm.m_bits + 7) / 8;
        std::vector<uint8_t> msg(4 + 24 + (size_t)prm.n_bits * colbytes, 0);
        std::memcpy(msg.data(), "H|v2", 4);
        const uint64_t hdr[3] = {prm.m_bits, prm.n_bits, prm.h_col_wt};
        for (int k = 0; k < 3; ++k)
            for (int i = 0; i < 8; ++i) msg[4 + 8 * k + i] = (uint8_t)(hdr[k] >> (8 * i));
        uint8_t* cols = msg.data() + 28;
        for (uint32_t c = 0; c < prm.n_bits; ++c)
            for (uint32_t k = 0; k < prm.h_col_wt; ++k) {
                const uint32_t r = rows[(size_t)c * T.width + k];
                cols[(size_t)c * colbytes + (r >> 3)] |= (uint8_t)(1u << (r & 7));
            }
        sha256_host(msg.data(), msg.size(), digest);
    } else {
        e = hipStreamSynchronize(st);
    }
    T.ready = e == hipSuccess;
    return e;
}

hipError_t launch_sigma(const sigma_tables& T, const pvac_hip_params& prm, const pvac_ct_batch& X,
                        const uint64_t* salts, const uint32_t* salt_pos, int num_cus, hipStream_t st) {
    if (!X.n) return hipSuccess;
    if (!T.ready || prm.m_bits % 128 || prm.n_bits % 32 || prm.x_col_wt > prm.n_bits || prm.err_wt > prm.m_bits ||
        X.sigma_words != prm.m_bits / 64 || prm.n_bits > 65536)
        return hipErrorInvalidValue;
    sig_args a;
    a.X = X;
    a.salts = salts;
    a.salt_pos = salt_pos;
    a.rows = T.rows;
    // Column expansion: byte-delta tables (default), else u16 rows with per-wave images, else the
    // per-lane-group image copies, else the generic guarded loop. PVAC_SIGMA_PATH = delta | u16 |
    // copies | generic caps the choice (read per launch: A/B runs and the tests of every path).
    int path = 0;
    if (const char* v = std::getenv("PVAC_SIGMA_PATH")) {
        const std::string pv(v);
        path = pv == "u16" ? 1 : pv == "copies" ? 2 : pv == "generic" ? 3 : 0;
    }
#if defined(PVAC_EXP_SIG_OLD)   // A/B builds only (make exp-sig)
    path = 2;
#elif defined(PVAC_EXP_SIG_U16)
    path = 1;
#endif
    const bool fast_ok = prm.m_bits == 8192 && prm.x_col_wt == 128 && T.full &&
                         sigma_wave_words(prm.m_bits, prm.n_bits, prm.x_col_wt) == kFastWaveWords &&
                         (kNoiseWords == 0 || prm.err_wt <= 2 * kNoiseWords);
    a.rows_fast = (fast_ok && path <= 1) ? T.rows_fast : nullptr;
    a.rows_delta = (a.rows_fast && path == 0) ? T.rows_delta : nullptr;
    a.counts = T.counts;
    a.width = T.width;
    a.full = (T.full && path <= 2) ? 1u : 0u;
    a.canon = prm.canon_tag;
    a.n_bits = prm.n_bits;
    a.m_bits = prm.m_bits;
    a.x_col_wt = prm.x_col_wt;
    a.err_wt = prm.err_wt;
    const size_t lds = (size_t)4 * sigma_wave_words(prm.m_bits, prm.n_bits, prm.x_col_wt) * 4;
    uint64_t gx = X.n < 4096 ? X.n : 4096;
    uint64_t sub = 1;
    const uint64_t want = (uint64_t)num_cus * 8;
    if (gx < want) sub = (want + gx - 1) / gx;
    if (sub > 64) sub = 64;
    a.sub_blocks = (uint32_t)sub;
    const bool pow2 = (prm.n_bits & (prm.n_bits - 1)) == 0 && (prm.m_bits & (prm.m_bits - 1)) == 0;
    if (pow2)
        hipLaunchKernelGGL(k_sigma<true>, dim3((unsigned)gx, (unsigned)sub), dim3(kSigBlock), lds, st, a);
    else
        hipLaunchKernelGGL(k_sigma<false>, dim3((unsigned)gx, (unsigned)sub), dim3(kSigBlock), lds, st, a);
    return hipGetLastError();
}

}  // namespace pvhip
