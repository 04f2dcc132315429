// fp127.hpp — Fp over p = 2^127 - 1 on CDNA4 (gfx950), bit-exact with the reference
// include/pvac/core/field.hpp (the product's own implementation).
//
// Layout: an element is two u64 limbs (lo, hi). gfx950 has no 64x64->128 multiply; the
// 64x64 partial products lower to v_mad_u64_u32 chains (4 per partial product). All
// branches of the reference (fp_from_words' conditional subtract) become selects so a
// wavefront never diverges on data.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pvhip {

struct fp { uint64_t lo, hi; };

constexpr uint64_t kM63 = 0x7FFFFFFFFFFFFFFFULL;
constexpr uint64_t kAll = ~0ULL;

// 64x64 -> 128 as four v_mad_u64_u32 (32x32 + 64 -> 64). `a*b` plus `__umul64hi(a, b)` would
// compute the partial products twice (~9 multiplies); here each partial product is formed once
// and carried through the accumulate operand. No step overflows: (2^32-1)^2 + 2(2^32-1) = 2^64-1.
__device__ __forceinline__ void mul_64x64(uint64_t a, uint64_t b, uint64_t& lo, uint64_t& hi) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
    const uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t p0 = (uint64_t)a0 * b0;
    const uint64_t p1 = (uint64_t)a0 * b1 + (p0 >> 32);
    const uint64_t p2 = (uint64_t)a1 * b0 + (uint32_t)p1;
    hi = (uint64_t)a1 * b1 + (p1 >> 32) + (p2 >> 32);
    lo = (p2 << 32) | (uint32_t)p0;
}

// add with carry-out
__device__ __forceinline__ uint64_t add_co(uint64_t a, uint64_t b, uint64_t& carry) {
    uint64_t s = a + b;
    carry = s < a;
    return s;
}

// field.hpp:26-48. Canonical for every 128-bit input.
__device__ __forceinline__ fp fp_from_words(uint64_t lo, uint64_t hi) {
    const uint64_t top = hi >> 63;
    hi &= kM63;
    uint64_t c;
    lo = add_co(lo, top, c);
    hi += c;
    const bool reduce = (hi >> 63) | ((hi == kM63) & (lo == kAll));
    const uint64_t borrow = lo != kAll;          // (old_lo < UINT64_MAX)
    const uint64_t rlo = lo + 1;                 // lo - (2^64 - 1)
    const uint64_t rhi = hi - kM63 - borrow;
    return fp{reduce ? rlo : lo, reduce ? rhi : hi};
}

// field.hpp:50-56 — the high sum is truncated to 64 bits before the fold (reference quirk
// for non-canonical inputs, reproduced exactly).
__device__ __forceinline__ fp fp_add(const fp& a, const fp& b) {
    uint64_t c;
    const uint64_t lo = add_co(a.lo, b.lo, c);
    return fp_from_words(lo, a.hi + b.hi + c);
}

// field.hpp:58-67: (2^64-1) - lo never borrows, so neg = fold(~lo, M63 - hi).
__device__ __forceinline__ fp fp_neg(const fp& a) { return fp_from_words(kAll - a.lo, kM63 - a.hi); }

__device__ __forceinline__ fp fp_sub(const fp& a, const fp& b) { return fp_add(a, fp_neg(b)); }

__device__ __forceinline__ bool fp_nonzero(const fp& a) { return (a.lo | a.hi) != 0; }

// ---- lazy products for sums ------------------------------------------------------------
// For CANONICAL a, b (< 2^127) the first Mersenne fold of the 254-bit product already gives a
// 128-bit x with x == a*b (mod p): z < 2^254, so (z mod 2^127) + (z >> 127) < 2^128. Sums of
// such x are reduced once (fp_fold3_lazy), which skips the second fold and fp_from_words per
// product. Equal mod p to the reference's fp_add chain of fp_mul results (field.hpp:50-56,
// 209-213), which computes the exact sum mod p for canonical addends.
//
// These helpers work on 32-bit words: products are v_mad_u64_u32 chains and every multi-word
// sum is a v_add_co_u32 / v_addc_co_u32 carry chain (__builtin_addc), instead of 64-bit adds
// with compare-and-select carries.
__device__ __forceinline__ uint32_t lo32(uint64_t x) { return (uint32_t)x; }
__device__ __forceinline__ uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
__device__ __forceinline__ uint64_t join32(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
// (hi:lo) >> sh for 0 < sh < 32 (v_alignbit_b32)
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
    return __builtin_amdgcn_alignbit(hi, lo, sh);
}
__device__ __forceinline__ uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t& cout) {
    unsigned co;
    const uint32_t r = __builtin_addc(a, b, cin, &co);
    cout = co;
    return r;
}

__device__ __forceinline__ void fp_mul_fold1(const fp& a, const fp& b, uint64_t& x0, uint64_t& x1) {
    const uint32_t A[4] = {lo32(a.lo), hi32(a.lo), lo32(a.hi), hi32(a.hi)};
    const uint32_t B[4] = {lo32(b.lo), hi32(b.lo), lo32(b.hi), hi32(b.hi)};
    uint32_t z[8];
    {   // row 0: one mad chain
        uint64_t t = (uint64_t)A[0] * B[0];
        z[0] = lo32(t);
#pragma unroll
        for (int j = 1; j < 4; ++j) {
            t = (uint64_t)A[0] * B[j] + (t >> 32);
            z[j] = lo32(t);
        }
        z[4] = hi32(t);
    }
#pragma unroll
    for (int i = 1; i < 4; ++i) {   // rows 1..3: mad chain into r, then z[i..i+4] += r
        uint32_t r[5];
        uint64_t t = (uint64_t)A[i] * B[0];
        r[0] = lo32(t);
#pragma unroll
        for (int j = 1; j < 4; ++j) {
            t = (uint64_t)A[i] * B[j] + (t >> 32);
            r[j] = lo32(t);
        }
        r[4] = hi32(t);
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) z[i + j] = addc(z[i + j], r[j], c, c);
        z[i + 4] = r[4] + c;   // the partial product fits in i + 5 words: no carry out
    }
    // x = (z mod 2^127) + (z >> 127); z < 2^254 so the high part has < 2^127 and x < 2^128
    uint32_t c = 0;
    const uint32_t w0 = addc(z[0], funnel(z[4], z[3], 31), 0u, c);
    const uint32_t w1 = addc(z[1], funnel(z[5], z[4], 31), c, c);
    const uint32_t w2 = addc(z[2], funnel(z[6], z[5], 31), c, c);
    const uint32_t w3 = (z[3] & 0x7FFFFFFFu) + funnel(z[7], z[6], 31) + c;
    x0 = join32(w0, w1);
    x1 = join32(w2, w3);
}

// 128-bit x -> 43/43/42-bit limbs; up to 2^21 of them sum in u64 limbs without overflow
__device__ __forceinline__ void fp_split3_128(uint64_t x0, uint64_t x1, uint64_t& l0, uint64_t& l1, uint64_t& l2) {
    const uint32_t w0 = lo32(x0), w1 = hi32(x0), w2 = lo32(x1), w3 = hi32(x1);
    l0 = join32(w0, w1 & 0x7FFu);                                 // bits 0..42
    l1 = join32(funnel(w2, w1, 11), (w2 >> 11) & 0x7FFu);        // bits 43..85
    l2 = join32(funnel(w3, w2, 22), w3 >> 22);                    // bits 86..127
}

// (l0 + l1 * 2^43 + l2 * 2^86) mod p, canonical, for limb sums l < 2^64
__device__ __forceinline__ fp fp_fold3_lazy(uint64_t l0, uint64_t l1, uint64_t l2) {
    // V as five words (V < 2^151): l0 + (l1 << 43), then + (l2 << 86)
    uint32_t c = 0;
    const uint32_t v0 = lo32(l0);
    const uint32_t v1 = addc(hi32(l0), lo32(l1) << 11, 0u, c);
    uint32_t v2 = addc(funnel(hi32(l1), lo32(l1), 21), 0u, c, c);
    uint32_t v3 = (hi32(l1) >> 21) + c;
    v2 = addc(v2, lo32(l2) << 22, 0u, c);
    v3 = addc(v3, funnel(hi32(l2), lo32(l2), 10), c, c);
    const uint32_t v4 = (hi32(l2) >> 10) + c;
    // fold bits >= 127 (2^127 == 1): x = (V mod 2^127) + (V >> 127) < 2^127 + 2^24
    const uint32_t top = funnel(v4, v3, 31);
    uint32_t x0 = addc(v0, top, 0u, c);
    uint32_t x1 = addc(v1, 0u, c, c);
    uint32_t x2 = addc(v2, 0u, c, c);
    uint32_t x3 = (v3 & 0x7FFFFFFFu) + c;
    // canonical: x >= 2^127 -> x - p = (x - 2^127) + 1, where x - 2^127 < 2^24 (no carry); x == p -> 0
    const uint32_t t = x3 >> 31;
    x3 &= 0x7FFFFFFFu;
    x0 += t;
    // x == p -> 0, as a mask (no exec branch: folds of several slots interleave)
    const uint32_t keep = ((x3 == 0x7FFFFFFFu) & ((x0 & x1 & x2) == 0xFFFFFFFFu)) ? 0u : ~0u;
    x0 &= keep; x1 &= keep; x2 &= keep; x3 &= keep;
    return fp{join32(x0, x1), join32(x2, x3)};
}

// field.hpp:113-213 (mul128x128 + fp_reduce256 + fp_from_words): the exact 256-bit product
// of ANY two 128-bit inputs, two Mersenne folds, canonical result. The reference's value is the
// unique canonical residue of a*b, so any exact evaluation is bit-identical; this one runs on
// 32-bit words (16 v_mad_u64_u32 + carry chains).
__device__ __forceinline__ fp fp_mul(const fp& a, const fp& b) {
    const uint32_t A[4] = {lo32(a.lo), hi32(a.lo), lo32(a.hi), hi32(a.hi)};
    const uint32_t B[4] = {lo32(b.lo), hi32(b.lo), lo32(b.hi), hi32(b.hi)};
    uint32_t z[8];
    {
        uint64_t t = (uint64_t)A[0] * B[0];
        z[0] = lo32(t);
#pragma unroll
        for (int j = 1; j < 4; ++j) {
            t = (uint64_t)A[0] * B[j] + (t >> 32);
            z[j] = lo32(t);
        }
        z[4] = hi32(t);
    }
#pragma unroll
    for (int i = 1; i < 4; ++i) {
        uint32_t r[5];
        uint64_t t = (uint64_t)A[i] * B[0];
        r[0] = lo32(t);
#pragma unroll
        for (int j = 1; j < 4; ++j) {
            t = (uint64_t)A[i] * B[j] + (t >> 32);
            r[j] = lo32(t);
        }
        r[4] = hi32(t);
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) z[i + j] = addc(z[i + j], r[j], c, c);
        z[i + 4] = r[4] + c;
    }
    // fold 1: x = (z mod 2^127) + (z >> 127) < 2^127 + 2^129 (five words)
    uint32_t c = 0;
    const uint32_t x0 = addc(z[0], funnel(z[4], z[3], 31), 0u, c);
    const uint32_t x1 = addc(z[1], funnel(z[5], z[4], 31), c, c);
    const uint32_t x2 = addc(z[2], funnel(z[6], z[5], 31), c, c);
    const uint32_t x3 = addc(z[3] & 0x7FFFFFFFu, funnel(z[7], z[6], 31), c, c);
    const uint32_t x4 = (z[7] >> 31) + c;
    // fold 2: y = (x mod 2^127) + (x >> 127) < 2^127 + 8
    const uint32_t top = funnel(x4, x3, 31);
    uint32_t y0 = addc(x0, top, 0u, c);
    uint32_t y1 = addc(x1, 0u, c, c);
    uint32_t y2 = addc(x2, 0u, c, c);
    uint32_t y3 = (x3 & 0x7FFFFFFFu) + c;
    // canonical: y >= 2^127 -> (y - 2^127) + 1 (< 9, no carry); y == p -> 0
    const uint32_t t = y3 >> 31;
    y3 &= 0x7FFFFFFFu;
    y0 += t;
    const bool is_p = (y3 == 0x7FFFFFFFu) & ((y0 & y1 & y2) == 0xFFFFFFFFu);
    if (is_p) { y0 = 0; y1 = 0; y2 = 0; y3 = 0; }
    return fp{join32(y0, y1), join32(y2, y3)};
}

// 128-bit x -> 44/44/40-bit limbs. Up to 4096 of them sum without overflow into u64 limbs of
// < 2^56, < 2^56 and < 2^52, so the top 12 bits of the third limb stay free (k_ct_mul_fresh keeps
// the emit cell id there).
__device__ __forceinline__ void fp_split3_44(uint64_t x0, uint64_t x1, uint64_t& l0, uint64_t& l1, uint64_t& l2) {
    const uint32_t w0 = lo32(x0), w1 = hi32(x0), w2 = lo32(x1), w3 = hi32(x1);
    l0 = join32(w0, w1 & 0xFFFu);                                 // bits 0..43
    l1 = join32(funnel(w2, w1, 12), (w2 >> 12) & 0xFFFu);        // bits 44..87
    l2 = join32(funnel(w3, w2, 24), w3 >> 24);                    // bits 88..127
}

// (l0 + l1 * 2^44 + l2 * 2^88) mod p, canonical, for l0, l1 < 2^56 and l2 < 2^52
__device__ __forceinline__ fp fp_fold3_44(uint64_t l0, uint64_t l1, uint64_t l2) {
    // V < 2^141 as five words
    uint32_t c = 0;
    const uint32_t v0 = lo32(l0);
    const uint32_t v1 = addc(hi32(l0), lo32(l1) << 12, 0u, c);
    uint32_t v2 = addc(funnel(hi32(l1), lo32(l1), 20), 0u, c, c);
    uint32_t v3 = (hi32(l1) >> 20) + c;
    v2 = addc(v2, lo32(l2) << 24, 0u, c);
    v3 = addc(v3, funnel(hi32(l2), lo32(l2), 8), c, c);
    const uint32_t v4 = (hi32(l2) >> 8) + c;
    // x = (V mod 2^127) + (V >> 127) < 2^127 + 2^14
    const uint32_t top = funnel(v4, v3, 31);
    uint32_t x0 = addc(v0, top, 0u, c);
    uint32_t x1 = addc(v1, 0u, c, c);
    uint32_t x2 = addc(v2, 0u, c, c);
    uint32_t x3 = (v3 & 0x7FFFFFFFu) + c;
    // x >= 2^127 -> (x - 2^127) + 1 (< 2^14: no carry); x == p -> 0
    const uint32_t t = x3 >> 31;
    x3 &= 0x7FFFFFFFu;
    x0 += t;
    const uint32_t keep = ((x3 == 0x7FFFFFFFu) & ((x0 & x1 & x2) == 0xFFFFFFFFu)) ? 0u : ~0u;
    x0 &= keep; x1 &= keep; x2 &= keep; x3 &= keep;
    return fp{join32(x0, x1), join32(x2, x3)};
}

// ---- lazy register accumulators ---------------------------------------------------------
// Sum of lazy products x < 2^128 (fp_mul_fold1 of canonical operands) as 128 bits + a carry
// count: up to 2^32 addends, 5 VALU ops per add. acc_fold returns the canonical residue, equal to
// the reference's fp_add chain of canonical fp_mul results (exact sum mod p).
struct acc128c { uint32_t w[4]; uint32_t c; };
__device__ __forceinline__ void acc_zero(acc128c& a) { a.w[0] = a.w[1] = a.w[2] = a.w[3] = 0; a.c = 0; }
__device__ __forceinline__ void acc_add(acc128c& a, uint64_t x0, uint64_t x1) {
    uint32_t c;
    a.w[0] = addc(a.w[0], lo32(x0), 0u, c);
    a.w[1] = addc(a.w[1], hi32(x0), c, c);
    a.w[2] = addc(a.w[2], lo32(x1), c, c);
    a.w[3] = addc(a.w[3], hi32(x1), c, c);
    a.c += c;
}
__device__ __forceinline__ fp acc_fold(const acc128c& a) {
    // V = c 2^128 + W, 2^128 == 2 (mod p): x = (W mod 2^127) + (W >> 127) + 2c < 2^127 + 2^34
    uint32_t c;
    const uint32_t add = (a.w[3] >> 31) + 2u * a.c;   // < 2^34 only when c >= 2^31: kept below
    uint32_t x0 = addc(a.w[0], add, 0u, c);
    uint32_t x1 = addc(a.w[1], 0u, c, c);
    uint32_t x2 = addc(a.w[2], 0u, c, c);
    uint32_t x3 = (a.w[3] & 0x7FFFFFFFu) + c;
    // x < 2^127 + 2^32: one conditional subtract of p = (x - 2^127) + 1, then x == p -> 0
    const uint32_t t = x3 >> 31;
    x3 &= 0x7FFFFFFFu;
    x0 = addc(x0, t, 0u, c);
    x1 = addc(x1, 0u, c, c);
    x2 = addc(x2, 0u, c, c);
    x3 += c;
    const bool is_p = (x3 == 0x7FFFFFFFu) & ((x0 & x1 & x2) == 0xFFFFFFFFu);
    if (is_p) { x0 = 0; x1 = 0; x2 = 0; x3 = 0; }
    return fp{join32(x0, x1), join32(x2, x3)};
}

// field.hpp:229-273 fp_inv = a^(p-2) (fp_inv_ct's windowed ladder). The power is unique, so any
// exact chain is bit-identical: a Mersenne addition chain x_k = a^(2^k - 1),
// a^(p-2) = a^(2^127 - 3) = (x_125)^4 * a: 126 squarings + 11 multiplies; fp_inv(0) = 0.
__device__ __forceinline__ fp fp_sqr_n(fp x, int n) {
    for (int i = 0; i < n; ++i) x = fp_mul(x, x);
    return x;
}
__device__ __forceinline__ fp fp_inv(const fp& a) {
    const fp x1 = a;
    const fp x2 = fp_mul(fp_sqr_n(x1, 1), x1);
    const fp x3 = fp_mul(fp_sqr_n(x2, 1), x1);
    const fp x6 = fp_mul(fp_sqr_n(x3, 3), x3);
    const fp x12 = fp_mul(fp_sqr_n(x6, 6), x6);
    const fp x24 = fp_mul(fp_sqr_n(x12, 12), x12);
    const fp x48 = fp_mul(fp_sqr_n(x24, 24), x24);
    const fp x96 = fp_mul(fp_sqr_n(x48, 48), x48);
    const fp x120 = fp_mul(fp_sqr_n(x96, 24), x24);
    const fp x123 = fp_mul(fp_sqr_n(x120, 3), x3);
    const fp x125 = fp_mul(fp_sqr_n(x123, 2), x2);
    return fp_mul(fp_sqr_n(x125, 2), x1);
}

// canonical representative of any 128-bit word pair (fp_from_words, field.hpp:26-48)
__device__ __forceinline__ fp fp_canon(uint64_t lo, uint64_t hi) { return fp_from_words(lo, hi); }

// ---- exact multi-product accumulation for LDS atomics ----------------------------------
// A canonical value v < 2^127 splits into three limbs of 43/42/42 bits. Up to 2^21 such
// values summed limb-wise in u64 accumulators cannot overflow; fold_limbs recombines and
// reduces mod p. The result equals the reference's sequential fp_add chain for canonical
// addends (that chain computes the exact sum mod p).
__device__ __forceinline__ void fp_split3(const fp& v, uint64_t& l0, uint64_t& l1, uint64_t& l2) {
    l0 = v.lo & ((1ULL << 43) - 1);
    l1 = ((v.lo >> 43) | (v.hi << 21)) & ((1ULL << 42) - 1);
    l2 = v.hi >> 21;
}

__device__ __forceinline__ fp fp_fold3(uint64_t l0, uint64_t l1, uint64_t l2) {
    // V = l0 + l1*2^43 + l2*2^85  (< 2^150)
    uint64_t c0, c1, c2;
    const uint64_t w0 = add_co(l0, l1 << 43, c0);
    uint64_t w1 = add_co(l1 >> 21, l2 << 21, c1);
    w1 = add_co(w1, c0, c2);
    const uint64_t w2 = (l2 >> 43) + c1 + c2;
    // V mod p = (V mod 2^127) + (V >> 127)
    const uint64_t top = (w1 >> 63) | (w2 << 1);
    uint64_t d;
    const uint64_t lo = add_co(w0, top, d);
    const uint64_t hi = (w1 & kM63) + d;
    return fp_from_words(lo, hi);
}

// ---- column accumulators over 26-bit limbs ------------------------------------------------
// Sum of many products a*b of canonical operands without a carry chain per product: a and b
// split into five limbs of 26/26/26/26/23 bits (< 2^26), and column k of the running sum is a
// u64 that takes a_i b_j (< 2^52) for every i + j = k, one v_mad_u64_u32 each (25 per product,
// nothing else). Limb 4 is < 2^23, so per product column 3 takes 4 terms < 2^52 and column 4 three
// terms < 2^52 plus two < 2^49: at most 4 * 2^52 = 2^54 per product and column. From a normalised
// start (< 2^26) col26_norm must therefore run within every 1023 products
// (1023 * 2^54 + 2^26 < 2^64; kCol26MaxProducts, checked where the loops size their chunks). col26_fold
// gives the canonical residue of the sum, the same value as the reference's fp_add chain of
// canonical fp_mul results (field.hpp:50-56, 209-213: that chain computes the exact sum mod p).
constexpr uint32_t kM26 = (1u << 26) - 1u;
constexpr uint32_t kCol26MaxProducts = 1023u;   // products per column set between col26_norm calls
__device__ __forceinline__ void fp_split26(const fp& v, uint32_t* l) {   // v canonical (< 2^127)
    l[0] = (uint32_t)v.lo & kM26;
    l[1] = (uint32_t)(v.lo >> 26) & kM26;
    l[2] = (uint32_t)((v.lo >> 52) | (v.hi << 12)) & kM26;
    l[3] = (uint32_t)(v.hi >> 14) & kM26;
    l[4] = (uint32_t)(v.hi >> 40);
}
__device__ __forceinline__ void col26_zero(uint64_t* c) {
#pragma unroll
    for (int k = 0; k < 9; ++k) c[k] = 0;
}
// c += a * b (limb vectors): 25 v_mad_u64_u32
__device__ __forceinline__ void col26_mac(uint64_t* c, const uint32_t* a, const uint32_t* b) {
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) c[i + j] += (uint64_t)a[i] * b[j];
}
// carries up: columns 0..7 < 2^26 afterwards, the value unchanged
__device__ __forceinline__ void col26_norm(uint64_t* c) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        c[k + 1] += c[k] >> 26;
        c[k] &= kM26;
    }
}
// canonical residue of sum_k c_k 2^(26k) for normalised columns (c_8 < 2^64)
__device__ __forceinline__ fp col26_fold(const uint64_t* c) {
    typedef unsigned __int128 u128;
    const u128 m127 = ((u128)1 << 127) - 1;
    // 2^130 == 2^3, 2^156 == 2^29, 2^182 == 2^55, 2^208 == 2^81 (mod p); bits >= 127 of c_4 2^104
    // and c_8 2^81 wrap to bit 0
    const u128 x = (u128)c[0] + ((u128)c[1] << 26) + ((u128)c[2] << 52) + ((u128)c[3] << 78) +
                   ((u128)(c[4] & ((1u << 23) - 1u)) << 104);                               // < 2^127
    const u128 y = ((u128)c[5] << 3) + ((u128)c[6] << 29) + ((u128)c[7] << 55) +
                   ((u128)(c[8] & ((1ull << 46) - 1ull)) << 81);                            // < 2^128
    const u128 t = x + (y & m127);                                                          // < 2^128
    const u128 f = (t & m127) + (t >> 127) + (y >> 127) + (c[4] >> 23) + (c[8] >> 46);      // < 2^127 + 2^19
    return fp_from_words((uint64_t)f, (uint64_t)(f >> 64));
}

}  // namespace pvhip
