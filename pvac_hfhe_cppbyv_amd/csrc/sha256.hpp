// sha256.hpp — FIPS 180-4 SHA-256 compression for device code (and host, for tables).
// Used for the layer ztag (crypto/matrix.hpp:254-264) and the counter-mode PRG of
// prg_choose_k / gen_H / sigma_from_H (crypto/matrix.hpp:15-92, 191-303). The message
// schedule is kept in a 16-word rolling window in registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pvhip {

#define PVH_HD __host__ __device__ __forceinline__

PVH_HD uint32_t rotr32(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }

// a ^ b ^ c in one VALU instruction on gfx950 (v_bitop3_b32, truth table 0x96); the compiler
// emits two v_xor_b32 for the expression. Host passes keep the plain expression.
PVH_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return a ^ b ^ c;
#endif
}

// majority(a, b, c) in one VALU instruction (v_bitop3_b32, truth table 0xE8); the compiler emits
// three (xor, and, bitop3) for the expression
PVH_HD uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe8" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return (a & b) ^ (a & c) ^ (b & c);
#endif
}

// x + y + k with the round constant k in an SGPR: one v_add3_u32 (gfx950 VOP3 takes no literal, so
// the compiler otherwise spends a VOP2 add on the literal and a second add)
PVH_HD uint32_t add3k(uint32_t x, uint32_t y, uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "s"(k));
    return r;
#else
    return x + y + k;
#endif
}

struct sha_state { uint32_t h[8]; };

PVH_HD void sha_init(sha_state& s) {
    s.h[0] = 0x6a09e667u; s.h[1] = 0xbb67ae85u; s.h[2] = 0x3c6ef372u; s.h[3] = 0xa54ff53au;
    s.h[4] = 0x510e527fu; s.h[5] = 0x9b05688cu; s.h[6] = 0x1f83d9abu; s.h[7] = 0x5be0cd19u;
}

static constexpr uint32_t kSHA_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

// One compression of a 64-byte block given as 16 big-endian words.
PVH_HD void sha_compress(sha_state& s, const uint32_t blk[16]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = blk[i];
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t x15 = w[(i - 15) & 15], x2 = w[(i - 2) & 15];
            const uint32_t s0 = xor3(rotr32(x15, 7), rotr32(x15, 18), x15 >> 3);
            const uint32_t s1 = xor3(rotr32(x2, 17), rotr32(x2, 19), x2 >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
        }
        const uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
        const uint32_t ch = (e & f) ^ (~e & g);
        const uint32_t t1 = add3k(h, wi, kSHA_K[i]) + S1 + ch;
        const uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
        const uint32_t mj = maj3(a, b, c);
        const uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d; s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

PVH_HD uint32_t bswap32(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}

// Builds messages byte-wise into a 64-byte block (big-endian word packing on the fly).
struct sha_writer {
    sha_state st;
    uint32_t blk[16];
    uint32_t used;    // bytes in the current block
    uint64_t total;   // total bytes fed
    PVH_HD void begin() {
        sha_init(st);
#pragma unroll
        for (int i = 0; i < 16; ++i) blk[i] = 0;
        used = 0; total = 0;
    }
    PVH_HD void byte(uint32_t b) {
        blk[used >> 2] |= (b & 0xFFu) << (24 - 8 * (used & 3));
        ++used; ++total;
        if (used == 64) {
            sha_compress(st, blk);
#pragma unroll
            for (int i = 0; i < 16; ++i) blk[i] = 0;
            used = 0;
        }
    }
    PVH_HD void u64le(uint64_t x) {
        for (int i = 0; i < 8; ++i) byte((uint32_t)(x >> (8 * i)));
    }
    PVH_HD void finish() {
        const uint64_t bits = total * 8;
        byte(0x80);
        while (used != 56) byte(0);
        for (int i = 7; i >= 0; --i) byte((uint32_t)(bits >> (8 * i)));
    }
    // first 8 digest bytes read little-endian (load_le64 of the digest)
    PVH_HD uint64_t digest_le64(int word_pair) const {
        const uint32_t a = bswap32(st.h[2 * word_pair]), b = bswap32(st.h[2 * word_pair + 1]);
        return (uint64_t)a | ((uint64_t)b << 32);
    }
};

// ztag = load_le64(SHA-256("pvac.dom.ztag" || le64 canon || le64 nonce.lo || le64 nonce.hi))
// (crypto/matrix.hpp:254-264). 37-byte message: one compression, built directly as words.
PVH_HD uint64_t layer_ztag(uint64_t canon, uint64_t nlo, uint64_t nhi) {
    uint8_t m[64];
    const char* lab = "pvac.dom.ztag";
    for (int i = 0; i < 13; ++i) m[i] = (uint8_t)lab[i];
    for (int i = 0; i < 8; ++i) {
        m[13 + i] = (uint8_t)(canon >> (8 * i));
        m[21 + i] = (uint8_t)(nlo >> (8 * i));
        m[29 + i] = (uint8_t)(nhi >> (8 * i));
    }
    m[37] = 0x80;
    for (int i = 38; i < 56; ++i) m[i] = 0;
    const uint64_t bits = 37 * 8;
    for (int i = 0; i < 8; ++i) m[56 + i] = (uint8_t)(bits >> (56 - 8 * i));
    uint32_t blk[16];
    for (int i = 0; i < 16; ++i)
        blk[i] = (uint32_t)m[4 * i] << 24 | (uint32_t)m[4 * i + 1] << 16 | (uint32_t)m[4 * i + 2] << 8 | m[4 * i + 3];
    sha_state s;
    sha_init(s);
    sha_compress(s, blk);
    return (uint64_t)bswap32(s.h[0]) | ((uint64_t)bswap32(s.h[1]) << 32);
}

}  // namespace pvhip
