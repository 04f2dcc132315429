// aes256.hpp — AES-256 (FIPS-197) for the LPN PRF's counter-mode keystream (reference
// crypto/lpn.hpp:39-148, AesCtr256 over AES-NI).
//
// State and round keys are little-endian column words (byte r of column c in bits 8r..8r+7), so a
// 16-byte block loads as four u32 words. One round is four T-table lookups per column:
//   out_c = T0[b0(w_c)] ^ T1[b1(w_c+1)] ^ T2[b2(w_c+2)] ^ T3[b3(w_c+3)] ^ rk_c
// with T0[x] = (2s, s, s, 3s) bytes (s = S[x]) and T1..T3 its byte rotations; the final round
// takes S-box bytes from T0's byte 1. The key schedule is FIPS-197's Nk = 8 expansion, which is
// what the reference's aeskeygenassist sequence computes. The counter block is the reference's
// _mm_set_epi64x(0, nonce) + i: le64(nonce + i) followed by 8 zero bytes (the low lane wraps
// without carrying into the high lane).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pvhip {

constexpr uint8_t kAesSbox[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76, 0xca, 0x82, 0xc9,
    0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0, 0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f,
    0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15, 0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07,
    0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75, 0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3,
    0x29, 0xe3, 0x2f, 0x84, 0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58,
    0xcf, 0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8, 0x51, 0xa3,
    0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2, 0xcd, 0x0c, 0x13, 0xec, 0x5f,
    0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73, 0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88,
    0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb, 0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac,
    0x62, 0x91, 0x95, 0xe4, 0x79, 0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a,
    0xae, 0x08, 0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a, 0x70,
    0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e, 0xe1, 0xf8, 0x98, 0x11,
    0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf, 0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42,
    0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16};

__host__ __device__ constexpr uint32_t aes_xtime(uint32_t b) { return ((b << 1) ^ ((b & 0x80u) ? 0x1bu : 0u)) & 0xFFu; }
__host__ __device__ constexpr uint32_t aes_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// T0[x] as a little-endian column contribution (rows 0..3 = 2s, s, s, 3s)
__host__ __device__ constexpr uint32_t aes_t0(uint32_t x) {
    const uint32_t s = kAesSbox[x];
    const uint32_t s2 = aes_xtime(s), s3 = s2 ^ s;
    return s2 | (s << 8) | (s << 16) | (s3 << 24);
}

struct aes_ttables {
    uint32_t T[4][256];
};

inline aes_ttables aes_make_tables() {
    aes_ttables t{};
    for (int x = 0; x < 256; ++x) {
        const uint32_t v = aes_t0((uint32_t)x);
        t.T[0][x] = v;
        t.T[1][x] = aes_rotl(v, 8);
        t.T[2][x] = aes_rotl(v, 16);
        t.T[3][x] = aes_rotl(v, 24);
    }
    return t;
}

// FIPS-197 key expansion, Nk = 8: 60 little-endian words (round r uses rk[4r .. 4r+3]).
// sbox: any indexable byte table (the constant array on the host, T0 bytes on the device).
template <class SBOX>
__host__ __device__ inline void aes256_expand(const uint32_t key[8], uint32_t rk[60], SBOX sbox) {
    for (int i = 0; i < 8; ++i) rk[i] = key[i];
    uint32_t rcon = 1;
    for (int i = 8; i < 60; ++i) {
        uint32_t t = rk[i - 1];
        if ((i & 7) == 0) {
            t = (t >> 8) | (t << 24);   // RotWord on little-endian words
            t = sbox(t & 0xFF) | (sbox((t >> 8) & 0xFF) << 8) | (sbox((t >> 16) & 0xFF) << 16) |
                (sbox(t >> 24) << 24);
            t ^= rcon;
            rcon = aes_xtime(rcon);
        } else if ((i & 7) == 4) {
            t = sbox(t & 0xFF) | (sbox((t >> 8) & 0xFF) << 8) | (sbox((t >> 16) & 0xFF) << 16) | (sbox(t >> 24) << 24);
        }
        rk[i] = rk[i - 8] ^ t;
    }
}

// One block in place; T: four 256-entry tables (T[k * 256 + x]), rk: 60 words.
template <class TBL, class RK>
__host__ __device__ inline void aes256_encrypt(uint32_t& w0, uint32_t& w1, uint32_t& w2, uint32_t& w3, TBL T,
                                               RK rk) {
    w0 ^= rk(0); w1 ^= rk(1); w2 ^= rk(2); w3 ^= rk(3);
#pragma unroll
    for (int r = 1; r < 14; ++r) {
        const uint32_t n0 = T(0, w0 & 0xFF) ^ T(1, (w1 >> 8) & 0xFF) ^ T(2, (w2 >> 16) & 0xFF) ^ T(3, w3 >> 24) ^ rk(4 * r);
        const uint32_t n1 = T(0, w1 & 0xFF) ^ T(1, (w2 >> 8) & 0xFF) ^ T(2, (w3 >> 16) & 0xFF) ^ T(3, w0 >> 24) ^ rk(4 * r + 1);
        const uint32_t n2 = T(0, w2 & 0xFF) ^ T(1, (w3 >> 8) & 0xFF) ^ T(2, (w0 >> 16) & 0xFF) ^ T(3, w1 >> 24) ^ rk(4 * r + 2);
        const uint32_t n3 = T(0, w3 & 0xFF) ^ T(1, (w0 >> 8) & 0xFF) ^ T(2, (w1 >> 16) & 0xFF) ^ T(3, w2 >> 24) ^ rk(4 * r + 3);
        w0 = n0; w1 = n1; w2 = n2; w3 = n3;
    }
    // final round: SubBytes + ShiftRows (S-box byte = byte 1 of T0)
    auto S = [&](uint32_t x) { return (T(0, x) >> 8) & 0xFFu; };
    const uint32_t n0 = S(w0 & 0xFF) | (S((w1 >> 8) & 0xFF) << 8) | (S((w2 >> 16) & 0xFF) << 16) | (S(w3 >> 24) << 24);
    const uint32_t n1 = S(w1 & 0xFF) | (S((w2 >> 8) & 0xFF) << 8) | (S((w3 >> 16) & 0xFF) << 16) | (S(w0 >> 24) << 24);
    const uint32_t n2 = S(w2 & 0xFF) | (S((w3 >> 8) & 0xFF) << 8) | (S((w0 >> 16) & 0xFF) << 16) | (S(w1 >> 24) << 24);
    const uint32_t n3 = S(w3 & 0xFF) | (S((w0 >> 8) & 0xFF) << 8) | (S((w1 >> 16) & 0xFF) << 16) | (S(w2 >> 24) << 24);
    w0 = n0 ^ rk(56); w1 = n1 ^ rk(57); w2 = n2 ^ rk(58); w3 = n3 ^ rk(59);
}


}  // namespace pvhip
