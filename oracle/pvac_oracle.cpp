// pvac_oracle.cpp — TEST INFRASTRUCTURE ONLY: CPU restatement of the pvac-hfhe hot path.
//
// This is the CHECKER for the MI355X engine. Only tests/, __graft_entry__.smoke() and the
// cpu_baseline leg of bench.py load it; the product library never does. Parity of this
// restatement against the unmodified reference is PINNED by tests/test_oracle.py using the
// golden vectors in tests/golden/ (minted by oracle/ref_harness.cpp from /root/reference).
//
// Written C-style in C++17 because one piece of the algorithm IS a libstdc++ container: the
// emit order of ct_mul is the iteration order of std::unordered_map after reserve()
// (reference include/pvac/ops/arithmetic.hpp:72-101), so the restatement aggregates through
// the same container to stay faithful.
#include "pvac_oracle.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <cmath>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

using u64 = uint64_t;
using u128 = unsigned __int128;
constexpr u64 M63 = 0x7FFFFFFFFFFFFFFFULL;
constexpr u64 ALL = ~0ULL;

struct F { u64 lo, hi; };

// core/field.hpp:26-48 — fold bit 127 (2^127 == 1 mod p), then subtract p once when the
// folded value is p or 2^127. Canonical for every 128-bit input.
inline F from_words(u64 lo, u64 hi) {
    u64 top = hi >> 63;
    hi &= M63;
    u128 s = (u128)lo + top;
    lo = (u64)s;
    hi += (u64)(s >> 64);
    const bool reduce = (hi >> 63) != 0 || (hi == M63 && lo == ALL);
    if (!reduce) return {lo, hi};
    // value - p = value - (2^127 - 1): lo - (2^64-1) with borrow, hi - (2^63-1) - borrow
    u64 borrow = lo < ALL ? 1u : 0u;
    return {lo - ALL, hi - M63 - borrow};
}

// core/field.hpp:50-56 — NOTE the high word sum is truncated to 64 bits before folding.
inline F add(const F& a, const F& b) {
    u128 l = (u128)a.lo + b.lo;
    u64 h = a.hi + b.hi + (u64)(l >> 64);   // truncated exactly as (uint64_t)t1
    return from_words((u64)l, h);
}

// core/field.hpp:58-67 — p - a with a 128-bit borrow, then fold.
inline F neg(const F& a) {
    u128 l = (u128)ALL - a.lo;
    u64 borrow = (u64)(l >> 64);            // always 0: (2^64-1) - lo never borrows (kept for fidelity)
    u64 h = M63 - a.hi - borrow;
    return from_words((u64)l, h);
}

inline F sub(const F& a, const F& b) { return add(a, neg(b)); }   // core/field.hpp:69-71

// core/field.hpp:113-154 + 179-213 — exact 256-bit product, two Mersenne folds, canonicalise.
inline F mul(const F& a, const F& b) {
    u128 p00 = (u128)a.lo * b.lo, p01 = (u128)a.lo * b.hi, p10 = (u128)a.hi * b.lo, p11 = (u128)a.hi * b.hi;
    u64 z0 = (u64)p00;
    u128 m1 = (p00 >> 64) + (u64)p01 + (u64)p10;
    u64 z1 = (u64)m1;
    u128 m2 = (p01 >> 64) + (p10 >> 64) + (u64)p11 + (m1 >> 64);
    u64 z2 = (u64)m2;
    u64 z3 = (u64)(p11 >> 64) + (u64)(m2 >> 64);
    // first fold: low 127 bits + (z >> 127)
    u64 h0 = (z1 >> 63) | (z2 << 1), h1 = (z2 >> 63) | (z3 << 1), h2 = z3 >> 63;
    u128 t0 = (u128)z0 + h0;
    u128 t1 = (u128)(z1 & M63) + h1 + (u64)(t0 >> 64);
    u64 x0 = (u64)t0, x1 = (u64)t1, x2 = h2 + (u64)(t1 >> 64);
    // second fold
    u64 y_h = (x1 >> 63) | (x2 << 1);
    u128 s0 = (u128)x0 + y_h;
    u64 y1 = (x1 & M63) + (u64)(s0 >> 64);
    return from_words((u64)s0, y1);
}

inline F fpow(F a, u64 e) {   // core/field.hpp:215-227
    F r{1, 0};
    while (e) { if (e & 1) r = mul(r, a); a = mul(a, a); e >>= 1; }
    return r;
}

// core/field.hpp:229-273 computes a^(p-2) with a 5-bit window; the inverse is unique and
// canonical, so plain square-and-multiply over the exponent bits gives identical words.
inline F inv(const F& a) {
    F r{1, 0};
    // e = 2^127 - 3 : bits 126..2 set, bit1 = 0, bit0 = 1
    for (int bit = 126; bit >= 0; --bit) {
        r = mul(r, r);
        bool set = (bit >= 2) || (bit == 0);
        if (set) r = mul(r, a);
    }
    return r;
}

// ------------------------------------------------------------------ SHA-256 (FIPS 180-4)
// core/hash.hpp:24-178 is a textbook FIPS 180-4 implementation; restated here.
struct Sha {
    uint32_t st[8];
    u64 total;
    uint8_t blk[64];
    size_t used;
    static uint32_t ror(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }
    void begin() {
        static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                       0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
        std::memcpy(st, iv, sizeof iv);
        total = 0; used = 0;
    }
    void compress(const uint8_t* p) {
        static const uint32_t K[64] = {
            0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
            0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
            0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
            0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
            0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
            0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
            0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
            0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
        uint32_t w[64];
        for (int i = 0; i < 16; ++i)
            w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 64; ++i) {
            uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
            uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
        for (int i = 0; i < 64; ++i) {
            uint32_t t1 = h + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
            uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
    }
    void feed(const void* data, size_t n) {
        const uint8_t* p = (const uint8_t*)data;
        total += n;
        while (n) {
            size_t k = std::min(n, (size_t)64 - used);
            std::memcpy(blk + used, p, k);
            used += k; p += k; n -= k;
            if (used == 64) { compress(blk); used = 0; }
        }
    }
    void feed64(u64 x) { uint8_t b[8]; for (int i = 0; i < 8; ++i) b[i] = (uint8_t)(x >> (8 * i)); feed(b, 8); }
    void end(uint8_t out[32]) {
        u64 bits = total * 8;
        uint8_t pad = 0x80;
        feed(&pad, 1);
        uint8_t z = 0;
        while (used != 56) feed(&z, 1);
        uint8_t L[8];
        for (int i = 0; i < 8; ++i) L[i] = (uint8_t)(bits >> (56 - 8 * i));
        feed(L, 8);
        for (int i = 0; i < 8; ++i) {
            out[4 * i] = (uint8_t)(st[i] >> 24); out[4 * i + 1] = (uint8_t)(st[i] >> 16);
            out[4 * i + 2] = (uint8_t)(st[i] >> 8); out[4 * i + 3] = (uint8_t)st[i];
        }
    }
};

inline u64 le64(const uint8_t* p) { u64 x = 0; for (int i = 7; i >= 0; --i) x = (x << 8) | p[i]; return x; }

// crypto/matrix.hpp:15-92 — counter-mode SHA-256 stream, rejection-bounded draws, first k
// distinct values in draw order.
std::vector<int> choose_k(int k, int N, const char* label, const u64* words, int nwords) {
    std::vector<int> out;
    if (k <= 0) return out;
    if (N < k) return out;   // the reference would spin forever here
    const size_t lablen = std::strlen(label);
    u64 ctr = 0;
    uint8_t buf[32];
    int pos = 32;
    auto next = [&]() -> u64 {
        if (pos >= 32) {
            Sha s; s.begin();
            s.feed(label, lablen);
            for (int i = 0; i < nwords; ++i) s.feed64(words[i]);
            s.feed64(ctr++);
            s.end(buf);
            pos = 0;
        }
        u64 v = le64(buf + pos);
        pos += 8;
        return v;
    };
    auto bounded = [&](u64 M) -> u64 {
        if (M <= 1) return 0;   // no draw consumed (matrix.hpp:62-65)
        const u64 lim = ALL - (ALL % M);
        for (;;) { u64 x = next(); if (x <= lim) return x % M; }
    };
    std::vector<uint8_t> seen((size_t)N, 0);
    out.reserve((size_t)k);
    while ((int)out.size() < k) {
        int x = (int)bounded((u64)N);
        if (!seen[(size_t)x]) { seen[(size_t)x] = 1; out.push_back(x); }
    }
    return out;
}

// ------------------------------------------------------------------ cipher model
struct Lyr { uint32_t rule, pa, pb; u64 ztag, nlo, nhi; };
struct Edg { uint32_t layer; uint16_t idx; uint8_t ch; F w; const u64* s_in; std::vector<u64> s; };
struct Ct { std::vector<Lyr> L; std::vector<Edg> E; };

Ct load(const orc_cipher* c) {
    Ct C;
    C.L.resize(c->nL);
    for (u64 i = 0; i < c->nL; ++i) {
        const orc_layer& l = c->layers[i];
        C.L[i] = {l.rule, l.pa, l.pb, l.ztag, l.nonce_lo, l.nonce_hi};
    }
    C.E.resize(c->nE);
    for (u64 i = 0; i < c->nE; ++i) {
        u64 m = c->meta[i];
        Edg& e = C.E[i];
        e.layer = (uint32_t)m; e.idx = (uint16_t)(m >> 32); e.ch = (uint8_t)(m >> 48);
        e.w = {c->w_lo[i], c->w_hi[i]};
        e.s_in = c->sigma ? c->sigma + i * c->sigma_words : nullptr;
        if (e.s_in) e.s.assign(e.s_in, e.s_in + c->sigma_words);
    }
    return C;
}

int store(const Ct& C, orc_cipher* o, uint32_t sigma_words) {
    if (C.L.size() > o->capL || C.E.size() > o->capE) return -1;
    o->nL = C.L.size(); o->nE = C.E.size();
    for (size_t i = 0; i < C.L.size(); ++i) {
        const Lyr& l = C.L[i];
        o->layers[i] = orc_layer{l.rule, l.pa, l.pb, 0, l.ztag, l.nlo, l.nhi};
    }
    for (size_t i = 0; i < C.E.size(); ++i) {
        const Edg& e = C.E[i];
        o->meta[i] = (u64)e.layer | ((u64)e.idx << 32) | ((u64)e.ch << 48);
        o->w_lo[i] = e.w.lo; o->w_hi[i] = e.w.hi;
        if (o->sigma) {
            if (e.s.size() == sigma_words) std::memcpy(o->sigma + i * sigma_words, e.s.data(), sigma_words * 8);
            else std::memset(o->sigma + i * sigma_words, 0, sigma_words * 8);
        }
    }
    return 0;
}

// ops/encrypt.hpp:73-104 — keep layers referenced by edges plus everything their PROD
// parents reach; renumber preserving order; a no-op when nothing is dropped.
void compact_layers(Ct& C) {
    const size_t L = C.L.size();
    if (!L) return;
    std::vector<uint8_t> keep(L, 0);
    for (auto& e : C.E) if (e.layer < L) keep[e.layer] = 1;
    bool grew = true;
    while (grew) {
        grew = false;
        for (size_t i = 0; i < L; ++i) {
            if (!keep[i] || C.L[i].rule != 1) continue;
            for (uint32_t p : {C.L[i].pa, C.L[i].pb})
                if (p < L && !keep[p]) { keep[p] = 1; grew = true; }
        }
    }
    std::vector<uint32_t> id(L, 0xFFFFFFFFu);
    std::vector<Lyr> out;
    for (size_t i = 0; i < L; ++i) if (keep[i]) { id[i] = (uint32_t)out.size(); out.push_back(C.L[i]); }
    if (out.size() == L) return;
    for (auto& l : out) if (l.rule == 1) { l.pa = l.pa < L ? id[l.pa] : 0xFFFFFFFFu; l.pb = l.pb < L ? id[l.pb] : 0xFFFFFFFFu; }
    for (auto& e : C.E) e.layer = e.layer < L ? id[e.layer] : 0xFFFFFFFFu;
    C.L.swap(out);
}

// ops/encrypt.hpp:39-71 — merge equal (layer, idx, ch): sequential fp_add of weights in edge
// order (quirk-exact), XOR of sigmas; drop merged entries with w == 0 and sigma == 0; output
// ordered by (layer, idx, P before M). With sigma tracking off (weights-only projection) a
// merged entry is dropped when its weight is zero: real sigmas XOR to zero exactly when copies
// of the same edge cancel (A - A: w = 0 and sigma = 0, dropped by the reference), while a zero
// sum of distinct edges (whose sigmas would not cancel) has probability ~1/p.
void compact_edges(Ct& C, uint32_t B, uint32_t sigma_words, bool track_sigma) {
    struct Acc { bool hp = false, hm = false; F wp{0, 0}, wm{0, 0}; std::vector<u64> sp, sm; };
    const size_t L = C.L.size();
    std::vector<Acc> acc(L * B);
    for (auto& e : C.E) {
        Acc& a = acc[(size_t)e.layer * B + e.idx];
        bool p = e.ch == 0;
        bool& have = p ? a.hp : a.hm;
        F& w = p ? a.wp : a.wm;
        std::vector<u64>& s = p ? a.sp : a.sm;
        if (!have) { have = true; w = {0, 0}; if (track_sigma) s.assign(sigma_words, 0); }
        w = add(w, e.w);
        if (track_sigma && e.s.size() == sigma_words) for (uint32_t i = 0; i < sigma_words; ++i) s[i] ^= e.s[i];
    }
    auto nonzero = [&](const F& w, const std::vector<u64>& s) {
        if (w.lo | w.hi) return true;
        if (!track_sigma) return false;
        for (u64 x : s) if (x) return true;
        return false;
    };
    std::vector<Edg> out;
    for (size_t l = 0; l < L; ++l)
        for (uint32_t k = 0; k < B; ++k) {
            Acc& a = acc[l * B + k];
            if (a.hp && nonzero(a.wp, a.sp)) out.push_back(Edg{(uint32_t)l, (uint16_t)k, 0, a.wp, nullptr, a.sp});
            if (a.hm && nonzero(a.wm, a.sm)) out.push_back(Edg{(uint32_t)l, (uint16_t)k, 1, a.wm, nullptr, a.sm});
        }
    C.E.swap(out);
}

void guard(const orc_params* prm, Ct& C, uint32_t sigma_words, bool track_sigma) {   // encrypt.hpp:106-111
    if (C.E.size() > prm->edge_budget) compact_edges(C, prm->B, sigma_words, track_sigma);
}

// crypto/matrix.hpp:254-264
u64 ztag_of(u64 canon, u64 nlo, u64 nhi) {
    Sha s; s.begin();
    s.feed("pvac.dom.ztag", 13);
    s.feed64(canon); s.feed64(nlo); s.feed64(nhi);
    uint8_t d[32]; s.end(d);
    return le64(d);
}

// crypto/matrix.hpp:267-303
void sigma_of(const orc_params* prm, const u64* H, u64 ztag, u64 nlo, u64 nhi, uint32_t idx, uint32_t ch, u64 salt,
              u64* out) {
    const uint32_t words_per_col = (prm->m_bits + 63) / 64;
    std::memset(out, 0, words_per_col * 8);
    const u64 w[7] = {prm->canon_tag, ztag, nlo, nhi, (u64)idx, (u64)ch, salt};
    for (int c : choose_k((int)prm->x_col_wt, (int)prm->n_bits, "pvac.dom.x_seed", w, 7)) {
        const u64* col = H + (size_t)c * words_per_col;
        for (uint32_t i = 0; i < words_per_col; ++i) out[i] ^= col[i];
    }
    for (int r : choose_k((int)prm->err_wt, (int)prm->m_bits, "pvac.dom.noise", w, 7))
        out[(size_t)r >> 6] ^= 1ULL << (r & 63);
}

// ------------------------------------------------------------------ LPN PRF (crypto/lpn.hpp)
// AES-256 (FIPS-197), byte-oriented: SubBytes / ShiftRows / MixColumns / AddRoundKey.
const uint8_t kSbox[256] = {
    0x63,0x7c,0x77,0x7b,0xf2,0x6b,0x6f,0xc5,0x30,0x01,0x67,0x2b,0xfe,0xd7,0xab,0x76,0xca,0x82,0xc9,0x7d,0xfa,0x59,0x47,0xf0,
    0xad,0xd4,0xa2,0xaf,0x9c,0xa4,0x72,0xc0,0xb7,0xfd,0x93,0x26,0x36,0x3f,0xf7,0xcc,0x34,0xa5,0xe5,0xf1,0x71,0xd8,0x31,0x15,
    0x04,0xc7,0x23,0xc3,0x18,0x96,0x05,0x9a,0x07,0x12,0x80,0xe2,0xeb,0x27,0xb2,0x75,0x09,0x83,0x2c,0x1a,0x1b,0x6e,0x5a,0xa0,
    0x52,0x3b,0xd6,0xb3,0x29,0xe3,0x2f,0x84,0x53,0xd1,0x00,0xed,0x20,0xfc,0xb1,0x5b,0x6a,0xcb,0xbe,0x39,0x4a,0x4c,0x58,0xcf,
    0xd0,0xef,0xaa,0xfb,0x43,0x4d,0x33,0x85,0x45,0xf9,0x02,0x7f,0x50,0x3c,0x9f,0xa8,0x51,0xa3,0x40,0x8f,0x92,0x9d,0x38,0xf5,
    0xbc,0xb6,0xda,0x21,0x10,0xff,0xf3,0xd2,0xcd,0x0c,0x13,0xec,0x5f,0x97,0x44,0x17,0xc4,0xa7,0x7e,0x3d,0x64,0x5d,0x19,0x73,
    0x60,0x81,0x4f,0xdc,0x22,0x2a,0x90,0x88,0x46,0xee,0xb8,0x14,0xde,0x5e,0x0b,0xdb,0xe0,0x32,0x3a,0x0a,0x49,0x06,0x24,0x5c,
    0xc2,0xd3,0xac,0x62,0x91,0x95,0xe4,0x79,0xe7,0xc8,0x37,0x6d,0x8d,0xd5,0x4e,0xa9,0x6c,0x56,0xf4,0xea,0x65,0x7a,0xae,0x08,
    0xba,0x78,0x25,0x2e,0x1c,0xa6,0xb4,0xc6,0xe8,0xdd,0x74,0x1f,0x4b,0xbd,0x8b,0x8a,0x70,0x3e,0xb5,0x66,0x48,0x03,0xf6,0x0e,
    0x61,0x35,0x57,0xb9,0x86,0xc1,0x1d,0x9e,0xe1,0xf8,0x98,0x11,0x69,0xd9,0x8e,0x94,0x9b,0x1e,0x87,0xe9,0xce,0x55,0x28,0xdf,
    0x8c,0xa1,0x89,0x0d,0xbf,0xe6,0x42,0x68,0x41,0x99,0x2d,0x0f,0xb0,0x54,0xbb,0x16};

inline uint8_t xt(uint8_t b) { return (uint8_t)((b << 1) ^ ((b & 0x80) ? 0x1b : 0)); }

struct Aes256 {
    uint8_t rk[15][16];
    void init(const uint8_t key[32]) {
        uint8_t w[60][4];
        for (int i = 0; i < 8; ++i) for (int j = 0; j < 4; ++j) w[i][j] = key[4 * i + j];
        uint8_t rcon = 1;
        for (int i = 8; i < 60; ++i) {
            uint8_t t[4] = {w[i - 1][0], w[i - 1][1], w[i - 1][2], w[i - 1][3]};
            if (i % 8 == 0) {
                const uint8_t t0 = t[0];
                t[0] = kSbox[t[1]] ^ rcon; t[1] = kSbox[t[2]]; t[2] = kSbox[t[3]]; t[3] = kSbox[t0];
                rcon = xt(rcon);
            } else if (i % 8 == 4) {
                for (auto& b : t) b = kSbox[b];
            }
            for (int j = 0; j < 4; ++j) w[i][j] = w[i - 8][j] ^ t[j];
        }
        for (int r = 0; r < 15; ++r) for (int c = 0; c < 4; ++c) for (int j = 0; j < 4; ++j) rk[r][4 * c + j] = w[4 * r + c][j];
    }
    void encrypt(uint8_t s[16]) const {   // s[4c + r] = row r of column c
        for (int i = 0; i < 16; ++i) s[i] ^= rk[0][i];
        for (int r = 1; r <= 14; ++r) {
            uint8_t t[16];
            for (int c = 0; c < 4; ++c)
                for (int row = 0; row < 4; ++row) t[4 * c + row] = kSbox[s[4 * ((c + row) & 3) + row]];   // Sub+Shift
            if (r < 14)
                for (int c = 0; c < 4; ++c) {   // MixColumns
                    const uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                    t[4 * c] = xt(a0) ^ (xt(a1) ^ a1) ^ a2 ^ a3;
                    t[4 * c + 1] = a0 ^ xt(a1) ^ (xt(a2) ^ a2) ^ a3;
                    t[4 * c + 2] = a0 ^ a1 ^ xt(a2) ^ (xt(a3) ^ a3);
                    t[4 * c + 3] = (xt(a0) ^ a0) ^ a1 ^ a2 ^ xt(a3);
                }
            for (int i = 0; i < 16; ++i) s[i] = t[i] ^ rk[r][i];
        }
    }
};

// crypto/lpn.hpp:41-147 AesCtr256: counter block = le64(nonce + i) || 0^64, u64 stream with a
// one-word buffer, rejection-bounded draws.
struct Ctr {
    Aes256 aes;
    u64 ctr = 0, buf = 0;
    bool has = false;
    void init(const uint8_t key[32], u64 nonce) { aes.init(key); ctr = nonce; has = false; }
    u64 next() {
        if (has) { has = false; return buf; }
        uint8_t b[16] = {0};
        for (int i = 0; i < 8; ++i) b[i] = (uint8_t)(ctr >> (8 * i));
        ++ctr;
        aes.encrypt(b);
        buf = le64(b + 8);
        has = true;
        return le64(b);
    }
    u64 bounded(u64 M) {
        if (M <= 1) return 0;
        const u64 lim = ~0ULL - (~0ULL % M);
        for (;;) { const u64 x = next(); if (x < lim) return x % M; }
    }
};

u64 fnv1a(const char* d) {   // lpn.hpp:150-157
    u64 h = 0xcbf29ce484222325ull;
    for (const char* p = d; *p; ++p) { h ^= (uint8_t)*p; h *= 0x100000001b3ull; }
    return h;
}

// lpn.hpp:159-186
void derive_key(const orc_secret* sk, u64 canon, u64 ztag, u64 nlo, u64 nhi, const char* dom, uint8_t key[32],
                u64& nonce) {
    Sha h; h.begin();
    for (int i = 0; i < 4; ++i) h.feed64(sk->prf_k[i]);
    h.feed64(canon);
    h.feed(sk->H_digest, 32);
    h.feed64(ztag); h.feed64(nlo); h.feed64(nhi);
    const u64 dh = fnv1a(dom);
    h.feed64(dh);
    h.end(key);
    nonce = dh ^ nlo;
}

inline int parity(u64 x) { return __builtin_parityll(x); }

const char* const kDoms[6] = {"pvac.prf.r.1", "pvac.prf.r.2", "pvac.prf.r.3",
                              "pvac.prf.noise.1", "pvac.prf.noise.2", "pvac.prf.noise.3"};

// lpn.hpp:188-261 prf_R_core. toep_127 keeps the low 127 coefficients of ybits x top over GF(2),
// and coefficient j only involves coefficients <= j of either factor, so rows >= 127 of the LPN
// stream never reach the output: rows = 127 is exact. full_rows = 1 runs all lpn_t rows.
F prf_core(const orc_secret* sk, u64 canon, u64 ztag, u64 nlo, u64 nhi, const char* dom, bool full_rows) {
    const uint32_t sw = (sk->lpn_n + 63) / 64;
    uint8_t key[32];
    u64 nonce;
    derive_key(sk, canon, ztag, nlo, nhi, dom, key, nonce);
    Ctr prg;
    prg.init(key, nonce);
    const uint32_t rows = full_rows ? sk->lpn_t : std::min<uint32_t>(sk->lpn_t, 127);
    u64 y[2] = {0, 0};
    for (uint32_t r = 0; r < rows; ++r) {
        u64 acc = 0;
        for (uint32_t w = 0; w < sw; ++w) acc ^= prg.next() & sk->lpn_s[w];
        const int e = prg.bounded(sk->tau_den) < sk->tau_num ? 1 : 0;
        if (r < 128) y[r >> 6] |= (u64)(parity(acc) ^ e) << (r & 63);
    }
    uint8_t tk[32];
    u64 tn;
    derive_key(sk, canon, ztag, nlo, nhi, "pvac.dom.toeplitz", tk, tn);
    tn ^= fnv1a(dom);
    Ctr tp;
    tp.init(tk, tn);
    const u64 t0 = tp.next(), t1 = tp.next();
    // low 127 bits of y * top (carry-less)
    u64 lo = 0, hi = 0;
    for (int i = 0; i < 127; ++i) {
        if (!((y[i >> 6] >> (i & 63)) & 1)) continue;
        if (i == 0) { lo ^= t0; hi ^= t1; }
        else if (i < 64) { lo ^= t0 << i; hi ^= (t1 << i) | (t0 >> (64 - i)); }
        else if (i == 64) { hi ^= t0; }
        else { hi ^= t0 << (i - 64); }
    }
    hi &= 0x7FFFFFFFFFFFFFFFull;
    F r = from_words(lo, hi);   // hash_to_fp_nonzero (lpn.hpp:25-37)
    if (!(r.lo | r.hi)) r = F{1, 0};
    return r;
}

F prf_R(const orc_secret* sk, u64 canon, u64 z, u64 lo, u64 hi) {   // lpn.hpp:263-268
    return mul(mul(prf_core(sk, canon, z, lo, hi, kDoms[0], false), prf_core(sk, canon, z, lo, hi, kDoms[1], false)),
               prf_core(sk, canon, z, lo, hi, kDoms[2], false));
}
F prf_R_noise(const orc_secret* sk, u64 canon, u64 z, u64 lo, u64 hi) {   // lpn.hpp:270-275
    return mul(mul(prf_core(sk, canon, z, lo, hi, kDoms[3], false), prf_core(sk, canon, z, lo, hi, kDoms[4], false)),
               prf_core(sk, canon, z, lo, hi, kDoms[5], false));
}
// ops/encrypt.hpp:113-128
F prf_noise_delta(const orc_secret* sk, u64 canon, u64 z, u64 lo, u64 hi, uint32_t group, uint32_t kind) {
    const u64 g = (u64)group + 1, k = (u64)kind + 1;
    lo ^= 0x9e3779b97f4a7c15ull * g;
    hi ^= 0x94d049bb133111ebull * g;
    z ^= 0x517cc1b727220a95ull * g;
    lo ^= k;
    hi ^= k << 32;
    z ^= k << 48;
    return prf_R_noise(sk, canon, z, lo, hi);
}

// ------------------------------------------------------------------ enc_value (ops/encrypt.hpp)
struct Stream {
    const u64* p;
    size_t n, i = 0;
    bool over = false;
    u64 next() { if (i < n) return p[i++]; over = true; return 0; }
};

F rand_fp_nonzero(Stream& rs) {   // types.hpp:145-155
    for (;;) {
        const u64 lo = rs.next();
        const u64 hi = rs.next() & 0x7FFFFFFFFFFFFFFFull;
        const F x = from_words(lo, hi);
        if ((x.lo | x.hi) || rs.over) return x;
    }
}

// ops/encrypt.hpp:162-258 enc_fp_depth
Ct enc_fp_depth(const orc_params* prm, const orc_secret* sk, const u64* H, const u64* powg, const F& v, int Z2, int Z3,
                Stream& rs) {
    const uint32_t B = prm->B, sw = (prm->m_bits + 63) / 64;
    auto pg = [&](uint32_t i) { return F{powg[2 * i], powg[2 * i + 1]}; };
    Ct C;
    Lyr L{0, 0, 0, 0, 0, 0};
    L.nlo = rs.next();
    L.nhi = rs.next();
    L.ztag = ztag_of(prm->canon_tag, L.nlo, L.nhi);
    C.L.push_back(L);
    constexpr int S = 8;
    int idx[S];
    uint8_t ch[S];
    F r[S];
    std::vector<int> used;
    for (int j = 0; j < S; ++j) {
        int x;
        do { x = (int)(rs.next() % B); } while (std::find(used.begin(), used.end(), x) != used.end() && !rs.over);
        used.push_back(x);
        idx[j] = x;
        ch[j] = (uint8_t)(rs.next() & 1);
    }
    F sumg{0, 0};
    for (int j = 0; j < S - 1; ++j) {
        r[j] = rand_fp_nonzero(rs);
        const F term = mul(r[j], pg(idx[j]));
        sumg = ch[j] == 0 ? add(sumg, term) : sub(sumg, term);
    }
    const F r_last = mul(sub(v, sumg), inv(pg(idx[S - 1])));
    r[S - 1] = ch[S - 1] == 0 ? r_last : neg(r_last);
    const F R = prf_R(sk, prm->canon_tag, L.ztag, L.nlo, L.nhi);
    auto edge = [&](uint32_t i, uint8_t c, const F& w) {
        Edg e{0, (uint16_t)i, c, w, nullptr, {}};
        const u64 salt = rs.next();
        if (H) { e.s.assign(sw, 0); sigma_of(prm, H, L.ztag, L.nlo, L.nhi, i, c, salt, e.s.data()); }
        C.E.push_back(std::move(e));
    };
    for (int j = 0; j < S; ++j) edge((uint32_t)idx[j], ch[j], mul(r[j], R));
    const int total = Z2 + Z3;
    F dacc{0, 0};
    int gid = 0;
    auto next_delta = [&](int left, uint32_t kind) {
        if (left <= 1) return neg(dacc);
        const F d = prf_noise_delta(sk, prm->canon_tag, L.ztag, L.nlo, L.nhi, (uint32_t)gid, kind);
        dacc = add(dacc, d);
        return d;
    };
    for (int t = 0; t < Z2; ++t, ++gid) {
        const uint32_t i = (uint32_t)(rs.next() % B);
        uint32_t j;
        do { j = (uint32_t)(rs.next() % B); } while (j == i && !rs.over);
        const uint8_t s1 = (uint8_t)(rs.next() & 1), s2 = s1 ^ 1;
        const F D = next_delta(total - gid, 0);
        const F Dp = s1 == 0 ? D : neg(D);
        const F ri = rand_fp_nonzero(rs);
        const F rj = mul(sub(mul(ri, pg(i)), Dp), inv(pg(j)));
        edge(i, s1, mul(ri, R));
        edge(j, s2, mul(rj, R));
    }
    for (int t = 0; t < Z3; ++t, ++gid) {
        const uint32_t i = (uint32_t)(rs.next() % B);
        uint32_t j, k;
        do { j = (uint32_t)(rs.next() % B); } while (j == i && !rs.over);
        do { k = (uint32_t)(rs.next() % B); } while ((k == i || k == j) && !rs.over);
        const uint8_t s1 = (uint8_t)(rs.next() & 1), s2 = (uint8_t)(rs.next() & 1), s3 = (uint8_t)(rs.next() & 1);
        const F D = next_delta(total - gid, 1);
        const F a = rand_fp_nonzero(rs), b = rand_fp_nonzero(rs);
        F t1 = mul(a, pg(i)), t2 = mul(b, pg(j));
        if (s1) t1 = neg(t1);
        if (s2) t2 = neg(t2);
        const F gk = s3 == 0 ? pg(k) : neg(pg(k));
        const F c = mul(sub(D, add(t1, t2)), inv(gk));
        edge(i, s1, mul(a, R));
        edge(j, s2, mul(b, R));
        edge(k, s3, mul(c, R));
    }
    compact_edges(C, B, sw, H != nullptr);
    guard(prm, C, sw, H != nullptr);
    const size_t n = C.E.size();   // shuffle_edges (encrypt.hpp:156-160)
    for (size_t i = n > 1 ? n - 1 : 0; i > 0; --i) std::swap(C.E[i], C.E[rs.next() % (i + 1)]);
    return C;
}

struct MulHash { size_t operator()(u64 x) const noexcept { return x * 0x9E3779B97F4A7C15ull; } };

// ops/arithmetic.hpp:47-106
int ct_mul_impl(const orc_params* prm, const u64* H, const Ct& A, const Ct& B, const u64* nonces, const u64* salts,
                Ct& C) {
    C.L.clear(); C.E.clear();
    const uint32_t LA = (uint32_t)A.L.size(), LB = (uint32_t)B.L.size();
    for (auto& l : A.L) C.L.push_back(l);
    const uint32_t off = (uint32_t)C.L.size();
    for (Lyr l : B.L) { if (l.rule == 1) { l.pa += off; l.pb += off; } C.L.push_back(l); }
    const uint32_t base = (uint32_t)C.L.size();
    size_t nx = 0;
    for (uint32_t la = 0; la < LA; ++la)
        for (uint32_t lb = 0; lb < LB; ++lb) {
            Lyr l{1, la, off + lb, 0, nonces ? nonces[nx] : 0, nonces ? nonces[nx + 1] : 0};
            nx += 2;
            l.ztag = ztag_of(prm->canon_tag, l.nlo, l.nhi);
            C.L.push_back(l);
        }
    struct Agg { F p{0, 0}, m{0, 0}; bool hp = false, hm = false; };
    std::unordered_map<u64, Agg, MulHash> acc;
    acc.reserve(A.E.size() * B.E.size());
    const uint32_t Bm = prm->B;
    for (const Edg& x : A.E)
        for (const Edg& y : B.E) {
            u64 key = ((u64)(x.layer * LB + y.layer) << 32) | (u64)((x.idx + y.idx) % Bm);
            Agg& a = acc[key];
            F prod = mul(x.w, y.w);
            if (x.ch == y.ch) { if (!a.hp) { a.hp = true; a.p = {0, 0}; } a.p = add(a.p, prod); }
            else { if (!a.hm) { a.hm = true; a.m = {0, 0}; } a.m = add(a.m, prod); }
        }
    const uint32_t sw = (prm->m_bits + 63) / 64;
    size_t ns = 0;
    auto emit = [&](uint32_t lid, uint16_t idx, uint8_t ch, const F& w) {
        Edg e{lid, idx, ch, w, nullptr, {}};
        u64 salt = salts ? salts[ns] : 0;
        ++ns;
        if (H) {
            e.s.resize(sw);
            const Lyr& l = C.L[lid];
            sigma_of(prm, H, l.ztag, l.nlo, l.nhi, idx, ch, salt, e.s.data());
        }
        C.E.push_back(std::move(e));
    };
    for (const auto& kv : acc) {
        const uint32_t lid = base + (uint32_t)(kv.first >> 32);
        const uint16_t idx = (uint16_t)(kv.first & 0xFFFF);
        if (kv.second.hp && (kv.second.p.lo | kv.second.p.hi)) emit(lid, idx, 0, kv.second.p);
        if (kv.second.hm && (kv.second.m.lo | kv.second.m.hi)) emit(lid, idx, 1, kv.second.m);
    }
    guard(prm, C, sw, H != nullptr);
    compact_layers(C);
    return 0;
}

// ops/arithmetic.hpp:12-45 (ct_add; ct_sub = ct_add(A, ct_scale(B, p-1)))
void ct_add_impl(const orc_params* prm, const Ct& A, const Ct& Bc, bool negate_b, uint32_t sw, bool track, Ct& C) {
    C.L = A.L;
    const uint32_t off = (uint32_t)A.L.size();
    for (Lyr l : Bc.L) { if (l.rule == 1) { l.pa += off; l.pb += off; } C.L.push_back(l); }
    C.E = A.E;
    const F pm1{ALL - 1, M63};   // fp_neg(1) = p - 1  (arithmetic.hpp:39-41)
    for (Edg e : Bc.E) {
        e.layer += off;
        if (negate_b) e.w = mul(e.w, pm1);
        C.E.push_back(std::move(e));
    }
    guard(prm, C, sw, track);
    compact_layers(C);
}

inline u64 fnv_step(u64 h, u64 x) {
    for (int i = 0; i < 8; ++i) { h ^= (x >> (8 * i)) & 0xFF; h *= 0x100000001b3ULL; }
    return h;
}

}  // namespace

// ==================================================================== C ABI
extern "C" {

#define ELEMWISE(body) for (size_t i = 0; i < n; ++i) { body; }

void orc_fp_from_words(const u64* lo, const u64* hi, u64* olo, u64* ohi, size_t n) {
    ELEMWISE(F r = from_words(lo[i], hi[i]); olo[i] = r.lo; ohi[i] = r.hi)
}
void orc_fp_add(const u64* alo, const u64* ahi, const u64* blo, const u64* bhi, u64* olo, u64* ohi, size_t n) {
    ELEMWISE(F r = add({alo[i], ahi[i]}, {blo[i], bhi[i]}); olo[i] = r.lo; ohi[i] = r.hi)
}
void orc_fp_sub(const u64* alo, const u64* ahi, const u64* blo, const u64* bhi, u64* olo, u64* ohi, size_t n) {
    ELEMWISE(F r = sub({alo[i], ahi[i]}, {blo[i], bhi[i]}); olo[i] = r.lo; ohi[i] = r.hi)
}
void orc_fp_neg(const u64* alo, const u64* ahi, u64* olo, u64* ohi, size_t n) {
    ELEMWISE(F r = neg({alo[i], ahi[i]}); olo[i] = r.lo; ohi[i] = r.hi)
}
void orc_fp_mul(const u64* alo, const u64* ahi, const u64* blo, const u64* bhi, u64* olo, u64* ohi, size_t n) {
    ELEMWISE(F r = mul({alo[i], ahi[i]}, {blo[i], bhi[i]}); olo[i] = r.lo; ohi[i] = r.hi)
}
void orc_fp_inv(const u64* alo, const u64* ahi, u64* olo, u64* ohi, size_t n) {
    ELEMWISE(F r = inv({alo[i], ahi[i]}); olo[i] = r.lo; ohi[i] = r.hi)
}
void orc_fp_pow(const u64* alo, const u64* ahi, const u64* e, u64* olo, u64* ohi, size_t n) {
    ELEMWISE(F r = fpow({alo[i], ahi[i]}, e[i]); olo[i] = r.lo; ohi[i] = r.hi)
}

double orc_fp_binop_timed(int op, const u64* alo, const u64* ahi, const u64* blo, const u64* bhi, u64* olo, u64* ohi,
                          size_t n, int threads) {
    if (threads < 1) threads = 1;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([=] {
            size_t b = n * (size_t)t / (size_t)threads, e = n * (size_t)(t + 1) / (size_t)threads;
            if (op == 0) orc_fp_add(alo + b, ahi + b, blo + b, bhi + b, olo + b, ohi + b, e - b);
            else if (op == 1) orc_fp_sub(alo + b, ahi + b, blo + b, bhi + b, olo + b, ohi + b, e - b);
            else orc_fp_mul(alo + b, ahi + b, blo + b, bhi + b, olo + b, ohi + b, e - b);
        });
    for (auto& x : th) x.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void orc_sha256(const uint8_t* msg, size_t n, uint8_t out[32]) {
    Sha s; s.begin(); s.feed(msg, n); s.end(out);
}

uint64_t orc_layer_ztag(uint64_t canon_tag, uint64_t nlo, uint64_t nhi) { return ztag_of(canon_tag, nlo, nhi); }

int orc_prg_choose_k(int k, int N, const char* label, const uint64_t* words, int nwords, int32_t* out) {
    auto v = choose_k(k, N, label, words, nwords);
    for (size_t i = 0; i < v.size(); ++i) out[i] = v[i];
    return (int)v.size();
}

// crypto/matrix.hpp:191-251
int orc_gen_H(const orc_params* prm, uint64_t* H, uint8_t digest[32]) {
    const uint32_t wpc = (prm->m_bits + 63) / 64;
    std::memset(H, 0, (size_t)prm->n_bits * wpc * 8);
    for (uint32_t c = 0; c < prm->n_bits; ++c) {
        const u64 w[5] = {prm->m_bits, prm->n_bits, prm->h_col_wt, c, prm->canon_tag};
        u64* col = H + (size_t)c * wpc;
        for (int r : choose_k((int)prm->h_col_wt, (int)prm->m_bits, "pvac.dom.h_gen", w, 5)) col[r >> 6] |= 1ULL << (r & 63);
    }
    Sha s; s.begin();
    s.feed("H|v2", 4);
    s.feed64(prm->m_bits); s.feed64(prm->n_bits); s.feed64(prm->h_col_wt);
    const size_t bytes = (prm->m_bits + 7) / 8;
    for (uint32_t c = 0; c < prm->n_bits; ++c) {
        const u64* col = H + (size_t)c * wpc;
        for (size_t b = 0; b < bytes; ++b) { uint8_t x = (uint8_t)(col[b >> 3] >> (8 * (b & 7))); s.feed(&x, 1); }
    }
    s.end(digest);
    return 0;
}

void orc_sigma_from_H(const orc_params* prm, const uint64_t* H, uint64_t ztag, uint64_t nlo, uint64_t nhi, uint32_t idx,
                      uint32_t ch, uint64_t salt, uint64_t* out) {
    sigma_of(prm, H, ztag, nlo, nhi, idx, ch, salt, out);
}

int orc_ct_add(const orc_params* prm, const orc_cipher* A, const orc_cipher* B, int negate_b, orc_cipher* C) {
    Ct a = load(A), b = load(B), c;
    const uint32_t sw = (prm->m_bits + 63) / 64;
    const bool track = A->sigma && B->sigma;
    ct_add_impl(prm, a, b, negate_b != 0, sw, track, c);
    return store(c, C, sw);
}

void orc_ct_mul_caps(const orc_params* prm, const orc_cipher* A, const orc_cipher* B, uint64_t* capL, uint64_t* capE) {
    const u64 keys = A->nL * B->nL * prm->B;
    *capL = A->nL + B->nL + A->nL * B->nL;
    *capE = 2 * std::min<u64>(A->nE * B->nE, keys);
}

int orc_ct_mul(const orc_params* prm, const uint64_t* H, const orc_cipher* A, const orc_cipher* B,
               const uint64_t* nonces, const uint64_t* salts, orc_cipher* C) {
    Ct a = load(A), b = load(B), c;
    int rc = ct_mul_impl(prm, H, a, b, nonces, salts, c);
    if (rc) return rc;
    return store(c, C, (prm->m_bits + 63) / 64);
}

// ops/commit.hpp:12-88
void orc_commit_ct(const orc_params* prm, const uint8_t Hd[32], const orc_cipher* C, uint8_t out[32]) {
    Sha s; s.begin();
    s.feed("pvac.dom.commit", 15);
    s.feed(Hd, 32);
    s.feed64(prm->canon_tag);
    for (u64 i = 0; i < C->nL; ++i) {
        const orc_layer& l = C->layers[i];
        uint8_t r = (uint8_t)l.rule;
        s.feed(&r, 1);
        if (l.rule == 0) { s.feed64(l.ztag); s.feed64(l.nonce_lo); s.feed64(l.nonce_hi); }
        else { s.feed64(l.pa); s.feed64(l.pb); }
    }
    const size_t bytes = (prm->m_bits + 7) / 8;
    for (u64 i = 0; i < C->nE; ++i) {
        u64 m = C->meta[i];
        s.feed64((uint32_t)m);
        s.feed64((uint16_t)(m >> 32));
        uint8_t ch = (uint8_t)(m >> 48);
        s.feed(&ch, 1);
        s.feed64(C->w_lo[i]);
        s.feed64(C->w_hi[i] & M63);
        if (C->sigma) {
            const u64* sg = C->sigma + i * C->sigma_words;
            for (size_t b = 0; b < bytes; ++b) { uint8_t x = (uint8_t)(sg[b >> 3] >> (8 * (b & 7))); s.feed(&x, 1); }
        }
    }
    s.end(out);
}

// ops/decrypt.hpp:12-89, with BASE-layer R supplied by the caller (fixtures hold them).
void orc_prf_core(const orc_secret* sk, uint64_t canon, uint64_t z, uint64_t lo, uint64_t hi, int dom, int full,
                  uint64_t out[2]) {
    const F r = prf_core(sk, canon, z, lo, hi, kDoms[dom], full != 0);
    out[0] = r.lo; out[1] = r.hi;
}
void orc_prf_R(const orc_secret* sk, uint64_t canon, uint64_t z, uint64_t lo, uint64_t hi, int noise, uint64_t out[2]) {
    const F r = noise ? prf_R_noise(sk, canon, z, lo, hi) : prf_R(sk, canon, z, lo, hi);
    out[0] = r.lo; out[1] = r.hi;
}
void orc_prf_noise_delta(const orc_secret* sk, uint64_t canon, uint64_t z, uint64_t lo, uint64_t hi, uint32_t g,
                         uint32_t kind, uint64_t out[2]) {
    const F r = prf_noise_delta(sk, canon, z, lo, hi, g, kind);
    out[0] = r.lo; out[1] = r.hi;
}

// ops/encrypt.hpp:16-27; the Params noise fields (core/types.hpp:48-50), defaults 120 / 0.55 / 16,
// set process-wide for tests by orc_set_noise
static double g_noise_bits = 120.0, g_noise_t2 = 0.55, g_noise_slope = 16.0;
void orc_set_noise(double noise_entropy_bits, double tuple2_fraction, double depth_slope_bits) {
    g_noise_bits = noise_entropy_bits;
    g_noise_t2 = tuple2_fraction;
    g_noise_slope = depth_slope_bits;
}
static void plan_noise(uint32_t B, int depth, int& z2, int& z3) {
    const double budget = g_noise_bits + g_noise_slope * std::max(0, depth);
    const double per2 = 2.0 * std::log2((double)B), per3 = 3.0 * std::log2((double)B);
    z2 = std::max(0, (int)std::floor((budget * g_noise_t2) / std::max(1e-6, per2)));
    z3 = std::max(0, (int)std::floor((budget * (1.0 - g_noise_t2)) / std::max(1e-6, per3)));
    if (z2 + z3 == 1) { if (z3 > 0) ++z3; else ++z2; }
}

int orc_enc_value(const orc_params* prm, const orc_secret* sk, const uint64_t* H, const uint64_t* powg, uint64_t v,
                  const uint64_t* stream, size_t n, int order, orc_cipher* out, size_t* consumed) {
    return orc_enc_value_depth(prm, sk, H, powg, v, 0, stream, n, order, out, consumed);
}

// enc_value_depth (ops/encrypt.hpp:281-287); v = 0 is enc_zero_depth (:293-298): fp_add(0, mask) is
// mask, and the draws are the same
int orc_enc_value_depth(const orc_params* prm, const orc_secret* sk, const uint64_t* H, const uint64_t* powg,
                        uint64_t v, int depth_hint, const uint64_t* stream, size_t n, int order, orc_cipher* out,
                        size_t* consumed) {
    Stream rs{stream, n};
    int Z2, Z3;
    plan_noise(prm->B, depth_hint, Z2, Z3);
    const F val{v, 0};
    const F mask = rand_fp_nonzero(rs);   // encrypt.hpp:281-287
    Ct a, b;
    if (order == 0) {
        a = enc_fp_depth(prm, sk, H, powg, add(val, mask), Z2, Z3, rs);
        b = enc_fp_depth(prm, sk, H, powg, neg(mask), Z2, Z3, rs);
    } else {
        b = enc_fp_depth(prm, sk, H, powg, neg(mask), Z2, Z3, rs);
        a = enc_fp_depth(prm, sk, H, powg, add(val, mask), Z2, Z3, rs);
    }
    // combine_ciphers (encrypt.hpp:260-279)
    Ct C;
    C.L = a.L;
    const uint32_t off = (uint32_t)a.L.size();
    for (Lyr L : b.L) { if (L.rule == 1) { L.pa += off; L.pb += off; } C.L.push_back(L); }
    C.E = std::move(a.E);
    for (auto& e : b.E) { e.layer += off; C.E.push_back(std::move(e)); }
    const uint32_t sw = (prm->m_bits + 63) / 64;
    guard(prm, C, sw, H != nullptr);
    compact_layers(C);
    if (consumed) *consumed = rs.i;
    if (rs.over) return -1;
    return store(C, out, H ? sw : 0) ? -2 : 0;
}

void orc_dec_value(const orc_params* prm, const uint64_t* powg, const orc_cipher* C, const uint64_t* R_base,
                   uint64_t out[2]) {
    const u64 L = C->nL;
    std::vector<F> R(L, F{0, 0});
    std::vector<uint8_t> done(L, 0);
    // PROD layers reference earlier layers in every cipher the ops produce; resolve with an
    // explicit stack so any order works.
    for (u64 root = 0; root < L; ++root) {
        std::vector<u64> stk{root};
        while (!stk.empty()) {
            u64 id = stk.back();
            if (done[id]) { stk.pop_back(); continue; }
            const orc_layer& l = C->layers[id];
            if (l.rule == 0) { R[id] = {R_base[2 * id], R_base[2 * id + 1]}; done[id] = 1; stk.pop_back(); continue; }
            if (!done[l.pa]) { stk.push_back(l.pa); continue; }
            if (!done[l.pb]) { stk.push_back(l.pb); continue; }
            R[id] = mul(R[l.pa], R[l.pb]); done[id] = 1; stk.pop_back();
        }
    }
    std::vector<F> Ri(L);
    for (u64 i = 0; i < L; ++i) Ri[i] = inv(R[i]);
    F acc{0, 0};
    for (u64 i = 0; i < C->nE; ++i) {
        u64 m = C->meta[i];
        uint32_t lid = (uint32_t)m; uint16_t idx = (uint16_t)(m >> 32); uint8_t ch = (uint8_t)(m >> 48);
        F t = mul({C->w_lo[i], C->w_hi[i]}, {powg[2 * idx], powg[2 * idx + 1]});
        t = mul(t, Ri[lid]);
        acc = ch == 0 ? add(acc, t) : sub(acc, t);
    }
    (void)prm;
    out[0] = acc.lo; out[1] = acc.hi;
}

uint64_t orc_bucket_count_after_reserve(uint64_t n) {
    std::unordered_map<u64, int, MulHash> m;
    m.reserve(n);
    return m.bucket_count();
}

double orc_ct_mul_batch_timed(const orc_params* prm, uint64_t npairs, const uint64_t* a_loff, const orc_layer* a_layers,
                              const uint64_t* a_eoff, const uint64_t* a_meta, const uint64_t* a_wlo,
                              const uint64_t* a_whi, const uint64_t* b_loff, const orc_layer* b_layers,
                              const uint64_t* b_eoff, const uint64_t* b_meta, const uint64_t* b_wlo,
                              const uint64_t* b_whi, int threads, uint64_t* out_counts, uint64_t* out_digests) {
    if (threads < 1) threads = 1;
    auto view = [](const uint64_t* loff, const orc_layer* layers, const uint64_t* eoff, const uint64_t* meta,
                   const uint64_t* wlo, const uint64_t* whi, uint64_t i) {
        orc_cipher c{};
        c.nL = loff[i + 1] - loff[i]; c.nE = eoff[i + 1] - eoff[i];
        c.layers = const_cast<orc_layer*>(layers + loff[i]);
        c.meta = const_cast<uint64_t*>(meta + eoff[i]);
        c.w_lo = const_cast<uint64_t*>(wlo + eoff[i]);
        c.w_hi = const_cast<uint64_t*>(whi + eoff[i]);
        return c;
    };
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            std::vector<u64> nonces;
            for (uint64_t i = (uint64_t)t; i < npairs; i += (uint64_t)threads) {
                orc_cipher A = view(a_loff, a_layers, a_eoff, a_meta, a_wlo, a_whi, i);
                orc_cipher B = view(b_loff, b_layers, b_eoff, b_meta, b_wlo, b_whi, i);
                Ct a = load(&A), b = load(&B), c;
                nonces.assign(2 * A.nL * B.nL, 0);
                for (size_t k = 0; k < nonces.size(); ++k) nonces[k] = i * 0x100000001b3ULL + k;
                ct_mul_impl(prm, nullptr, a, b, nonces.data(), nullptr, c);
                u64 h = 0xcbf29ce484222325ULL;
                for (auto& e : c.E) {
                    h = fnv_step(h, (u64)e.layer | ((u64)e.idx << 32) | ((u64)e.ch << 48));
                    h = fnv_step(h, e.w.lo);
                    h = fnv_step(h, e.w.hi);
                }
                if (out_counts) out_counts[i] = c.E.size();
                if (out_digests) out_digests[i] = h;
            }
        });
    for (auto& x : th) x.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

/* batched weights-only ct_add / ct_sub (A13 / A6) over packed pairs, for bench.py's cpu_baseline of
 * the cfg-3 add/sub leg: per-pair output edge counts and FNV-1a edge digests. Returns seconds. */
double orc_ct_add_batch_timed(const orc_params* prm, uint64_t npairs, const uint64_t* a_loff, const orc_layer* a_layers,
                              const uint64_t* a_eoff, const uint64_t* a_meta, const uint64_t* a_wlo,
                              const uint64_t* a_whi, const uint64_t* b_loff, const orc_layer* b_layers,
                              const uint64_t* b_eoff, const uint64_t* b_meta, const uint64_t* b_wlo,
                              const uint64_t* b_whi, int negate_b, int threads, uint64_t* out_counts,
                              uint64_t* out_digests) {
    if (threads < 1) threads = 1;
    auto view = [](const uint64_t* loff, const orc_layer* layers, const uint64_t* eoff, const uint64_t* meta,
                   const uint64_t* wlo, const uint64_t* whi, uint64_t i) {
        orc_cipher c{};
        c.nL = loff[i + 1] - loff[i]; c.nE = eoff[i + 1] - eoff[i];
        c.layers = const_cast<orc_layer*>(layers + loff[i]);
        c.meta = const_cast<uint64_t*>(meta + eoff[i]);
        c.w_lo = const_cast<uint64_t*>(wlo + eoff[i]);
        c.w_hi = const_cast<uint64_t*>(whi + eoff[i]);
        return c;
    };
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            for (uint64_t i = (uint64_t)t; i < npairs; i += (uint64_t)threads) {
                orc_cipher A = view(a_loff, a_layers, a_eoff, a_meta, a_wlo, a_whi, i);
                orc_cipher B = view(b_loff, b_layers, b_eoff, b_meta, b_wlo, b_whi, i);
                Ct a = load(&A), b = load(&B), c;
                ct_add_impl(prm, a, b, negate_b != 0, (prm->m_bits + 63) / 64, false, c);
                u64 h = 0xcbf29ce484222325ULL;
                for (auto& e : c.E) {
                    h = fnv_step(h, (u64)e.layer | ((u64)e.idx << 32) | ((u64)e.ch << 48));
                    h = fnv_step(h, e.w.lo);
                    h = fnv_step(h, e.w.hi);
                }
                if (out_counts) out_counts[i] = c.E.size();
                if (out_digests) out_digests[i] = h;
            }
        });
    for (auto& x : th) x.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

/* cfg 4 on the CPU port (SURVEY 8(d) restatement of tests/test_main.cpp:289-295): per input i,
 * c_0 = x_i, c_k = ct_mul(c_{k-1}, y_{k,i}) for k = 1..depth, weights only, with y_{k,i} = x_i (the
 * cfg-4 shape) or, for k <= nops, operand d = k - 1 of input i: cipher d * ninputs + i of the packed
 * operand batch (the reference's own loop, a fresh enc_value per step, :291-292). Nonces do not reach
 * the edges (only layer records), so they are synthetic here; the FNV-1a edge digest of c_depth is
 * comparable with the engine's. step_edges[d] accumulates |c_{d+1}.E| over the inputs. */
double orc_ct_mul_chain_ops_timed(const orc_params* prm, uint64_t ninputs, const uint64_t* loff, const orc_layer* layers,
                                  const uint64_t* eoff, const uint64_t* meta, const uint64_t* wlo, const uint64_t* whi,
                                  int depth, int nops, const uint64_t* oloff, const orc_layer* olayers,
                                  const uint64_t* oeoff, const uint64_t* ometa, const uint64_t* owlo,
                                  const uint64_t* owhi, int threads, uint64_t* out_counts, uint64_t* out_digests,
                                  uint64_t* step_edges) {
    if (threads < 1) threads = 1;
    std::vector<std::vector<u64>> per((size_t)threads, std::vector<u64>((size_t)(depth > 0 ? depth : 1), 0));
    auto view = [](uint64_t j, const uint64_t* lo, const orc_layer* ly, const uint64_t* eo, const uint64_t* m,
                   const uint64_t* wl, const uint64_t* wh) {
        orc_cipher X{};
        X.nL = lo[j + 1] - lo[j]; X.nE = eo[j + 1] - eo[j];
        X.layers = const_cast<orc_layer*>(ly + lo[j]);
        X.meta = const_cast<uint64_t*>(m + eo[j]);
        X.w_lo = const_cast<uint64_t*>(wl + eo[j]);
        X.w_hi = const_cast<uint64_t*>(wh + eo[j]);
        return load(&X);
    };
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            std::vector<u64> nonces;
            for (uint64_t i = (uint64_t)t; i < ninputs; i += (uint64_t)threads) {
                const Ct x = view(i, loff, layers, eoff, meta, wlo, whi);
                Ct c = x;
                for (int d = 0; d < depth; ++d) {
                    Ct nxt;
                    const Ct y = d < nops ? view((uint64_t)d * ninputs + i, oloff, olayers, oeoff, ometa, owlo, owhi) : x;
                    nonces.assign(2 * c.L.size() * y.L.size(), 0);
                    for (size_t k = 0; k < nonces.size(); ++k) nonces[k] = i * 0x100000001b3ULL + 977u * (u64)d + k;
                    ct_mul_impl(prm, nullptr, c, y, nonces.data(), nullptr, nxt);
                    c = std::move(nxt);
                    per[(size_t)t][(size_t)d] += c.E.size();
                }
                u64 h = 0xcbf29ce484222325ULL;
                for (auto& e : c.E) {
                    h = fnv_step(h, (u64)e.layer | ((u64)e.idx << 32) | ((u64)e.ch << 48));
                    h = fnv_step(h, e.w.lo);
                    h = fnv_step(h, e.w.hi);
                }
                if (out_counts) out_counts[i] = c.E.size();
                if (out_digests) out_digests[i] = h;
            }
        });
    for (auto& x : th) x.join();
    double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (step_edges)
        for (int d = 0; d < depth; ++d) {
            step_edges[d] = 0;
            for (int t = 0; t < threads; ++t) step_edges[d] += per[(size_t)t][(size_t)d];
        }
    return secs;
}

double orc_ct_mul_chain_timed(const orc_params* prm, uint64_t ninputs, const uint64_t* loff, const orc_layer* layers,
                              const uint64_t* eoff, const uint64_t* meta, const uint64_t* wlo, const uint64_t* whi,
                              int depth, int threads, uint64_t* out_counts, uint64_t* out_digests,
                              uint64_t* step_edges) {
    return orc_ct_mul_chain_ops_timed(prm, ninputs, loff, layers, eoff, meta, wlo, whi, depth, 0, nullptr, nullptr,
                                      nullptr, nullptr, nullptr, nullptr, threads, out_counts, out_digests, step_edges);
}

}  // extern "C"
