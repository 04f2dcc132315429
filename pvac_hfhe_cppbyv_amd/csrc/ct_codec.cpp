// ct_codec.cpp — the reference's .ct ciphertext file format <-> SoA batches (host memory).
//
// Format (reference tests/add.cpp:22-155), all little-endian:
//   file   : u32 magic 0x66699666 | u32 version 1 | u64 n_ciphers | cipher * n
//   cipher : u32 |L| | u32 |E| | layer * |L| | edge * |E|
//   layer  : u8 rule | rule 0 (BASE): u64 ztag, u64 nonce_lo, u64 nonce_hi
//                    | rule 1 (PROD): u32 pa, u32 pb
//                    | other        : 24 bytes, read and dropped (written as zeros)
//   edge   : u32 layer_id | u16 idx | u8 ch | u8 0 | u64 w_lo | u64 w_hi | u32 nbits | u64 * ceil(nbits/64)
// PROD layers carry no seed on disk (the reference's putLayer writes pa/pb only), so parsed PROD
// layers have ztag = nonce = 0. Sigma bit-vectors map to the batch's sigma rows; every edge of
// a file must carry the same nbits (the reference's outputs always do).
//
// Parsing is two passes: a sequential header walk (skips only) records each cipher's byte
// offset, then worker threads decode ciphers in parallel into dense CSR arrays. Writing sizes
// every cipher, scans the sizes and serializes ciphers in parallel.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/pvac_hip.h"

namespace {

constexpr uint32_t kCtMagic = 0x66699666u;
constexpr uint32_t kCtVersion = 1u;
constexpr size_t kBaseBytes = 24, kProdBytes = 8, kEdgeHdr = 28;

struct reader {
    const uint8_t* p;
    size_t n, off = 0;
    bool ok = true;
    bool need(size_t k) {
        if (!ok || k > n - off) ok = false;
        return ok;
    }
    uint32_t u32() {
        uint32_t x = 0;
        if (need(4)) { std::memcpy(&x, p + off, 4); off += 4; }
        return x;
    }
    uint64_t u64() {
        uint64_t x = 0;
        if (need(8)) { std::memcpy(&x, p + off, 8); off += 8; }
        return x;
    }
    uint8_t u8() {
        uint8_t x = 0;
        if (need(1)) { x = p[off]; off += 1; }
        return x;
    }
    void skip(size_t k) {
        if (need(k)) off += k;
    }
};

struct cipher_span {
    size_t off;       // byte offset of the cipher's |L| field
    uint32_t nL, nE;
};

// Header walk: per-cipher offsets and counts, common nbits. Returns PVAC_OK or an error code.
int walk(const uint8_t* buf, size_t len, std::vector<cipher_span>& spans, uint32_t& nbits, bool& mixed) {
    reader r{buf, len};
    if (r.u32() != kCtMagic || r.u32() != kCtVersion) return PVAC_EINVAL;
    const uint64_t n = r.u64();
    if (!r.ok || n > len / 8) return PVAC_EINVAL;   // every cipher needs >= 8 bytes
    spans.clear();
    spans.reserve((size_t)n);
    nbits = 0;
    mixed = false;
    bool first_edge = true;
    for (uint64_t c = 0; c < n; ++c) {
        cipher_span s{r.off, 0, 0};
        s.nL = r.u32();
        s.nE = r.u32();
        for (uint32_t l = 0; l < s.nL && r.ok; ++l) r.skip(r.u8() == 1 ? kProdBytes : kBaseBytes);
        for (uint32_t e = 0; e < s.nE && r.ok; ++e) {
            r.skip(kEdgeHdr - 4);
            const uint32_t nb = r.u32();
            if (first_edge) { nbits = nb; first_edge = false; }
            else if (nb != nbits) mixed = true;
            r.skip(8 * (size_t)((nb + 63u) / 64u));
        }
        if (!r.ok) return PVAC_EINVAL;
        spans.push_back(s);
    }
    if (r.off != len) return PVAC_EINVAL;   // trailing bytes: not a .ct file of this shape
    return PVAC_OK;
}

template <class F>
void parallel_for(size_t n, int threads, F&& f) {
    unsigned t = threads > 0 ? (unsigned)threads : std::max(1u, std::thread::hardware_concurrency());
    t = (unsigned)std::min<size_t>(t, std::max<size_t>(n, 1));
    if (t <= 1) {
        for (size_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::vector<std::thread> pool;
    pool.reserve(t);
    for (unsigned k = 0; k < t; ++k)
        pool.emplace_back([&, k] {
            for (size_t i = k; i < n; i += t) f(i);
        });
    for (auto& th : pool) th.join();
}

size_t cipher_bytes(const pvac_ct_batch* X, uint64_t i, uint32_t nbits) {
    size_t b = 8;
    const pvac_layer* L = X->layers + X->l_off[i];
    for (uint64_t l = 0; l < X->l_cnt[i]; ++l) b += 1 + (L[l].rule == 1 ? kProdBytes : kBaseBytes);
    b += X->e_cnt[i] * (kEdgeHdr + 8 * (size_t)((nbits + 63u) / 64u));
    return b;
}

}  // namespace

extern "C" {

int pvac_ct_scan(const uint8_t* buf, size_t len, pvac_ct_file_info* info) {
    if (!buf || !info) return PVAC_EINVAL;
    std::vector<cipher_span> spans;
    uint32_t nbits = 0;
    bool mixed = false;
    const int rc = walk(buf, len, spans, nbits, mixed);
    if (rc) return rc;
    std::memset(info, 0, sizeof *info);
    info->n_ciphers = spans.size();
    for (const auto& s : spans) {
        info->total_layers += s.nL;
        info->total_edges += s.nE;
    }
    info->sigma_bits = nbits;
    info->sigma_words = (nbits + 63u) / 64u;
    info->flags = mixed ? PVAC_CT_MIXED_SIGMA : 0u;
    return PVAC_OK;
}

int pvac_ct_parse(const uint8_t* buf, size_t len, pvac_ct_batch* X, int threads) {
    if (!buf || !X) return PVAC_EINVAL;
    std::vector<cipher_span> spans;
    uint32_t nbits = 0;
    bool mixed = false;
    int rc = walk(buf, len, spans, nbits, mixed);
    if (rc) return rc;
    if (mixed) return PVAC_ENOSYS;
    const uint32_t nw = (nbits + 63u) / 64u;
    if (X->n != spans.size() || !X->l_off || !X->l_cnt || !X->e_off || !X->e_cnt) return PVAC_EINVAL;
    if (nw && X->sigma && X->sigma_words < nw) return PVAC_EINVAL;
    // dense CSR offsets
    uint64_t lo = 0, eo = 0;
    for (size_t c = 0; c < spans.size(); ++c) {
        X->l_off[c] = lo;
        X->l_cnt[c] = spans[c].nL;
        X->e_off[c] = eo;
        X->e_cnt[c] = spans[c].nE;
        lo += spans[c].nL;
        eo += spans[c].nE;
    }
    if ((lo && !X->layers) || (eo && (!X->meta || !X->w_lo || !X->w_hi))) return PVAC_EINVAL;
    parallel_for(spans.size(), threads, [&](size_t c) {
        reader r{buf, len, spans[c].off + 8};
        pvac_layer* L = X->layers + X->l_off[c];
        for (uint32_t l = 0; l < spans[c].nL; ++l) {
            pvac_layer y{};
            y.rule = r.u8();
            if (y.rule == 0) {
                y.ztag = r.u64();
                y.nonce_lo = r.u64();
                y.nonce_hi = r.u64();
            } else if (y.rule == 1) {
                y.pa = r.u32();
                y.pb = r.u32();
            } else {
                r.skip(kBaseBytes);
            }
            L[l] = y;
        }
        const uint64_t e0 = X->e_off[c];
        for (uint32_t e = 0; e < spans[c].nE; ++e) {
            const uint64_t lid = r.u32();
            uint16_t idx = 0;
            if (r.need(2)) { std::memcpy(&idx, buf + r.off, 2); r.off += 2; }
            const uint64_t ch = r.u8();
            r.u8();
            X->meta[e0 + e] = lid | ((uint64_t)idx << 32) | (ch << 48);
            X->w_lo[e0 + e] = r.u64();
            X->w_hi[e0 + e] = r.u64();
            r.u32();   // nbits (checked uniform by the walk)
            if (nw && X->sigma) {
                uint64_t* s = X->sigma + (e0 + e) * X->sigma_words;
                if (r.need(8 * (size_t)nw)) { std::memcpy(s, buf + r.off, 8 * (size_t)nw); r.off += 8 * (size_t)nw; }
                for (uint32_t w = nw; w < X->sigma_words; ++w) s[w] = 0;
            } else {
                r.skip(8 * (size_t)nw);
            }
        }
    });
    return PVAC_OK;
}

int pvac_ct_serialized_size(const pvac_ct_batch* X, uint32_t sigma_bits, uint64_t* bytes) {
    if (!X || !bytes) return PVAC_EINVAL;
    const uint32_t nbits = X->sigma ? sigma_bits : 0u;
    if (X->sigma && (nbits + 63u) / 64u > X->sigma_words) return PVAC_EINVAL;
    uint64_t b = 16;
    for (uint64_t i = 0; i < X->n; ++i) b += cipher_bytes(X, i, nbits);
    *bytes = b;
    return PVAC_OK;
}

int pvac_ct_write(const pvac_ct_batch* X, uint32_t sigma_bits, uint8_t* out, size_t cap, uint64_t* written,
                  int threads) {
    if (!X || !out) return PVAC_EINVAL;
    const uint32_t nbits = X->sigma ? sigma_bits : 0u;
    const uint32_t nw = (nbits + 63u) / 64u;
    if (X->sigma && nw > X->sigma_words) return PVAC_EINVAL;
    std::vector<uint64_t> pos(X->n + 1, 0);
    pos[0] = 16;
    for (uint64_t i = 0; i < X->n; ++i) pos[i + 1] = pos[i] + cipher_bytes(X, i, nbits);
    if (pos[X->n] > cap) return PVAC_ERANGE;
    const uint32_t magic = kCtMagic, ver = kCtVersion;
    const uint64_t n = X->n;
    std::memcpy(out, &magic, 4);
    std::memcpy(out + 4, &ver, 4);
    std::memcpy(out + 8, &n, 8);
    parallel_for((size_t)X->n, threads, [&](size_t i) {
        uint8_t* o = out + pos[i];
        auto put = [&](const void* v, size_t k) { std::memcpy(o, v, k); o += k; };
        const uint32_t nL = (uint32_t)X->l_cnt[i], nE = (uint32_t)X->e_cnt[i];
        put(&nL, 4);
        put(&nE, 4);
        const pvac_layer* L = X->layers + X->l_off[i];
        for (uint32_t l = 0; l < nL; ++l) {
            const uint8_t rule = (uint8_t)L[l].rule;
            put(&rule, 1);
            if (rule == 0) {
                put(&L[l].ztag, 8);
                put(&L[l].nonce_lo, 8);
                put(&L[l].nonce_hi, 8);
            } else if (rule == 1) {
                put(&L[l].pa, 4);
                put(&L[l].pb, 4);
            } else {
                std::memset(o, 0, kBaseBytes);
                o += kBaseBytes;
            }
        }
        const uint64_t e0 = X->e_off[i];
        for (uint32_t e = 0; e < nE; ++e) {
            const uint64_t m = X->meta[e0 + e];
            const uint32_t lid = (uint32_t)m;
            const uint16_t idx = (uint16_t)(m >> 32);
            const uint8_t ch = (uint8_t)(m >> 48), zero = 0;
            put(&lid, 4);
            put(&idx, 2);
            put(&ch, 1);
            put(&zero, 1);
            put(&X->w_lo[e0 + e], 8);
            put(&X->w_hi[e0 + e], 8);
            put(&nbits, 4);
            if (nw) put(X->sigma + (e0 + e) * X->sigma_words, 8 * (size_t)nw);
        }
    });
    if (written) *written = pos[X->n];
    return PVAC_OK;
}

}  // extern "C"
