// test_adapter.cpp — the C++ drop-in adapter (include/pvac_hip.hpp) driven the way reference code
// calls the by-value API (tests/test_main.cpp:172-313 style), on types that mirror the reference's
// field layout (include/pvac/core/types.hpp:72-139), checked against the golden fixtures minted by
// the unmodified reference (tests/golden/ref, tests/golden/bounty). Runs on the GPU box:
//   test_adapter <golden_dir> <canon_tag> <H_digest_hex>
// Exit 0 = every check passed; failures abort with a message (like the reference's must()).
//   test_adapter --time <pairs>   end-to-end (host ciphers in and out) ct_mul rate, JSON
#include <algorithm>
#include <array>
#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <vector>

#include "pvac_hip.hpp"

namespace mirror {   // same member names/types as pvac:: (core/types.hpp, core/field.hpp, core/bitvec.hpp)
struct Fp { uint64_t lo, hi; };
struct BitVec { size_t nbits = 0; std::vector<uint64_t> w; };
struct Nonce128 { uint64_t lo, hi; };
struct RSeed { uint64_t ztag; Nonce128 nonce; };
enum class RRule : uint8_t { BASE = 0, PROD = 1 };
struct Layer { RRule rule; RSeed seed; uint32_t pa; uint32_t pb; };
struct Edge { uint32_t layer_id; uint16_t idx; uint8_t ch; Fp w; BitVec s; };
struct Cipher { std::vector<Layer> L; std::vector<Edge> E; };
struct Params {
    int B = 337, m_bits = 8192, n_bits = 16384, h_col_wt = 192, x_col_wt = 128, err_wt = 128;
    double noise_entropy_bits = 120.0, tuple2_fraction = 0.55, depth_slope_bits = 16.0;
    size_t edge_budget = 1200000;
    int lpn_n = 4096, lpn_t = 16384, lpn_tau_num = 1, lpn_tau_den = 8;
};
struct PubKey {
    Params prm; uint64_t canon_tag = 0; std::vector<BitVec> H;
    std::array<uint8_t, 32> H_digest{}; std::vector<Fp> powg_B;
};
struct SecKey { std::array<uint64_t, 4> prf_k{}; std::vector<uint64_t> lpn_s_bits; };
}  // namespace mirror

using mirror::Cipher;

static int g_checks = 0;
#define MUST(cond, ...)                                                        \
    do {                                                                       \
        ++g_checks;                                                            \
        if (!(cond)) {                                                         \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);          \
            std::fprintf(stderr, __VA_ARGS__);                                 \
            std::fprintf(stderr, "\n");                                        \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

// ---- .ct codec (format of the reference's tests/add.cpp:22-155; our own reader/writer)
static std::vector<uint8_t> slurp(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    MUST(f.good(), "open %s", p.c_str());
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

struct reader {
    const std::vector<uint8_t>& b;
    size_t o = 0;
    template <class T> T get() {
        T v;
        MUST(o + sizeof(T) <= b.size(), "truncated .ct");
        std::memcpy(&v, &b[o], sizeof(T));
        o += sizeof(T);
        return v;
    }
};

static std::vector<Cipher> read_ct(const std::string& path) {
    const auto buf = slurp(path);
    reader r{buf};
    MUST(r.get<uint32_t>() == 0x66699666u && r.get<uint32_t>() == 1u, "bad .ct header %s", path.c_str());
    const uint64_t n = r.get<uint64_t>();
    std::vector<Cipher> out(n);
    for (auto& c : out) {
        const uint32_t nL = r.get<uint32_t>(), nE = r.get<uint32_t>();
        c.L.resize(nL);
        for (auto& L : c.L) {
            L = mirror::Layer{};
            L.rule = (mirror::RRule)r.get<uint8_t>();
            if (L.rule == mirror::RRule::BASE) {
                L.seed.ztag = r.get<uint64_t>();
                L.seed.nonce.lo = r.get<uint64_t>();
                L.seed.nonce.hi = r.get<uint64_t>();
            } else if (L.rule == mirror::RRule::PROD) {
                L.pa = r.get<uint32_t>();
                L.pb = r.get<uint32_t>();
            } else {
                r.o += 24;
            }
        }
        c.E.resize(nE);
        for (auto& E : c.E) {
            E.layer_id = r.get<uint32_t>();
            E.idx = r.get<uint16_t>();
            E.ch = r.get<uint8_t>();
            (void)r.get<uint8_t>();
            E.w.lo = r.get<uint64_t>();
            E.w.hi = r.get<uint64_t>();
            E.s.nbits = r.get<uint32_t>();
            E.s.w.resize((E.s.nbits + 63) / 64);
            for (auto& w : E.s.w) w = r.get<uint64_t>();
        }
    }
    MUST(r.o == buf.size(), "trailing bytes in %s", path.c_str());
    return out;
}

template <class T>
static void put(std::vector<uint8_t>& o, T v) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
    o.insert(o.end(), p, p + sizeof(T));
}

static std::vector<uint8_t> write_ct(const std::vector<Cipher>& cs) {
    std::vector<uint8_t> o;
    put<uint32_t>(o, 0x66699666u);
    put<uint32_t>(o, 1u);
    put<uint64_t>(o, cs.size());
    for (const auto& c : cs) {
        put<uint32_t>(o, (uint32_t)c.L.size());
        put<uint32_t>(o, (uint32_t)c.E.size());
        for (const auto& L : c.L) {
            put<uint8_t>(o, (uint8_t)L.rule);
            if (L.rule == mirror::RRule::BASE) {
                put(o, L.seed.ztag); put(o, L.seed.nonce.lo); put(o, L.seed.nonce.hi);
            } else {
                put(o, L.pa); put(o, L.pb);
            }
        }
        for (const auto& E : c.E) {
            put(o, E.layer_id); put(o, E.idx); put(o, E.ch); put<uint8_t>(o, 0);
            put(o, E.w.lo); put(o, E.w.hi);
            put<uint32_t>(o, (uint32_t)E.s.nbits);
            for (uint64_t w : E.s.w) put(o, w);
        }
    }
    return o;
}

static std::vector<uint64_t> read_u64(const std::string& p) {
    const auto b = slurp(p);
    std::vector<uint64_t> v(b.size() / 8);
    std::memcpy(v.data(), b.data(), v.size() * 8);
    return v;
}

// every "[a, b]" pair that follows an occurrence of `key` in a manifest's text (the harness writes them)
static std::vector<std::pair<size_t, size_t>> json_pairs(const std::string& js, const std::string& key) {
    std::vector<std::pair<size_t, size_t>> out;
    for (size_t at = js.find(key); at != std::string::npos; at = js.find(key, at + 1)) {
        const size_t lb = js.find('[', at);
        char* e = nullptr;
        const size_t a = std::strtoull(js.c_str() + lb + 1, &e, 10);
        const size_t b = std::strtoull(e + 1, nullptr, 10);
        out.emplace_back(a, b);
    }
    return out;
}

// A .ct keeps BASE seeds and PROD parents only: project a full cipher the same way.
static Cipher ct_view(Cipher c) {
    for (auto& L : c.L) {
        if (L.rule == mirror::RRule::PROD) L.seed = mirror::RSeed{};
        else { L.pa = 0; L.pb = 0; }
    }
    return c;
}

static bool same_edges(const Cipher& a, const Cipher& b, bool sigma) {
    if (a.E.size() != b.E.size()) return false;
    for (size_t i = 0; i < a.E.size(); ++i) {
        const auto &x = a.E[i], &y = b.E[i];
        if (x.layer_id != y.layer_id || x.idx != y.idx || x.ch != y.ch || x.w.lo != y.w.lo || x.w.hi != y.w.hi)
            return false;
        if (sigma && x.s.w != y.s.w) return false;
    }
    return true;
}

static bool same_layers(const Cipher& a, const Cipher& b) {
    if (a.L.size() != b.L.size()) return false;
    for (size_t i = 0; i < a.L.size(); ++i) {
        const auto &x = a.L[i], &y = b.L[i];
        if (x.rule != y.rule || x.pa != y.pa || x.pb != y.pb || x.seed.ztag != y.seed.ztag ||
            x.seed.nonce.lo != y.seed.nonce.lo || x.seed.nonce.hi != y.seed.nonce.hi)
            return false;
    }
    return true;
}

// replays a reference random stream (nonces, then salts) like the harness' getrandom log
struct replay {
    std::vector<uint64_t> s;
    size_t k = 0;
    uint64_t operator()() {
        MUST(k < s.size(), "random stream exhausted");
        return s[k++];
    }
};

// FIPS 180-4 SHA-256 (test side only: per-edge sigma digests of the fixtures, first 8 bytes LE of the
// hash of the sigma words as little-endian bytes, as the harness's sigma_digests writes them)
static uint64_t sigma_digest(const std::vector<uint64_t>& words) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
        0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
        0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
        0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
        0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
        0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
        0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
        0xc67178f2};
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    std::vector<uint8_t> m(words.size() * 8);
    for (size_t i = 0; i < words.size(); ++i)
        for (int b = 0; b < 8; ++b) m[8 * i + b] = (uint8_t)(words[i] >> (8 * b));
    const uint64_t bits = (uint64_t)m.size() * 8;
    m.push_back(0x80);
    while (m.size() % 64 != 56) m.push_back(0);
    for (int b = 7; b >= 0; --b) m.push_back((uint8_t)(bits >> (8 * b)));
    auto rotr = [](uint32_t x, int r) { return (x >> r) | (x << (32 - r)); };
    for (size_t o = 0; o < m.size(); o += 64) {
        uint32_t w[64];
        for (int t = 0; t < 16; ++t)
            w[t] = (uint32_t)m[o + 4 * t] << 24 | (uint32_t)m[o + 4 * t + 1] << 16 | (uint32_t)m[o + 4 * t + 2] << 8 |
                   m[o + 4 * t + 3];
        for (int t = 16; t < 64; ++t)
            w[t] = (rotr(w[t - 2], 17) ^ rotr(w[t - 2], 19) ^ (w[t - 2] >> 10)) + w[t - 7] +
                   (rotr(w[t - 15], 7) ^ rotr(w[t - 15], 18) ^ (w[t - 15] >> 3)) + w[t - 16];
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int t = 0; t < 64; ++t) {
            const uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[t] + w[t];
            const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    }
    uint64_t r = 0;   // digest bytes 0..7, read little-endian
    for (int b = 0; b < 8; ++b) r |= (uint64_t)(uint8_t)(h[b / 4] >> (24 - 8 * (b % 4))) << (8 * b);
    return r;
}

// a seeded splitmix64 word source (reproducible randomness for the multi-device comparisons)
static pvac_hip::RandomSource os_splitmix(uint64_t seed) {
    auto st = std::make_shared<uint64_t>(seed);
    return [st] {
        uint64_t z = (*st += 0x9e3779b97f4a7c15ULL);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
        return z ^ (z >> 31);
    };
}

// replays an enc_value getrandom log; the adapter draws a whole stride per value, so reads
// past the log return 0 (they are never consumed by the kernels) and are counted
struct replay_pad {
    std::vector<uint64_t> s;
    size_t k = 0;
    uint64_t operator()() { return k < s.size() ? s[k++] : (++k, 0ull); }
};

// --time <pairs>: end-to-end rate of the by-value batched ct_mul (weights only) on host ciphers
// shaped like enc_value output (2 BASE layers x 20 distinct (idx, ch) edges): AoS -> SoA, H2D,
// plan + exec, D2H, SoA -> AoS all inside the timed region. Prints one JSON line.
static int time_host_roundtrip(size_t n) {
    uint64_t st = 0x5EED0006;
    auto rnd = [&]() {
        uint64_t z = (st += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    auto fresh = [&]() {
        Cipher c;
        c.L.resize(2);
        for (auto& l : c.L) { l.rule = mirror::RRule::BASE; l.seed.ztag = rnd(); l.seed.nonce = {rnd(), rnd()}; l.pa = l.pb = 0; }
        for (uint32_t la = 0; la < 2; ++la) {
            std::vector<uint32_t> used;
            while (used.size() < 20) {
                const uint32_t k = (uint32_t)(rnd() % (2 * 337));
                bool dup = false;
                for (uint32_t u : used) dup |= u == k;
                if (dup) continue;
                used.push_back(k);
                mirror::Edge e{};
                e.layer_id = la; e.idx = (uint16_t)(k >> 1); e.ch = (uint8_t)(k & 1);
                e.w = mirror::Fp{rnd(), rnd() & 0x7FFFFFFFFFFFFFFFull};
                c.E.push_back(e);
            }
        }
        return c;
    };
    std::vector<Cipher> A(n), B(n);
    for (size_t i = 0; i < n; ++i) { A[i] = fresh(); B[i] = fresh(); }
    mirror::PubKey pk;
    pk.canon_tag = 0x5EED0006;
    auto src = [&]() { return rnd(); };
    (void)pvac_hip::ct_mul_batch(pk, A, B, false, src);   // warm-up (allocations, code objects)
    const auto t0 = std::chrono::steady_clock::now();
    const auto C = pvac_hip::ct_mul_batch(pk, A, B, false, src);
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    size_t edges = 0;
    for (const auto& c : C) edges += c.E.size();
    const auto& ph = pvac_hip::engine_for(pk).last_phases();
    std::printf("{\"pairs\": %zu, \"seconds\": %.6f, \"ct_mul_per_s\": %.1f, \"output_edges\": %zu, "
                "\"phases_s\": {\"to_soa\": %.4f, \"h2d\": %.4f, \"plan\": %.4f, \"exec\": %.4f, \"d2h\": %.4f, "
                "\"to_aos\": %.4f}}\n",
                n, sec, n / sec, edges, ph.to_soa, ph.h2d, ph.plan, ph.exec, ph.d2h, ph.to_aos);
    return 0;
}

// --time-single <calls>: latency of ONE by-value drop-in call pvac_hip::ct_mul(pk, A, B) WITH sigma
// (the reference's full ct_mul, ops/arithmetic.hpp:47-106, as tests/test_main.cpp:178-188 and the
// chain at :291-292 call it: one pair at a time, host ciphers in and out, getrandom nonces and
// salts), on fresh x fresh and on chain step 3 x fresh (c_3 = ((x x) x) x). Prints one JSON line
// with p50 / p99 / mean per call in ms.
static int time_single(size_t calls) {
    uint64_t st = 0x5EED0007;
    auto rnd = [&]() {
        uint64_t z = (st += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    auto fresh = [&]() {
        Cipher c;
        c.L.resize(2);
        for (auto& l : c.L) { l.rule = mirror::RRule::BASE; l.seed.ztag = rnd(); l.seed.nonce = {rnd(), rnd()}; l.pa = l.pb = 0; }
        for (uint32_t la = 0; la < 2; ++la) {
            std::vector<uint32_t> used;
            while (used.size() < 20) {
                const uint32_t k = (uint32_t)(rnd() % (2 * 337));
                bool dup = false;
                for (uint32_t u : used) dup |= u == k;
                if (dup) continue;
                used.push_back(k);
                mirror::Edge e{};
                e.layer_id = la; e.idx = (uint16_t)(k >> 1); e.ch = (uint8_t)(k & 1);
                e.w = mirror::Fp{rnd(), rnd() & 0x7FFFFFFFFFFFFFFFull};
                e.s.nbits = 8192;
                e.s.w.assign(128, rnd());
                c.E.push_back(e);
            }
        }
        return c;
    };
    mirror::PubKey pk;   // empty pk.H: regenerated on the device from canon_tag (pvac_hip_ctx_gen_H)
    pk.canon_tag = 0x5EED0007;
    auto src = [&]() { return rnd(); };
    auto pct = [](std::vector<double> v, double q) {
        std::sort(v.begin(), v.end());
        return v[std::min(v.size() - 1, (size_t)(q * (v.size() - 1) + 0.5))];
    };
    auto run = [&](const Cipher& a, const Cipher& b, size_t k, size_t& edges) {
        std::vector<double> ms;
        (void)pvac_hip::ct_mul(pk, a, b, src);   // warm-up: H, code objects, allocations
        for (size_t i = 0; i < k; ++i) {
            const auto t0 = std::chrono::steady_clock::now();
            const Cipher c = pvac_hip::ct_mul(pk, a, b, src);
            ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
            edges = c.E.size();
            MUST(!c.E.empty() && c.E[0].s.w.size() == 128, "sigma missing");
        }
        double mean = 0;
        for (double x : ms) mean += x;
        return std::array<double, 3>{pct(ms, 0.5), pct(ms, 0.99), mean / ms.size()};
    };
    const Cipher x = fresh(), y = fresh();
    size_t e1 = 0, e2 = 0;
    const auto f = run(x, y, calls, e1);
    Cipher c = x;   // chain c_k = c_{k-1} * x (tests/test_main.cpp:291-292)
    for (int k = 0; k < 3; ++k) c = pvac_hip::ct_mul(pk, c, x, src);
    const auto g = run(c, x, std::max<size_t>(calls / 5, 5), e2);
    std::printf("{\"fresh_x_fresh\": {\"calls\": %zu, \"p50_ms\": %.4f, \"p99_ms\": %.4f, \"mean_ms\": %.4f, "
                "\"output_edges\": %zu}, \"chain3_x_fresh\": {\"calls\": %zu, \"input_edges\": %zu, \"p50_ms\": %.4f, "
                "\"p99_ms\": %.4f, \"mean_ms\": %.4f, \"output_edges\": %zu}}\n",
                calls, f[0], f[1], f[2], e1, std::max<size_t>(calls / 5, 5), c.E.size(), g[0], g[1], g[2], e2);
    return 0;
}

int main(int argc, char** argv) {
    if (argc == 3 && std::string(argv[1]) == "--time") return time_host_roundtrip(std::strtoull(argv[2], nullptr, 10));
    if (argc == 3 && std::string(argv[1]) == "--time-single") return time_single(std::strtoull(argv[2], nullptr, 10));
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s <golden_dir> <canon_tag> <H_digest_hex> <v0,v1,...>\n", argv[0]);
        return 2;
    }
    const std::string gold = argv[1], ref = gold + "/ref", bounty = gold + "/bounty";
    mirror::PubKey pk;
    pk.canon_tag = std::strtoull(argv[2], nullptr, 10);
    const std::string hdig = argv[3];

    // H regenerated on the device from canon_tag matches the reference key's H_digest
    auto& eng = pvac_hip::engine_for(pk);
    const auto d = eng.gen_H();
    char hex[65];
    for (int i = 0; i < 32; ++i) std::snprintf(hex + 2 * i, 3, "%02x", d[i]);
    MUST(hdig == hex, "H_digest %s != %s", hex, hdig.c_str());

    // ct_add / ct_sub (ops/arithmetic.hpp:12-45) on the 8 golden pairs, sigmas carried
    for (int p = 0; p < 8; ++p) {
        const Cipher x = read_ct(ref + "/pair" + std::to_string(p) + "_x.ct")[0];
        const Cipher y = read_ct(ref + "/pair" + std::to_string(p) + "_y.ct")[0];
        const Cipher s = pvac_hip::ct_add(pk, x, y);
        const Cipher r_add = read_ct(ref + "/pair" + std::to_string(p) + "_add.ct")[0];
        MUST(same_layers(ct_view(s), r_add) && same_edges(s, r_add, true), "ct_add pair %d", p);
        const Cipher dlt = pvac_hip::ct_sub(pk, x, y);
        const Cipher r_sub = read_ct(ref + "/pair" + std::to_string(p) + "_sub.ct")[0];
        MUST(same_layers(ct_view(dlt), r_sub) && same_edges(dlt, r_sub, true), "ct_sub pair %d", p);
        // ct_scale by p-1 (= ct_neg, arithmetic.hpp:39-41) gives the B half of ct_sub
        const Cipher ny = pvac_hip::ct_scale(pk, y, mirror::Fp{~0ull - 1, 0x7FFFFFFFFFFFFFFFull});
        for (size_t e = 0; e < ny.E.size(); ++e) {
            const auto& want = r_sub.E[x.E.size() + e].w;
            MUST(ny.E[e].w.lo == want.lo && ny.E[e].w.hi == want.hi, "ct_scale pair %d edge %zu", p, e);
        }
        // ct_neg (arithmetic.hpp:39-41) is that same scale; layers and sigmas are y's
        const Cipher ng = pvac_hip::ct_neg(pk, y);
        MUST(same_layers(ng, y) && ng.E.size() == y.E.size(), "ct_neg pair %d shape", p);
        for (size_t e = 0; e < ng.E.size(); ++e) {
            const auto& want = r_sub.E[x.E.size() + e];
            MUST(ng.E[e].w.lo == want.w.lo && ng.E[e].w.hi == want.w.hi && ng.E[e].s.w == y.E[e].s.w,
                 "ct_neg pair %d edge %zu", p, e);
        }
        // ct_div_const (arithmetic.hpp:108-110): dividing by k then scaling by k gives x back
        // (canonical weights); k = 2 has the known inverse (p + 1) / 2 = 2^126
        const mirror::Fp ks[3] = {{2, 0}, {0x0123456789ABCDEFull, 0x0FEDCBA987654321ull}, {~0ull - 1, 0x7FFFFFFFFFFFFFFFull}};
        for (const auto& k : ks) {
            const Cipher q = pvac_hip::ct_div_const(pk, x, k);
            const Cipher back = pvac_hip::ct_scale(pk, q, k);
            MUST(same_layers(back, x) && same_edges(back, x, true), "ct_div_const pair %d k.lo %" PRIx64, p, k.lo);
        }
        const Cipher h = pvac_hip::ct_div_const(pk, x, mirror::Fp{2, 0});
        const Cipher h2 = pvac_hip::ct_scale(pk, x, mirror::Fp{0, 0x4000000000000000ull});
        MUST(same_edges(h, h2, true), "ct_div_const by 2 == ct_scale by 2^126, pair %d", p);
    }

    // bounty2_data: sum.ct == combine(a.ct, b.ct) byte for byte through the adapter
    {
        const Cipher a = read_ct(bounty + "/a.ct")[0], b = read_ct(bounty + "/b.ct")[0];
        const Cipher s = pvac_hip::ct_add(pk, a, b);
        MUST(write_ct({ct_view(s)}) == slurp(bounty + "/sum.ct"), "bounty2 sum.ct bytes");
    }

    // full ct_mul with sigma (ops/arithmetic.hpp:47-106): pair 0 byte-identical to the reference
    {
        const Cipher x = read_ct(ref + "/pair0_x.ct")[0], y = read_ct(ref + "/pair0_y.ct")[0];
        replay rs{read_u64(ref + "/pair0_mul_stream.u64")};
        const Cipher m = pvac_hip::ct_mul(pk, x, y, std::ref(rs));
        const Cipher r = read_ct(ref + "/pair0_mul.ct")[0];
        MUST(rs.k == rs.s.size(), "ct_mul consumed %zu of %zu random words", rs.k, rs.s.size());
        MUST(same_layers(ct_view(m), r) && same_edges(m, r, true), "ct_mul pair 0 (with sigma)");
        MUST(write_ct({ct_view(m)}) == slurp(ref + "/pair0_mul.ct"), "ct_mul pair 0 .ct bytes");
    }

    // chain c_k = c_{k-1} * x_k (tests/test_main.cpp:289-295), weights and order, steps 1..3
    {
        const auto lay = [&](int k) {
            const auto v = read_u64(ref + "/chain" + std::to_string(k) + "_layers.u64");
            std::vector<mirror::Layer> L(v.size() / 6);
            for (size_t i = 0; i < L.size(); ++i) {
                L[i].rule = (mirror::RRule)v[6 * i];
                L[i].pa = (uint32_t)v[6 * i + 1]; L[i].pb = (uint32_t)v[6 * i + 2];
                L[i].seed.ztag = v[6 * i + 3]; L[i].seed.nonce.lo = v[6 * i + 4]; L[i].seed.nonce.hi = v[6 * i + 5];
            }
            return L;
        };
        Cipher cur = read_ct(ref + "/chain0.ct")[0];
        for (int k = 1; k <= 3; ++k) {
            const Cipher x = read_ct(ref + "/chain" + std::to_string(k) + "_x.ct")[0];
            replay rs{read_u64(ref + "/chain" + std::to_string(k) + "_stream.u64")};
            std::vector<Cipher> A{cur}, B{x};
            const Cipher c = pvac_hip::ct_mul_batch(pk, A, B, false, std::ref(rs))[0];
            const Cipher r = read_ct(ref + "/chain" + std::to_string(k) + ".ct")[0];
            MUST(same_layers(ct_view(c), r) && same_edges(c, r, false), "chain step %d", k);
            const auto full = lay(k);
            MUST(c.L.size() == full.size(), "chain step %d layers", k);
            for (size_t l = 0; l < full.size(); ++l) MUST(c.L[l].seed.ztag == full[l].seed.ztag, "ztag %zu", l);
            cur = c;
        }
    }

    // the chain entry point (pvac_hip_ct_mul_chain) with a final-step WITH_SIGMA, replaying the
    // reference's stream of c_k = ct_mul(c_{k-1}, x), k = 1..4 (harness cmd_chainx): every step's
    // nonces placed, the intermediate salts skipped, the final salts placed; c_4 byte-identical
    // (weights-only .ct, full layer table) and every sigma's digest equal to the reference's
    {
        const Cipher x = read_ct(ref + "/chainx_x.ct")[0];
        const auto stream = read_u64(ref + "/chainx_stream.u64");
        auto rp = std::make_shared<replay>(replay{stream});
        std::vector<pvac_hip::RandomSource> rnds{[rp] { return (*rp)(); }};
        const Cipher c = pvac_hip::ct_mul_chain(pk, std::vector<Cipher>{x}, 4, true, rnds)[0];
        MUST(rp->k == stream.size(), "chain consumed %zu of %zu random words", rp->k, stream.size());
        Cipher w = c;
        for (auto& E : w.E) E.s = mirror::BitVec{};   // the fixture is the weights-only .ct
        MUST(write_ct({w}) == slurp(ref + "/chainx_final.ct"), "chainx c_4 weights .ct bytes");
        const auto lay = read_u64(ref + "/chainx_final_layers.u64");
        MUST(c.L.size() * 6 == lay.size(), "chainx layers %zu", c.L.size());
        for (size_t l = 0; l < c.L.size(); ++l)
            MUST((uint64_t)c.L[l].rule == lay[6 * l] && c.L[l].seed.ztag == lay[6 * l + 3] &&
                     c.L[l].seed.nonce.lo == lay[6 * l + 4] && c.L[l].seed.nonce.hi == lay[6 * l + 5],
                 "chainx layer %zu", l);
        const auto dig = read_u64(ref + "/chainx_final_sigdig.u64");
        MUST(dig.size() == c.E.size(), "chainx sigma digests");
        for (size_t e = 0; e < c.E.size(); ++e) MUST(sigma_digest(c.E[e].s.w) == dig[e], "chainx sigma %zu", e);
        // two device ranges on this GPU (devices {0, 0}): the same bytes and sigmas
        auto rp2 = std::make_shared<replay>(replay{stream});
        std::vector<Cipher> xs{x, x, x};
        std::vector<pvac_hip::RandomSource> r3{[rp2] { return (*rp2)(); }, os_splitmix(11), os_splitmix(12)};
        const auto c3 = pvac_hip::ct_mul_chain(pk, xs, 4, true, r3, std::vector<int>{0, 0});
        MUST(write_ct({ct_view(c3[0])}) == write_ct({ct_view(c)}) && same_edges(c3[0], c, true), "chain 2-range c_4");
        MUST(same_edges(c3[1], c3[2], false) && same_edges(c3[1], c, false), "chain 2-range weights");
    }

    // multi-device batch ct_mul (devices {0, 0}: two ranges, two contexts, one GPU) with sigma from one
    // seeded source: the bytes of the one-device batch (draw order preserved)
    {
        std::vector<Cipher> A, B;
        for (int p = 0; p < 8; ++p) {
            A.push_back(read_ct(ref + "/pair" + std::to_string(p) + "_x.ct")[0]);
            B.push_back(read_ct(ref + "/pair" + std::to_string(p) + "_y.ct")[0]);
        }
        const auto one = pvac_hip::ct_mul_batch(pk, A, B, true, os_splitmix(7), std::vector<int>{});
        const auto two = pvac_hip::ct_mul_batch(pk, A, B, true, os_splitmix(7), std::vector<int>{0, 0});
        const auto three = pvac_hip::ct_mul_batch(pk, A, B, true, os_splitmix(7), std::vector<int>{0, 0, 0});
        MUST(one.size() == 8 && two.size() == 8 && three.size() == 8, "multi-device batch sizes");
        for (int p = 0; p < 8; ++p)
            MUST(write_ct({ct_view(one[p])}) == write_ct({ct_view(two[p])}) && same_edges(one[p], two[p], true) &&
                     same_edges(one[p], three[p], true),
                 "multi-device batch pair %d", p);
        // the engine's kept arrays handed back, then grown again: the same bytes; and a batch of
        // one pair after the 8-pair one (the kept arrays larger than needed) equals its own pair
        pvac_hip::engine_for(pk).trim();
        const auto again = pvac_hip::ct_mul_batch(pk, A, B, true, os_splitmix(7), std::vector<int>{});
        for (int p = 0; p < 8; ++p)
            MUST(write_ct({ct_view(one[p])}) == write_ct({ct_view(again[p])}) && same_edges(one[p], again[p], true),
                 "batch after trim, pair %d", p);
        // (edges and weights do not depend on the random source, only layer nonces and sigmas do)
        const std::vector<Cipher> A1{A[3]}, B1{B[3]};
        const auto solo = pvac_hip::ct_mul_batch(pk, A1, B1, false, os_splitmix(9), std::vector<int>{});
        MUST(solo.size() == 1 && same_edges(solo[0], one[3], false), "one-pair batch on grown arrays");
    }

    // fp_binop through the adapter on the golden vectors (core/field.hpp:50-213)
    {
        const auto alo = read_u64(ref + "/fp_a_lo.u64"), ahi = read_u64(ref + "/fp_a_hi.u64");
        const auto blo = read_u64(ref + "/fp_b_lo.u64"), bhi = read_u64(ref + "/fp_b_hi.u64");
        const size_t n = alo.size();
        std::vector<uint64_t> lo(n), hi(n);
        const std::pair<int, const char*> ops[] = {{PVAC_FP_ADD, "add"}, {PVAC_FP_SUB, "sub"}, {PVAC_FP_MUL, "mul"}};
        for (const auto& op : ops) {
            eng.fp_binop(op.first, alo.data(), ahi.data(), blo.data(), bhi.data(), lo.data(), hi.data(), n);
            MUST(lo == read_u64(ref + "/fp_" + op.second + "_lo.u64") && hi == read_u64(ref + "/fp_" + op.second + "_hi.u64"),
                 "fp_%s", op.second);
        }
    }

    // enc_value / dec_value (ops/encrypt.hpp:289, ops/decrypt.hpp:62) replaying the getrandom
    // streams the reference consumed (harness cmd_enc): byte-identical .ct, decrypts to v
    {
        for (int i = 0; i < 32; ++i) pk.H_digest[i] = (uint8_t)std::strtoul(hdig.substr(2 * i, 2).c_str(), nullptr, 16);
        const auto pg = read_u64(ref + "/powg_B.u64");
        for (size_t i = 0; i + 1 < pg.size(); i += 2) pk.powg_B.push_back(mirror::Fp{pg[i], pg[i + 1]});
        mirror::SecKey sk;
        const auto kk = read_u64(ref + "/sk_prf_k.u64");
        MUST(kk.size() == 4, "sk_prf_k.u64");
        for (int i = 0; i < 4; ++i) sk.prf_k[i] = kk[i];
        sk.lpn_s_bits = read_u64(ref + "/sk_lpn_s.u64");
        std::vector<uint64_t> vs;
        for (const char* p = argv[4]; *p;) {
            char* e = nullptr;
            vs.push_back(std::strtoull(p, &e, 10));
            p = *e ? e + 1 : e;
        }
        MUST(!vs.empty(), "no enc values");
        for (size_t i = 0; i < vs.size(); ++i) {
            replay_pad rs{read_u64(ref + "/enc" + std::to_string(i) + "_stream.u64")};
            const Cipher c = pvac_hip::enc_value<Cipher>(pk, sk, vs[i], std::ref(rs));
            MUST(rs.k >= rs.s.size(), "enc %zu consumed %zu of %zu words", i, rs.k, rs.s.size());
            MUST(write_ct({c}) == slurp(ref + "/enc" + std::to_string(i) + ".ct"), "enc_value %zu .ct bytes", i);
            const auto m = pvac_hip::dec_value(pk, sk, c);
            MUST(m.lo == vs[i] && m.hi == 0, "dec_value(enc %zu)", i);
        }
        // enc_value_depth / enc_zero_depth (encrypt.hpp:281-298) from the harness's encdepth streams:
        // argv[5] = "kind:v:depth,..." (kind 0 value, 1 zero), case i replays encd<i>_stream.u64
        if (argc > 5) {
            size_t i = 0;
            for (const char* p = argv[5]; *p; ++i) {
                char* e = nullptr;
                const unsigned long kind = std::strtoul(p, &e, 10);
                const unsigned long long v = std::strtoull(e + 1, &e, 10);
                const int d = (int)std::strtol(e + 1, &e, 10);
                p = *e ? e + 1 : e;
                const std::string base = ref + "/encd" + std::to_string(i);
                replay_pad rs{read_u64(base + "_stream.u64")};
                const Cipher c = kind ? pvac_hip::enc_zero_depth<Cipher>(pk, sk, d, std::ref(rs))
                                      : pvac_hip::enc_value_depth<Cipher>(pk, sk, v, d, std::ref(rs));
                MUST(rs.k >= rs.s.size(), "encd %zu consumed %zu of %zu words", i, rs.k, rs.s.size());
                MUST(write_ct({c}) == slurp(base + ".ct"), "enc depth case %zu .ct bytes", i);
                MUST(pvac_hip::dec_value(pk, sk, c).lo == v, "dec_value(enc depth case %zu)", i);
            }
            MUST(i > 0, "no enc depth cases");
        }
        // the reference's own chain loop (tests/test_main.cpp:289-293, harness cmd_chainf): chain =
        // enc_value(2), then chain = ct_mul(chain, enc_value(2)) with a FRESH operand per step, depth 4,
        // replayed from its one interleaved stream (enc, mul, enc, mul, ...): (a) by value, the loop as
        // the reference writes it (enc_value, then ct_mul with sigmas, step by step); (b) through the
        // chain entry point with per-step operands (rnds carry the mul stretches only). Both give c_4
        // byte-identical to the reference's (weights-only .ct, layer table, every sigma's digest).
        {
            const auto mb = slurp(ref + "/chainf_manifest.json");
            const std::string man(mb.begin(), mb.end());
            const auto stream = read_u64(ref + "/chainf_stream.u64");
            const auto xst = json_pairs(man, "\"x_stream\"");
            const auto encs = json_pairs(man, "\"enc_stream\""), muls = json_pairs(man, "\"mul_stream\"");
            MUST(xst.size() == 1 && encs.size() == 4 && muls.size() == 4, "chainf manifest");
            auto weights = [](Cipher c) {   // the fixture files are weights-only .ct
                for (auto& E : c.E) E.s = mirror::BitVec{};
                return ct_view(c);
            };
            auto stretch = [&](std::pair<size_t, size_t> p) {
                MUST(p.first + p.second <= stream.size(), "chainf stretch");
                return std::vector<uint64_t>(stream.begin() + (long)p.first, stream.begin() + (long)(p.first + p.second));
            };
            replay_pad rx{stretch(xst[0])};
            const Cipher x = pvac_hip::enc_value<Cipher>(pk, sk, 2, std::ref(rx));
            MUST(write_ct({weights(x)}) == slurp(ref + "/chainf_x.ct"), "chainf x .ct bytes");
            Cipher c = x;
            std::vector<std::vector<Cipher>> ys;
            std::vector<uint64_t> mul_words;
            for (size_t k = 0; k < 4; ++k) {
                replay_pad ry{stretch(encs[k])};
                const Cipher y = pvac_hip::enc_value<Cipher>(pk, sk, 2, std::ref(ry));
                MUST(write_ct({weights(y)}) == slurp(ref + "/chainf_y" + std::to_string(k + 1) + ".ct"), "chainf y%zu", k + 1);
                ys.push_back({y});
                replay rm{stretch(muls[k])};
                c = pvac_hip::ct_mul(pk, c, y, std::ref(rm));
                MUST(rm.k == rm.s.size(), "chainf step %zu consumed %zu of %zu words", k + 1, rm.k, rm.s.size());
                mul_words.insert(mul_words.end(), rm.s.begin(), rm.s.end());
            }
            MUST(write_ct({weights(c)}) == slurp(ref + "/chainf_final.ct"), "chainf c_4 weights .ct bytes (by value)");
            const auto lay = read_u64(ref + "/chainf_final_layers.u64");
            MUST(c.L.size() * 6 == lay.size(), "chainf layers %zu", c.L.size());
            for (size_t l = 0; l < c.L.size(); ++l)
                MUST(c.L[l].seed.ztag == lay[6 * l + 3] && c.L[l].seed.nonce.lo == lay[6 * l + 4], "chainf layer %zu", l);
            const auto dig = read_u64(ref + "/chainf_final_sigdig.u64");
            MUST(dig.size() == c.E.size(), "chainf sigma digests");
            for (size_t e = 0; e < c.E.size(); ++e) MUST(sigma_digest(c.E[e].s.w) == dig[e], "chainf sigma %zu", e);
            MUST(pvac_hip::dec_value(pk, sk, c).lo == 32, "chainf dec_value");
            auto rp = std::make_shared<replay>(replay{mul_words});
            std::vector<pvac_hip::RandomSource> rnds{[rp] { return (*rp)(); }};
            const Cipher c2 = pvac_hip::ct_mul_chain(pk, std::vector<Cipher>{x}, ys, true, rnds)[0];
            MUST(rp->k == mul_words.size(), "chainf chain entry consumed %zu of %zu words", rp->k, mul_words.size());
            MUST(same_layers(c2, c) && same_edges(c2, c, true), "chainf c_4 (chain entry point) == by value");
        }
        // fresh randomness, batched both ways
        const auto cs = pvac_hip::enc_value_batch<Cipher>(pk, sk, vs);
        const auto ms = pvac_hip::dec_value_batch(pk, sk, cs);
        for (size_t i = 0; i < vs.size(); ++i) MUST(ms[i].lo == vs[i] && ms[i].hi == 0, "batch roundtrip %zu", i);
        // homomorphic: dec(enc(a) + enc(b)) = a + b, dec(enc(a) * enc(b)) = a * b (small values)
        const Cipher s = pvac_hip::ct_add(pk, cs[1], cs[2]);
        const Cipher p = pvac_hip::ct_mul(pk, cs[1], cs[2]);
        MUST(pvac_hip::dec_value(pk, sk, s).lo == vs[1] + vs[2], "dec(ct_add)");
        MUST(pvac_hip::dec_value(pk, sk, p).lo == vs[1] * vs[2], "dec(ct_mul)");
    }

    // .ct codec through the adapter: load then save reproduces the reference's file bytes
    for (const char* f : {"/pair0_mul.ct", "/enc3.ct", "/chain3.ct"}) {
        const auto bytes = slurp(ref + f);
        const auto cs = pvac_hip::load_cts_bytes<Cipher>(bytes);
        MUST(same_edges(cs[0], read_ct(ref + f)[0], true), "load_cts %s", f);
        const uint32_t nb = cs[0].E.empty() ? 8192u : (uint32_t)cs[0].E[0].s.nbits;
        MUST(pvac_hip::save_cts_bytes(cs, nb) == bytes, "save_cts %s", f);
    }

    std::printf("test_adapter: %d checks passed\n", g_checks);
    return 0;
}
