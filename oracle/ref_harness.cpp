// ref_harness.cpp — TEST INFRASTRUCTURE ONLY: the reference itself, never the product.
//
// Two uses, nothing else: (1) minting the golden fixtures under tests/golden/ in this container;
// (2) the `kind: "reference"` CPU baseline legs of bench.py (time_mul / time_enc), for which the
// binary built here travels to the GPU box under oracle/_ref/ (git-ignored, not gpurun-ignored).
// The engine never links, loads or calls it.
//
// Compiles the UNMODIFIED header-only reference (pvac-hfhe 0.1.0) from
// /root/reference/include and drives it deterministically to mint the golden fixtures
// under tests/golden/. Built by oracle/Makefile into oracle/_ref/ (git-ignored).
//
// Determinism: every byte of entropy in the reference flows through libc getrandom(2)
// (reference include/pvac/core/random.hpp:40-56, csprng_u64 at :106-110). We interpose
// getrandom with a seeded splitmix64 stream (one 64-bit value per 8 requested bytes) and
// LOG every produced word, so the exact nonce/salt stream consumed by each ct_* call can be
// handed to the GPU engine's ABI as its explicit `nonces` / `salts` inputs.
//
// Output formats (all little-endian):
//   *.ct          — the reference's own on-disk format (tests/add.cpp:22-155 layout),
//                   written by our own writer below; "weights-only" files use nbits=0 sigmas.
//   *.u64         — raw u64 arrays.
//   manifest.json — metadata (counts, digests, plaintexts).
#include <pvac/pvac.hpp>

#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>
#include <chrono>
#include <thread>

using namespace pvac;

// ---------------------------------------------------------------- getrandom interposer
static uint64_t g_sm_state = 0x5EED0001ULL;
static std::vector<uint64_t> g_log;
static bool g_logging = true;

static uint64_t splitmix64_next() {
    uint64_t z = (g_sm_state += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

extern "C" ssize_t getrandom(void* buf, size_t n, unsigned int) {
    uint8_t* p = (uint8_t*)buf;
    size_t off = 0;
    while (off < n) {
        uint64_t v = splitmix64_next();
        if (g_logging) g_log.push_back(v);
        size_t take = (n - off < 8) ? (n - off) : 8;
        std::memcpy(p + off, &v, take);
        off += take;
    }
    return (ssize_t)n;
}

static void reseed(uint64_t s) { g_sm_state = s; }

// ---------------------------------------------------------------- writers
static void put32(std::ostream& o, uint32_t x) { o.write((const char*)&x, 4); }
static void put64(std::ostream& o, uint64_t x) { o.write((const char*)&x, 8); }

static void write_ct(const std::string& path, const std::vector<Cipher>& cts, bool with_sigma) {
    std::ofstream o(path, std::ios::binary);
    put32(o, 0x66699666u);
    put32(o, 1u);
    put64(o, (uint64_t)cts.size());
    for (const auto& C : cts) {
        put32(o, (uint32_t)C.L.size());
        put32(o, (uint32_t)C.E.size());
        for (const auto& L : C.L) {
            o.put((char)(uint8_t)L.rule);
            if (L.rule == RRule::BASE) {
                put64(o, L.seed.ztag); put64(o, L.seed.nonce.lo); put64(o, L.seed.nonce.hi);
            } else {
                put32(o, L.pa); put32(o, L.pb);
            }
        }
        for (const auto& e : C.E) {
            put32(o, e.layer_id);
            o.write((const char*)&e.idx, 2);
            o.put((char)e.ch);
            o.put(0);
            put64(o, e.w.lo); put64(o, e.w.hi);
            if (with_sigma) {
                put32(o, (uint32_t)e.s.nbits);
                for (size_t i = 0; i < (e.s.nbits + 63) / 64; ++i) put64(o, e.s.w[i]);
            } else {
                put32(o, 0u);
            }
        }
    }
}

// PROD layers carry seeds too (ct_mul sets them, arithmetic.hpp:59-70) but the .ct format
// drops them for PROD. Dump the full layer table separately: rule,pa,pb,ztag,nlo,nhi.
static void write_layers(const std::string& path, const Cipher& C) {
    std::ofstream o(path, std::ios::binary);
    for (const auto& L : C.L) {
        put64(o, (uint64_t)L.rule);
        put64(o, L.rule == RRule::PROD ? (uint64_t)L.pa : 0);
        put64(o, L.rule == RRule::PROD ? (uint64_t)L.pb : 0);
        put64(o, L.seed.ztag); put64(o, L.seed.nonce.lo); put64(o, L.seed.nonce.hi);
    }
}

static void write_u64(const std::string& path, const std::vector<uint64_t>& v) {
    std::ofstream o(path, std::ios::binary);
    o.write((const char*)v.data(), (std::streamsize)(v.size() * 8));
}

static std::string hex(const uint8_t* d, size_t n) {
    static const char* H = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < n; ++i) { s += H[d[i] >> 4]; s += H[d[i] & 15]; }
    return s;
}

// per-edge sigma digest: first 8 bytes (LE) of SHA-256 over the sigma words (LE)
static std::vector<uint64_t> sigma_digests(const Cipher& C) {
    std::vector<uint64_t> out;
    out.reserve(C.E.size());
    for (const auto& e : C.E) {
        Sha256 s; s.init();
        for (uint64_t w : e.s.w) sha256_acc_u64(s, w);
        uint8_t d[32]; s.finish(d);
        out.push_back(load_le64(d));
    }
    return out;
}

// ---------------------------------------------------------------- Fp vectors
static const uint64_t MAXU = ~0ULL;

static void cmd_fp(const std::string& dir) {
    reseed(0x5EED0F00ULL);
    std::vector<Fp> A, B;
    // edge cases: 0,1,2,p-1,p-2,2^64-1,2^64,2^126,2^127-2, and
    // non-canonical values (hi >= 2^63, == p) for the fp_add truncation / fp_neg quirks.
    std::vector<Fp> edge = {
        {0, 0}, {1, 0}, {2, 0}, {MAXU - 1, MASK63}, {MAXU - 2, MASK63}, {MAXU, 0}, {0, 1},
        {0, 1ULL << 62}, {MAXU - 2, MASK63}, {MAXU, MASK63} /* p */, {0, 1ULL << 63} /* 2^127 */,
        {MAXU, MAXU}, {MAXU, 1ULL << 63}, {1, 1ULL << 63}, {MAXU - 1, MAXU}, {12345, MASK63},
        {0x8000000000000000ULL, 0x4000000000000000ULL}, {MAXU, 0x7FFFFFFFFFFFFFFEULL},
        {3, 0xC000000000000000ULL}, {0xDEADBEEFULL, 0xFFFFFFFF00000000ULL},
        {MAXU, 0x3FFFFFFFFFFFFFFFULL}, {1, MASK63}, {0, MASK63}, {MAXU - 1, MASK63 - 1},
        {0x0123456789ABCDEFULL, 0x7EDCBA9876543210ULL}, {0x1ULL << 63, 0},
        {MAXU, 0x8000000000000001ULL}, {5, 0xFFFFFFFFFFFFFFF0ULL},
        {0xAAAAAAAAAAAAAAAAULL, 0x5555555555555555ULL}, {0x5555555555555555ULL, 0xAAAAAAAAAAAAAAAAULL},
        {2, MASK63}, {MAXU - 3, MASK63},
    };
    for (size_t i = 0; i < edge.size(); ++i)
        for (size_t j = 0; j < edge.size(); ++j) { A.push_back(edge[i]); B.push_back(edge[j]); }
    // random canonical
    for (int i = 0; i < 2048; ++i) {
        Fp a = fp_from_words(splitmix64_next(), splitmix64_next() & MASK63);
        Fp b = fp_from_words(splitmix64_next(), splitmix64_next() & MASK63);
        A.push_back(a); B.push_back(b);
    }
    // random arbitrary 128-bit (non-canonical allowed)
    for (int i = 0; i < 1024; ++i) {
        Fp a{splitmix64_next(), splitmix64_next()};
        Fp b{splitmix64_next(), splitmix64_next()};
        A.push_back(a); B.push_back(b);
    }
    size_t n = A.size();
    std::vector<uint64_t> a_lo(n), a_hi(n), b_lo(n), b_hi(n), add_lo(n), add_hi(n), sub_lo(n),
        sub_hi(n), neg_lo(n), neg_hi(n), mul_lo(n), mul_hi(n), fw_lo(n), fw_hi(n);
    for (size_t i = 0; i < n; ++i) {
        a_lo[i] = A[i].lo; a_hi[i] = A[i].hi; b_lo[i] = B[i].lo; b_hi[i] = B[i].hi;
        Fp s = fp_add(A[i], B[i]), d = fp_sub(A[i], B[i]), g = fp_neg(A[i]), m = fp_mul(A[i], B[i]);
        Fp f = fp_from_words(A[i].lo, A[i].hi);
        add_lo[i] = s.lo; add_hi[i] = s.hi; sub_lo[i] = d.lo; sub_hi[i] = d.hi;
        neg_lo[i] = g.lo; neg_hi[i] = g.hi; mul_lo[i] = m.lo; mul_hi[i] = m.hi;
        fw_lo[i] = f.lo; fw_hi[i] = f.hi;
    }
    // inverses of canonical nonzero values
    std::vector<uint64_t> inv_in_lo, inv_in_hi, inv_lo, inv_hi;
    for (int i = 0; i < 512; ++i) {
        Fp a = rand_fp_nonzero();
        Fp v = fp_inv(a);
        inv_in_lo.push_back(a.lo); inv_in_hi.push_back(a.hi); inv_lo.push_back(v.lo); inv_hi.push_back(v.hi);
    }
    // fp_pow_u64
    std::vector<uint64_t> pw_lo, pw_hi, pw_e, pw_rlo, pw_rhi;
    for (int i = 0; i < 256; ++i) {
        Fp a = fp_from_words(splitmix64_next(), splitmix64_next() & MASK63);
        uint64_t e = splitmix64_next() >> (i % 64);
        Fp r = fp_pow_u64(a, e);
        pw_lo.push_back(a.lo); pw_hi.push_back(a.hi); pw_e.push_back(e); pw_rlo.push_back(r.lo); pw_rhi.push_back(r.hi);
    }
    write_u64(dir + "/fp_a_lo.u64", a_lo); write_u64(dir + "/fp_a_hi.u64", a_hi);
    write_u64(dir + "/fp_b_lo.u64", b_lo); write_u64(dir + "/fp_b_hi.u64", b_hi);
    write_u64(dir + "/fp_add_lo.u64", add_lo); write_u64(dir + "/fp_add_hi.u64", add_hi);
    write_u64(dir + "/fp_sub_lo.u64", sub_lo); write_u64(dir + "/fp_sub_hi.u64", sub_hi);
    write_u64(dir + "/fp_neg_lo.u64", neg_lo); write_u64(dir + "/fp_neg_hi.u64", neg_hi);
    write_u64(dir + "/fp_mul_lo.u64", mul_lo); write_u64(dir + "/fp_mul_hi.u64", mul_hi);
    write_u64(dir + "/fp_fromw_lo.u64", fw_lo); write_u64(dir + "/fp_fromw_hi.u64", fw_hi);
    write_u64(dir + "/fp_inv_in_lo.u64", inv_in_lo); write_u64(dir + "/fp_inv_in_hi.u64", inv_in_hi);
    write_u64(dir + "/fp_inv_lo.u64", inv_lo); write_u64(dir + "/fp_inv_hi.u64", inv_hi);
    write_u64(dir + "/fp_pow_a_lo.u64", pw_lo); write_u64(dir + "/fp_pow_a_hi.u64", pw_hi);
    write_u64(dir + "/fp_pow_e.u64", pw_e); write_u64(dir + "/fp_pow_r_lo.u64", pw_rlo);
    write_u64(dir + "/fp_pow_r_hi.u64", pw_rhi);
    std::printf("fp vectors: %zu binop cases\n", n);
}

// ---------------------------------------------------------------- cipher fixtures
struct OpRecord {
    std::vector<uint64_t> stream;  // words consumed by the op (nonces then salts)
};

template <class F>
static Cipher run_logged(F&& f, std::vector<uint64_t>& consumed) {
    size_t before = g_log.size();
    Cipher C = f();
    consumed.assign(g_log.begin() + (long)before, g_log.end());
    return C;
}

static std::vector<Fp> base_layer_R(const PubKey& pk, const SecKey& sk, const Cipher& C) {
    std::vector<Fp> R;
    for (const auto& L : C.L) {
        if (L.rule == RRule::BASE) R.push_back(prf_R(pk, sk, L.seed));
        else R.push_back(Fp{0, 0});
    }
    return R;
}

static void dump_R(const std::string& path, const std::vector<Fp>& R) {
    std::vector<uint64_t> v;
    for (auto& r : R) { v.push_back(r.lo); v.push_back(r.hi); }
    write_u64(path, v);
}

static std::string fpjson(const Fp& f) {
    char b[96];
    std::snprintf(b, sizeof b, "[%" PRIu64 ", %" PRIu64 "]", f.lo, f.hi);
    return b;
}

static void cmd_fixtures(const std::string& dir, int npairs, int chain_steps, int sq_steps) {
    reseed(0x5EED0C00ULL);
    Params prm;
    PubKey pk;
    SecKey sk;
    g_logging = false;
    keygen(prm, pk, sk);
    g_logging = true;

    std::ostringstream js;
    js << "{\n  \"canon_tag\": " << pk.canon_tag << ",\n";
    js << "  \"H_digest\": \"" << hex(pk.H_digest.data(), 32) << "\",\n";
    js << "  \"params\": {\"B\": " << prm.B << ", \"m_bits\": " << prm.m_bits << ", \"n_bits\": " << prm.n_bits
       << ", \"h_col_wt\": " << prm.h_col_wt << ", \"x_col_wt\": " << prm.x_col_wt << ", \"err_wt\": " << prm.err_wt
       << ", \"edge_budget\": " << prm.edge_budget << "},\n";
    {
        std::vector<uint64_t> pg;
        for (auto& f : pk.powg_B) { pg.push_back(f.lo); pg.push_back(f.hi); }
        write_u64(dir + "/powg_B.u64", pg);
        // H columns 0..63 dense (64 x 128 words = 64 KiB) to pin gen_H restatements cheaply.
        std::vector<uint64_t> h;
        for (int c = 0; c < 64; ++c) for (uint64_t w : pk.H[c].w) h.push_back(w);
        write_u64(dir + "/H_cols0_63.u64", h);
    }

    // ---- fresh pairs: enc_value x/y, then ct_add / ct_sub / ct_mul
    js << "  \"pairs\": [\n";
    for (int p = 0; p < npairs; ++p) {
        uint64_t x = splitmix64_next() % 1000003, y = splitmix64_next() % 1000003;
        if (p == 0) { x = 2016733; y = 7083881; }   // test_main.cpp values
        if (p == 1) { x = 0; y = 1; }
        std::vector<uint64_t> dummy;
        Cipher X = run_logged([&] { return enc_value(pk, sk, x); }, dummy);
        Cipher Y = run_logged([&] { return enc_value(pk, sk, y); }, dummy);
        std::string pre = dir + "/pair" + std::to_string(p);
        write_ct(pre + "_x.ct", {X}, true);
        write_ct(pre + "_y.ct", {Y}, true);
        dump_R(pre + "_x_R.u64", base_layer_R(pk, sk, X));
        dump_R(pre + "_y_R.u64", base_layer_R(pk, sk, Y));

        std::vector<uint64_t> s_add, s_sub, s_mul;
        Cipher S = run_logged([&] { return ct_add(pk, X, Y); }, s_add);
        Cipher D = run_logged([&] { return ct_sub(pk, X, Y); }, s_sub);
        auto t0 = std::chrono::steady_clock::now();
        Cipher M = run_logged([&] { return ct_mul(pk, X, Y); }, s_mul);
        auto t1 = std::chrono::steady_clock::now();
        write_ct(pre + "_add.ct", {S}, true);
        write_ct(pre + "_sub.ct", {D}, true);
        write_ct(pre + "_mul_w.ct", {M}, false);
        write_layers(pre + "_mul_layers.u64", M);
        write_u64(pre + "_mul_stream.u64", s_mul);
        write_u64(pre + "_mul_sigdig.u64", sigma_digests(M));
        if (p == 0) write_ct(pre + "_mul.ct", {M}, true);   // one full product with sigmas
        auto cm = commit_ct(pk, M), ca = commit_ct(pk, S), cs = commit_ct(pk, D);
        Fp dm = dec_value(pk, sk, M);
        js << "    {\"x\": " << x << ", \"y\": " << y << ", \"nx\": " << X.E.size() << ", \"ny\": " << Y.E.size()
           << ", \"mul_edges\": " << M.E.size() << ", \"mul_layers\": " << M.L.size()
           << ", \"add_stream\": " << s_add.size() << ", \"sub_stream\": " << s_sub.size()
           << ", \"mul_stream\": " << s_mul.size()
           << ", \"commit_mul\": \"" << hex(cm.data(), 32) << "\", \"commit_add\": \"" << hex(ca.data(), 32)
           << "\", \"commit_sub\": \"" << hex(cs.data(), 32) << "\", \"dec_mul\": " << fpjson(dm)
           << ", \"mul_ms\": " << std::chrono::duration<double, std::milli>(t1 - t0).count() << "}"
           << (p + 1 < npairs ? "," : "") << "\n";
        std::fflush(stdout);
    }
    js << "  ],\n";

    // ---- chain x fresh (test_main.cpp:289-292 shape): c_k = c_{k-1} * x_k
    js << "  \"chain\": [\n";
    {
        std::vector<uint64_t> dummy;
        Cipher c = run_logged([&] { return enc_value(pk, sk, 2); }, dummy);
        write_ct(dir + "/chain0.ct", {c}, true);
        dump_R(dir + "/chain0_R.u64", base_layer_R(pk, sk, c));
        for (int k = 1; k <= chain_steps; ++k) {
            Cipher x = run_logged([&] { return enc_value(pk, sk, 2); }, dummy);
            std::string pre = dir + "/chain" + std::to_string(k);
            write_ct(pre + "_x.ct", {x}, true);
            dump_R(pre + "_x_R.u64", base_layer_R(pk, sk, x));
            std::vector<uint64_t> st;
            Cipher n = run_logged([&] { return ct_mul(pk, c, x); }, st);
            write_ct(pre + ".ct", {n}, false);
            write_layers(pre + "_layers.u64", n);
            write_u64(pre + "_stream.u64", st);
            write_u64(pre + "_sigdig.u64", sigma_digests(n));
            auto cm = commit_ct(pk, n);
            Fp d = dec_value(pk, sk, n);
            js << "    {\"step\": " << k << ", \"edges\": " << n.E.size() << ", \"layers\": " << n.L.size()
               << ", \"stream\": " << st.size() << ", \"commit\": \"" << hex(cm.data(), 32)
               << "\", \"dec\": " << fpjson(d) << "}" << (k < chain_steps ? "," : "") << "\n";
            c = std::move(n);
            std::printf("chain step %d edges %zu\n", k, c.E.size());
            std::fflush(stdout);
        }
    }
    js << "  ],\n";

    // ---- squaring chain (test_depth.cpp:46): c <- c*c
    js << "  \"square\": [\n";
    {
        std::vector<uint64_t> dummy;
        Cipher c = run_logged([&] { return enc_value(pk, sk, 2); }, dummy);
        write_ct(dir + "/sq0.ct", {c}, true);
        dump_R(dir + "/sq0_R.u64", base_layer_R(pk, sk, c));
        for (int k = 1; k <= sq_steps; ++k) {
            std::vector<uint64_t> st;
            Cipher n = run_logged([&] { return ct_mul(pk, c, c); }, st);
            std::string pre = dir + "/sq" + std::to_string(k);
            write_ct(pre + ".ct", {n}, false);
            write_layers(pre + "_layers.u64", n);
            write_u64(pre + "_stream.u64", st);
            write_u64(pre + "_sigdig.u64", sigma_digests(n));
            auto cm = commit_ct(pk, n);
            Fp d = dec_value(pk, sk, n);
            js << "    {\"step\": " << k << ", \"edges\": " << n.E.size() << ", \"layers\": " << n.L.size()
               << ", \"stream\": " << st.size() << ", \"commit\": \"" << hex(cm.data(), 32)
               << "\", \"dec\": " << fpjson(d) << "}" << (k < sq_steps ? "," : "") << "\n";
            c = std::move(n);
            std::printf("square step %d edges %zu\n", k, c.E.size());
            std::fflush(stdout);
        }
    }
    js << "  ],\n";

    // ---- guard_budget / compact_edges on a hand-made over-budget cipher is too large to
    // commit; instead exercise compact_edges directly on a small cipher with duplicates and
    // non-canonical weights (encrypt.hpp:39-71) using a tiny edge_budget.
    {
        PubKey pk2 = pk;
        pk2.prm.edge_budget = 16;
        std::vector<uint64_t> dummy;
        Cipher X = run_logged([&] { return enc_value(pk, sk, 5); }, dummy);
        Cipher Y = run_logged([&] { return enc_value(pk, sk, 7); }, dummy);
        // inject duplicates of (layer,idx,ch) and non-canonical weights into Y
        Y.E[1].idx = Y.E[0].idx; Y.E[1].ch = Y.E[0].ch; Y.E[1].layer_id = Y.E[0].layer_id;
        Y.E[2].w = Fp{MAXU, MAXU};
        Y.E[3].w = Fp{MAXU - 7, 0x8000000000000000ULL};
        write_ct(dir + "/guard_x.ct", {X}, true);
        write_ct(dir + "/guard_y.ct", {Y}, true);
        std::vector<uint64_t> st;
        Cipher S = run_logged([&] { return ct_add(pk2, X, Y); }, st);
        write_ct(dir + "/guard_add.ct", {S}, true);
        auto c = commit_ct(pk, S);
        js << "  \"guard\": {\"edge_budget\": 16, \"edges\": " << S.E.size() << ", \"layers\": " << S.L.size()
           << ", \"commit\": \"" << hex(c.data(), 32) << "\"},\n";
    }
    js << "  \"generator\": \"oracle/ref_harness.cpp (reference pvac-hfhe 0.1.0, g++ -O2)\"\n}\n";
    std::ofstream(dir + "/manifest.json") << js.str();
}

// ---------------------------------------------------------------- full-range ct_mul fixtures
// ct_mul on weights outside [0, p): fp_mul (core/field.hpp:113-213) takes any 128-bit operand.
// Case k (x, y from enc_value, then weights overwritten):
//   0, 1 : every weight full-range random (both words any u64)
//   2    : weights cycled over special values (p, p-1, 2^127, 2^128-1, 0, 1, ...)
//   3    : cancellation: x's edge 1 copies edge 0's (layer, idx, ch) with weight p - w0 (sum 0 mod
//          p for every key those two reach alone), x's edge 2 weight p (== 0), y's edge 0 weight 0
//   4    : general-path shape: (x0 * y0) with full-range weights, times a fresh full-range y
static void cmd_fullrange(const std::string& dir) {
    reseed(0x5EED0C00ULL);   // the same key as cmd_fixtures
    Params prm;
    PubKey pk;
    SecKey sk;
    g_logging = false;
    keygen(prm, pk, sk);
    reseed(0x5EED0F00ULL);
    const std::vector<Fp> special = {
        {MAXU, MASK63} /* p */,          {MAXU - 1, MASK63} /* p-1 */, {0, 1ULL << 63} /* 2^127 */,
        {MAXU, MAXU} /* 2^128-1 */,      {0, 0},                       {1, 0},
        {MAXU, 1ULL << 63},              {1, 1ULL << 63} /* p+2 */,    {MAXU, 0},
        {0x8000000000000000ULL, 0xC000000000000000ULL}, {MAXU - 2, MAXU}, {12345, 0xFFFFFFFF00000000ULL}};
    auto full = [&](Cipher& C) {
        for (auto& e : C.E) e.w = Fp{splitmix64_next(), splitmix64_next()};
    };
    std::ostringstream js;
    js << "{\n  \"canon_tag\": " << pk.canon_tag << ",\n  \"cases\": [\n";
    const int ncase = 5;
    for (int k = 0; k < ncase; ++k) {
        g_logging = false;
        Cipher X = enc_value(pk, sk, 11 + (uint64_t)k), Y = enc_value(pk, sk, 17 + (uint64_t)k);
        if (k <= 1) {
            full(X);
            full(Y);
        } else if (k == 2) {
            for (size_t i = 0; i < X.E.size(); ++i) X.E[i].w = special[i % special.size()];
            for (size_t i = 0; i < Y.E.size(); ++i) Y.E[i].w = special[(i * 5 + 3) % special.size()];
        } else if (k == 3) {
            full(X);
            X.E[1].layer_id = X.E[0].layer_id;
            X.E[1].idx = X.E[0].idx;
            X.E[1].ch = X.E[0].ch;
            X.E[1].w = fp_neg(fp_from_words(X.E[0].w.lo, X.E[0].w.hi & MASK63));
            X.E[2].w = Fp{MAXU, MASK63};
            Y.E[0].w = Fp{0, 0};
        } else {
            full(X);
            full(Y);
            Cipher P = ct_mul(pk, X, Y);
            full(P);
            for (auto& L : P.L)   // as after a .ct round trip, which drops PROD seeds
                if (L.rule == RRule::PROD) L.seed = RSeed{};
            X = std::move(P);
            Y = enc_value(pk, sk, 23);
            full(Y);
        }
        for (auto& e : X.E) e.s = BitVec::make(0);
        for (auto& e : Y.E) e.s = BitVec::make(0);
        g_logging = true;
        const std::string pre = dir + "/fr" + std::to_string(k);
        write_ct(pre + "_x.ct", {X}, false);
        write_ct(pre + "_y.ct", {Y}, false);
        std::vector<uint64_t> st;
        Cipher M = run_logged([&] { return ct_mul(pk, X, Y); }, st);
        write_ct(pre + "_mul_w.ct", {M}, false);
        write_layers(pre + "_mul_layers.u64", M);
        write_u64(pre + "_mul_stream.u64", st);
        js << "    {\"case\": " << k << ", \"nx\": " << X.E.size() << ", \"ny\": " << Y.E.size() << ", \"lx\": "
           << X.L.size() << ", \"ly\": " << Y.L.size() << ", \"mul_edges\": " << M.E.size() << ", \"mul_layers\": "
           << M.L.size() << ", \"stream\": " << st.size() << "}" << (k + 1 < ncase ? "," : "") << "\n";
        std::printf("fullrange case %d: %zu x %zu edges -> %zu\n", k, X.E.size(), Y.E.size(), M.E.size());
        std::fflush(stdout);
    }
    js << "  ],\n  \"generator\": \"oracle/ref_harness.cpp fullrange (reference pvac-hfhe 0.1.0)\"\n}\n";
    std::ofstream(dir + "/fr_manifest.json") << js.str();
}

// ---------------------------------------------------------------- enc_value_depth / enc_zero_depth
// The other encryption entry points (ops/encrypt.hpp:281-298): depth hints change the noise plan
// (plan_noise, encrypt.hpp:16-27). Same key as cmd_fixtures; each case logs the stream it consumed.
static void cmd_encdepth(const std::string& dir) {
    reseed(0x5EED0C00ULL);
    Params prm;
    PubKey pk;
    SecKey sk;
    g_logging = false;
    keygen(prm, pk, sk);
    (void)enc_value(pk, sk, 1);   // warm-up: the Toeplitz autotuner draws random words once
    struct Case { int kind; uint64_t v; int depth; };   // kind 0: enc_value_depth, 1: enc_zero_depth
    const Case cases[] = {{0, 2016733, 1}, {0, 5, 3}, {0, 7083881, 8}, {0, 42, 15}, {1, 0, 0}, {1, 0, 5}};
    const int nc = (int)(sizeof cases / sizeof cases[0]);
    std::ostringstream js;
    js << "{\n  \"canon_tag\": " << pk.canon_tag << ",\n  \"cases\": [\n";
    for (int i = 0; i < nc; ++i) {
        const Case& c = cases[i];
        reseed(0x5EED0D10ULL + (uint64_t)i);
        g_logging = true;
        std::vector<uint64_t> stream;
        Cipher X = run_logged([&] { return c.kind ? enc_zero_depth(pk, sk, c.depth) : enc_value_depth(pk, sk, c.v, c.depth); },
                              stream);
        g_logging = false;
        const std::string pre = dir + "/encd" + std::to_string(i);
        write_ct(pre + ".ct", {X}, true);
        write_u64(pre + "_stream.u64", stream);
        dump_R(pre + "_R.u64", base_layer_R(pk, sk, X));
        const Fp dv = dec_value(pk, sk, X);
        const auto z = plan_noise(pk, c.depth);
        js << "    {\"kind\": \"" << (c.kind ? "zero" : "value") << "\", \"v\": " << c.v << ", \"depth\": " << c.depth
           << ", \"Z2\": " << z.first << ", \"Z3\": " << z.second << ", \"edges\": " << X.E.size()
           << ", \"layers\": " << X.L.size() << ", \"stream\": " << stream.size() << ", \"dec\": " << fpjson(dv)
           << "}" << (i + 1 < nc ? "," : "") << "\n";
        std::printf("encdepth case %d: depth %d edges %zu stream %zu\n", i, c.depth, X.E.size(), stream.size());
    }
    js << "  ],\n  \"generator\": \"oracle/ref_harness.cpp encdepth (reference pvac-hfhe 0.1.0)\"\n}\n";
    std::ofstream(dir + "/encd_manifest.json") << js.str();
}

// ---------------------------------------------------------------- deep depth hints, other noise Params
// enc_value_depth / enc_zero_depth with depth hints past 15 and with non-default noise Params
// (noise_entropy_bits, tuple2_fraction, depth_slope_bits: plan_noise, encrypt.hpp:16-27), including
// a plan with no noise groups and one bumped from a single group to two. Same key as cmd_encdepth.
static void cmd_encdeep(const std::string& dir) {
    reseed(0x5EED0C00ULL);
    Params prm;
    PubKey pk;
    SecKey sk;
    g_logging = false;
    keygen(prm, pk, sk);
    (void)enc_value(pk, sk, 1);   // warm-up: the Toeplitz autotuner draws random words once
    struct Case { int kind; uint64_t v; int depth; double ent, frac, slope; };
    const Case cases[] = {{0, 77, 16, 120.0, 0.55, 16.0},   {0, 123456789, 31, 120.0, 0.55, 16.0},
                          {0, 9, 60, 120.0, 0.55, 16.0},    {1, 0, 100, 120.0, 0.55, 16.0},
                          {0, 31337, 2, 64.0, 0.8, 8.0},   {0, 4, 7, 200.0, 0.2, 20.0},
                          {0, 1000003, 0, 40.0, 0.5, 16.0}, {0, 11, 0, 0.0, 0.55, 0.0}};
    const int nc = (int)(sizeof cases / sizeof cases[0]);
    std::ostringstream js;
    js << "{\n  \"canon_tag\": " << pk.canon_tag << ",\n  \"cases\": [\n";
    for (int i = 0; i < nc; ++i) {
        const Case& c = cases[i];
        PubKey pkc = pk;
        pkc.prm.noise_entropy_bits = c.ent;
        pkc.prm.tuple2_fraction = c.frac;
        pkc.prm.depth_slope_bits = c.slope;
        reseed(0x5EED0F10ULL + (uint64_t)i);
        g_logging = true;
        std::vector<uint64_t> stream;
        Cipher X = run_logged([&] { return c.kind ? enc_zero_depth(pkc, sk, c.depth) : enc_value_depth(pkc, sk, c.v, c.depth); },
                              stream);
        g_logging = false;
        const std::string pre = dir + "/encx" + std::to_string(i);
        write_ct(pre + ".ct", {X}, true);
        write_u64(pre + "_stream.u64", stream);
        const Fp dv = dec_value(pkc, sk, X);
        const auto z = plan_noise(pkc, c.depth);
        js << "    {\"kind\": \"" << (c.kind ? "zero" : "value") << "\", \"v\": " << c.v << ", \"depth\": " << c.depth
           << ", \"noise_entropy_bits\": " << c.ent << ", \"tuple2_fraction\": " << c.frac << ", \"depth_slope_bits\": "
           << c.slope << ", \"Z2\": " << z.first << ", \"Z3\": " << z.second << ", \"edges\": " << X.E.size()
           << ", \"layers\": " << X.L.size() << ", \"stream\": " << stream.size() << ", \"dec\": " << fpjson(dv)
           << "}" << (i + 1 < nc ? "," : "") << "\n";
        std::printf("encdeep case %d: depth %d Z2 %d Z3 %d edges %zu stream %zu\n", i, c.depth, z.first, z.second,
                    X.E.size(), stream.size());
    }
    js << "  ],\n  \"generator\": \"oracle/ref_harness.cpp encdeep (reference pvac-hfhe 0.1.0)\"\n}\n";
    std::ofstream(dir + "/encx_manifest.json") << js.str();
}

// ---------------------------------------------------------------- timing (CPU baseline leg)
// Times the reference's own ct_mul (WITH sigma, arithmetic.hpp:47-106) on fresh pairs.
static void cmd_time_mul(int npairs, int threads) {
    reseed(0x5EED0D00ULL);
    g_logging = false;
    Params prm; PubKey pk; SecKey sk;
    keygen(prm, pk, sk);
    std::vector<Cipher> X, Y;
    for (int i = 0; i < 2 * threads; ++i) { X.push_back(enc_value(pk, sk, i + 3)); Y.push_back(enc_value(pk, sk, i + 5)); }
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    size_t edges_total[256] = {0};
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            for (int i = t; i < npairs; i += threads) {
                Cipher M = ct_mul(pk, X[(size_t)(i % (2 * threads))], Y[(size_t)(i % (2 * threads))]);
                edges_total[t] += M.E.size();
            }
        });
    for (auto& x : th) x.join();
    auto t1 = std::chrono::steady_clock::now();
    double s = std::chrono::duration<double>(t1 - t0).count();
    size_t et = 0;
    for (int t = 0; t < threads; ++t) et += edges_total[t];
    std::printf("{\"pairs\": %d, \"threads\": %d, \"seconds\": %.6f, \"ct_mul_per_s\": %.3f, \"edges\": %zu}\n",
                npairs, threads, s, npairs / s, et);
}

// cfg 4's workload on the unmodified reference (SURVEY 8(d) restatement of tests/test_main.cpp:289-295):
// x = enc_value(v), c_0 = x, c_k = ct_mul(c_{k-1}, x) for k = 1..depth (full ct_mul, sigma included).
// Only the ct_mul steps are timed; one line of JSON with the per-step edge counts.
static void cmd_time_chain(int ninputs, int depth) {
    reseed(0x5EED0D40ULL);
    g_logging = false;
    Params prm; PubKey pk; SecKey sk;
    keygen(prm, pk, sk);
    std::vector<Cipher> X;
    for (int i = 0; i < ninputs; ++i) X.push_back(enc_value(pk, sk, (uint64_t)i * 31u + 7u));
    std::vector<size_t> edges((size_t)depth, 0);
    double s = 0.0;
    for (int i = 0; i < ninputs; ++i) {
        Cipher c = X[(size_t)i];
        for (int d = 0; d < depth; ++d) {
            auto t0 = std::chrono::steady_clock::now();
            c = ct_mul(pk, c, X[(size_t)i]);
            s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            edges[(size_t)d] += c.E.size();
        }
    }
    std::printf("{\"inputs\": %d, \"depth\": %d, \"seconds\": %.6f, \"ct_mul_per_s\": %.6f, \"edges_by_step\": [",
                ninputs, depth, s, ninputs * depth / s);
    for (int d = 0; d < depth; ++d) std::printf("%s%zu", d ? ", " : "", edges[(size_t)d]);
    std::printf("]}\n");
}

static void cmd_time_enc(int ncalls) {
    reseed(0x5EED0D00ULL);
    g_logging = false;
    Params prm; PubKey pk; SecKey sk;
    keygen(prm, pk, sk);
    (void)enc_value(pk, sk, 1);   // warm-up (Toeplitz autotuner)
    size_t edges = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < ncalls; ++i) edges += enc_value(pk, sk, (uint64_t)i * 7919u).E.size();
    auto t1 = std::chrono::steady_clock::now();
    double s = std::chrono::duration<double>(t1 - t0).count();
    std::printf("{\"calls\": %d, \"seconds\": %.6f, \"enc_per_s\": %.3f, \"edges\": %zu}\n", ncalls, s, ncalls / s,
                edges);
}

// ---- f2 fixtures: key material, prf_R_core / prf_R / prf_noise_delta on seeded seeds, and
//      complete enc_value outputs with the exact getrandom stream each consumed.
static void cmd_enc(const std::string& dir, int nenc) {
    reseed(0x5EED0C00ULL);   // the same key as cmd_fixtures
    Params prm;
    PubKey pk;
    SecKey sk;
    g_logging = false;
    keygen(prm, pk, sk);
    g_logging = true;
    write_u64(dir + "/sk_prf_k.u64", std::vector<uint64_t>(sk.prf_k.begin(), sk.prf_k.end()));
    write_u64(dir + "/sk_lpn_s.u64", sk.lpn_s_bits);
    auto zz = plan_noise(pk, 0);
    std::ostringstream js;
    js << "{\n  \"canon_tag\": " << pk.canon_tag << ",\n  \"lpn_n\": " << prm.lpn_n << ", \"lpn_t\": " << prm.lpn_t
       << ", \"lpn_tau_num\": " << prm.lpn_tau_num << ", \"lpn_tau_den\": " << prm.lpn_tau_den
       << ",\n  \"Z2\": " << zz.first << ", \"Z3\": " << zz.second << ",\n";
    // prf outputs: per seed {ztag, nonce lo, hi} then R1 R2 R3 N1 N2 N3 (prf_R_core), prf_R,
    // prf_R_noise, prf_noise_delta(group 0..4, kind 0) and (group 0..4, kind 1): 2 words each
    reseed(0x5EED0E00ULL);
    g_logging = false;
    const char* doms[] = {Dom::PRF_R1, Dom::PRF_R2, Dom::PRF_R3, Dom::PRF_NOISE1, Dom::PRF_NOISE2, Dom::PRF_NOISE3};
    std::vector<uint64_t> seeds, outs;
    const int nseed = 12;
    for (int k = 0; k < nseed; ++k) {
        RSeed sd;
        sd.ztag = splitmix64_next();
        sd.nonce.lo = splitmix64_next();
        sd.nonce.hi = splitmix64_next();
        seeds.push_back(sd.ztag); seeds.push_back(sd.nonce.lo); seeds.push_back(sd.nonce.hi);
        for (const char* d : doms) { Fp r = prf_R_core(pk, sk, sd, d); outs.push_back(r.lo); outs.push_back(r.hi); }
        Fp R = prf_R(pk, sk, sd), N = prf_R_noise(pk, sk, sd);
        outs.push_back(R.lo); outs.push_back(R.hi); outs.push_back(N.lo); outs.push_back(N.hi);
        for (int kind = 0; kind < 2; ++kind)
            for (uint32_t g = 0; g < 5; ++g) {
                Fp d = prf_noise_delta(pk, sk, sd, g, (uint8_t)kind);
                outs.push_back(d.lo); outs.push_back(d.hi);
            }
    }
    write_u64(dir + "/prf_seeds.u64", seeds);
    write_u64(dir + "/prf_out.u64", outs);
    js << "  \"prf_seeds\": " << nseed << ",\n  \"enc\": [\n";
    // enc_value with logged streams
    const uint64_t vals[] = {0, 1, 2, 2016733, 7083881, 1000002, ~0ULL, 0x123456789abcdefULL,
                             42, 65537, 3, 999};
    g_logging = true;
    for (int i = 0; i < nenc; ++i) {
        const uint64_t v = vals[i % 12];
        reseed(0x5EED0E10ULL + (uint64_t)i);
        std::vector<uint64_t> stream;
        Cipher X = run_logged([&] { return enc_value(pk, sk, v); }, stream);
        const std::string pre = dir + "/enc" + std::to_string(i);
        write_ct(pre + ".ct", {X}, true);
        write_u64(pre + "_stream.u64", stream);
        g_logging = false;
        dump_R(pre + "_R.u64", base_layer_R(pk, sk, X));
        Fp dv = dec_value(pk, sk, X);
        g_logging = true;
        js << "    {\"v\": " << v << ", \"seed\": " << (0x5EED0E10ULL + (uint64_t)i) << ", \"edges\": " << X.E.size()
           << ", \"layers\": " << X.L.size() << ", \"stream\": " << stream.size() << ", \"dec\": " << fpjson(dv) << "}"
           << (i + 1 < nenc ? "," : "") << "\n";
    }
    js << "  ]\n}\n";
    std::ofstream(dir + "/enc_manifest.json") << js.str();
}

// ---- chain entry-point fixture (pvac_hip_ct_mul_chain with a final-step WITH_SIGMA): x = enc_value(2),
//      c_0 = x, c_k = ct_mul(pk, c_{k-1}, x) for k = 1..depth (the test_depth / cfg-4 chain shape;
//      tests/test_main.cpp:289-293 multiplies by a fresh enc_value(2) per step instead), the full
//      getrandom stream of the chain (every step's nonces and salts, in the reference's order), and
//      c_depth: weights-only .ct, full layer table, per-edge sigma digests, its decryption.
static void cmd_chainx(const std::string& dir, int depth) {
    reseed(0x5EED0C00ULL);   // the same key as cmd_fixtures
    Params prm;
    PubKey pk;
    SecKey sk;
    g_logging = false;
    keygen(prm, pk, sk);
    g_logging = true;
    reseed(0x5EED0CC0ULL);
    std::vector<uint64_t> sx;
    Cipher x = run_logged([&] { return enc_value(pk, sk, 2); }, sx);
    write_ct(dir + "/chainx_x.ct", {x}, true);
    dump_R(dir + "/chainx_x_R.u64", base_layer_R(pk, sk, x));
    std::ostringstream js;
    js << "{\n  \"canon_tag\": " << pk.canon_tag << ", \"depth\": " << depth << ", \"x_stream\": " << sx.size()
       << ",\n  \"steps\": [";
    const size_t before = g_log.size();
    Cipher c = x;
    for (int k = 1; k <= depth; ++k) {
        const size_t b0 = g_log.size();
        c = ct_mul(pk, c, x);
        js << (k > 1 ? ", " : "") << "{\"edges\": " << c.E.size() << ", \"layers\": " << c.L.size()
           << ", \"stream\": " << (g_log.size() - b0) << "}";
        std::printf("chainx step %d edges %zu\n", k, c.E.size());
        std::fflush(stdout);
    }
    std::vector<uint64_t> st(g_log.begin() + (long)before, g_log.end());
    write_u64(dir + "/chainx_stream.u64", st);
    write_ct(dir + "/chainx_final.ct", {c}, false);
    write_layers(dir + "/chainx_final_layers.u64", c);
    write_u64(dir + "/chainx_final_sigdig.u64", sigma_digests(c));
    g_logging = false;
    const Fp d = dec_value(pk, sk, c);
    js << "],\n  \"stream\": " << st.size() << ", \"dec\": " << fpjson(d) << "\n}\n";
    std::ofstream(dir + "/chainx_manifest.json") << js.str();
}

// ---- the reference's OWN chain loop (tests/test_main.cpp:289-293): chain = enc_value(pk, sk, 2), then
//      chain = ct_mul(pk, chain, enc_value(pk, sk, 2)) for steps 1..depth, a FRESH operand per step (the
//      operand is encrypted before the ct_mul consumes it, so the stream interleaves enc, mul, enc, ...).
//      The stream is the interposed splitmix64 sequence from reseed(S): word j (0-based) is
//      splitmix64(S + (j + 1) * golden), so a consumer regenerates any stretch of it from S and j. The
//      manifest gives each step's enc and mul stretches, the product-layer nonce words at the head of
//      the mul stretch (2 |c_{k-1}.L| |y_k.L|), |E| / |L| of c_k and two commit_ct digests (ops/commit.hpp)
//      of c_k: with its sigmas and of a sigma-less copy (weights, layers, order).
//      full = true (chainf): also the whole stream, every operand (weights-only .ct), c_depth's .ct,
//      layer table and per-edge sigma digests. full = false (chainf8): the manifest only.
static Cipher strip_sigma(const Cipher& c) {
    Cipher w = c;
    for (auto& e : w.E) e.s = BitVec();
    return w;
}

static void cmd_chainf(const std::string& dir, int depth, bool full) {
    reseed(0x5EED0C00ULL);   // the same key as cmd_fixtures
    Params prm;
    PubKey pk;
    SecKey sk;
    g_logging = false;
    keygen(prm, pk, sk);
    (void)enc_value(pk, sk, 1);   // the Toeplitz autotuner's own draws stay out of the logged stream
    const std::string tag = full ? "chainf" : "chainf8";
    const uint64_t S = full ? 0x5EED0CF0ULL : 0x5EED0CF8ULL;
    reseed(S);
    g_logging = true;
    const size_t base = g_log.size();
    Cipher c = enc_value(pk, sk, 2);
    const size_t x_len = g_log.size() - base;
    if (full) write_ct(dir + "/" + tag + "_x.ct", {c}, false);
    std::ostringstream js;
    js << "{\n  \"canon_tag\": " << pk.canon_tag << ", \"depth\": " << depth << ", \"seed\": " << S
       << ", \"x_stream\": [0, " << x_len << "],\n  \"steps\": [\n";
    for (int k = 1; k <= depth; ++k) {
        const size_t e0 = g_log.size() - base;
        Cipher y = enc_value(pk, sk, 2);
        const size_t m0 = g_log.size() - base;
        const size_t nonce_words = 2 * c.L.size() * y.L.size();
        c = ct_mul(pk, c, y);
        const size_t m1 = g_log.size() - base;
        g_logging = false;
        const auto cm = commit_ct(pk, c), cw = commit_ct(pk, strip_sigma(c));
        g_logging = true;
        if (full) write_ct(dir + "/" + tag + "_y" + std::to_string(k) + ".ct", {y}, false);
        js << "    {\"enc_stream\": [" << e0 << ", " << (m0 - e0) << "], \"mul_stream\": [" << m0 << ", " << (m1 - m0)
           << "], \"nonce_words\": " << nonce_words << ", \"edges\": " << c.E.size() << ", \"layers\": "
           << c.L.size() << ", \"commit\": \"" << hex(cm.data(), 32) << "\", \"commit_weights\": \""
           << hex(cw.data(), 32) << "\"}" << (k < depth ? "," : "") << "\n";
        std::printf("%s step %d edges %zu layers %zu\n", tag.c_str(), k, c.E.size(), c.L.size());
        std::fflush(stdout);
    }
    g_logging = false;
    const Fp d = dec_value(pk, sk, c);
    js << "  ],\n  \"stream\": " << (g_log.size() - base) << ", \"dec\": " << fpjson(d) << "\n}\n";
    if (full) {
        write_u64(dir + "/" + tag + "_stream.u64", std::vector<uint64_t>(g_log.begin() + (long)base, g_log.end()));
        write_ct(dir + "/" + tag + "_final.ct", {c}, false);
        write_layers(dir + "/" + tag + "_final_layers.u64", c);
        write_u64(dir + "/" + tag + "_final_sigdig.u64", sigma_digests(c));
    }
    std::ofstream(dir + "/" + tag + "_manifest.json") << js.str();
}

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: ref_harness fp|fixtures|time_mul ...\n"); return 2; }
    std::string cmd = argv[1];
    if (cmd == "fp" && argc >= 3) { cmd_fp(argv[2]); return 0; }
    if (cmd == "fixtures" && argc >= 3) {
        int np = argc > 3 ? std::atoi(argv[3]) : 8;
        int cs = argc > 4 ? std::atoi(argv[4]) : 3;
        int ss = argc > 5 ? std::atoi(argv[5]) : 2;
        cmd_fixtures(argv[2], np, cs, ss);
        return 0;
    }
    if (cmd == "chainx" && argc >= 3) {
        cmd_chainx(argv[2], argc > 3 ? std::atoi(argv[3]) : 4);
        return 0;
    }
    if ((cmd == "chainf" || cmd == "chainf8") && argc >= 3) {
        cmd_chainf(argv[2], argc > 3 ? std::atoi(argv[3]) : (cmd == "chainf" ? 4 : 8), cmd == "chainf");
        return 0;
    }
    if (cmd == "encdepth" && argc >= 3) {
        cmd_encdepth(argv[2]);
        return 0;
    }
    if (cmd == "encdeep" && argc >= 3) {
        cmd_encdeep(argv[2]);
        return 0;
    }
    if (cmd == "fullrange" && argc >= 3) {
        cmd_fullrange(argv[2]);
        return 0;
    }
    if (cmd == "enc" && argc >= 3) {
        cmd_enc(argv[2], argc > 3 ? std::atoi(argv[3]) : 12);
        return 0;
    }
    if (cmd == "time_enc") {
        cmd_time_enc(argc > 2 ? std::atoi(argv[2]) : 16);
        return 0;
    }
    if (cmd == "time_chain") {
        cmd_time_chain(argc > 2 ? std::atoi(argv[2]) : 1, argc > 3 ? std::atoi(argv[3]) : 3);
        return 0;
    }
    if (cmd == "time_mul") {
        int np = argc > 2 ? std::atoi(argv[2]) : 64;
        int th = argc > 3 ? std::atoi(argv[3]) : 1;
        cmd_time_mul(np, th);
        return 0;
    }
    std::fprintf(stderr, "bad args\n");
    return 2;
}
