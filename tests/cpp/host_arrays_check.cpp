// host_arrays_check.cpp — CPU-only checks of the C++ adapter's host side (include/pvac_hip.hpp):
// the AoS <-> SoA conversion of reference-shaped Ciphers (detail::to_host / detail::convert_host,
// with and without sigma, over enough ciphers to take the threaded path) and the page-locked host
// arrays' fallback: without a GPU the runtime refuses to pin, so pinned_batch arrays must come from
// ordinary memory and go back to it (pinned_registry stays empty). Exit 0 = every check passed.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pvac_hip.hpp"

namespace mirror {   // the reference's member names and types (core/types.hpp:72-139)
struct Fp { uint64_t lo, hi; };
struct BitVec { size_t nbits = 0; std::vector<uint64_t> w; };
struct Nonce128 { uint64_t lo, hi; };
struct RSeed { uint64_t ztag; Nonce128 nonce; };
enum class RRule : uint8_t { BASE = 0, PROD = 1 };
struct Layer { RRule rule; RSeed seed; uint32_t pa; uint32_t pb; };
struct Edge { uint32_t layer_id; uint16_t idx; uint8_t ch; Fp w; BitVec s; };
struct Cipher { std::vector<Layer> L; std::vector<Edge> E; };
}  // namespace mirror

static int g_fail = 0;
#define CHECK(c, ...)                                   \
    do {                                                \
        if (!(c)) {                                     \
            std::fprintf(stderr, "FAIL %d: ", __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);          \
            std::fprintf(stderr, "\n");                 \
            ++g_fail;                                   \
        }                                               \
    } while (0)

static uint64_t g_state = 0x5EED0C0FFEEull;
static uint64_t rnd() {
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main() {
    using mirror::Cipher;
    const uint32_t sw = 128;   // sigma words at m_bits = 8192
    // ragged ciphers: 0..5 layers, 0..90 edges, some with sigma words of every length up to sw
    std::vector<Cipher> cs(3000);
    for (auto& c : cs) {
        c.L.resize(rnd() % 6);
        for (auto& l : c.L) {
            l.rule = rnd() & 1 ? mirror::RRule::PROD : mirror::RRule::BASE;
            l.seed.ztag = rnd();
            l.seed.nonce = {rnd(), rnd()};
            l.pa = (uint32_t)rnd();
            l.pb = (uint32_t)rnd();
        }
        c.E.resize(rnd() % 91);
        for (auto& e : c.E) {
            e.layer_id = (uint32_t)(rnd() % 64);
            e.idx = (uint16_t)(rnd() % 337);
            e.ch = (uint8_t)(rnd() & 1);
            e.w = {rnd(), rnd() >> 1};
            e.s.nbits = 8192;
            e.s.w.resize(rnd() % (sw + 1));
            for (auto& x : e.s.w) x = rnd();
        }
    }
    std::vector<const Cipher*> ptrs;
    for (auto& c : cs) ptrs.push_back(&c);
    for (int sig = 0; sig < 2; ++sig) {
        for (int pinned = 0; pinned < 2; ++pinned) {
            std::vector<Cipher> back;
            if (pinned) {
                pvac_hip::detail::pinned_batch b;
                pvac_hip::detail::to_host(ptrs, sw, sig != 0, b);
                back = pvac_hip::detail::convert_host<Cipher>(b, cs.size(), 8192, sig != 0);
                b.release();
            } else {
                pvac_hip::detail::batch b;
                pvac_hip::detail::to_host(ptrs, sw, sig != 0, b);
                back = pvac_hip::detail::convert_host<Cipher>(b, cs.size(), 8192, sig != 0);
            }
            CHECK(back.size() == cs.size(), "count");
            for (size_t i = 0; i < cs.size() && !g_fail; ++i) {
                const Cipher &a = cs[i], &r = back[i];
                CHECK(a.L.size() == r.L.size() && a.E.size() == r.E.size(), "shape of cipher %zu", i);
                for (size_t l = 0; l < a.L.size() && !g_fail; ++l)
                    CHECK(a.L[l].rule == r.L[l].rule && a.L[l].pa == r.L[l].pa && a.L[l].pb == r.L[l].pb &&
                              a.L[l].seed.ztag == r.L[l].seed.ztag && a.L[l].seed.nonce.lo == r.L[l].seed.nonce.lo &&
                              a.L[l].seed.nonce.hi == r.L[l].seed.nonce.hi,
                          "layer %zu of cipher %zu", l, i);
                for (size_t e = 0; e < a.E.size() && !g_fail; ++e) {
                    const auto &x = a.E[e], &y = r.E[e];
                    CHECK(x.layer_id == y.layer_id && x.idx == y.idx && x.ch == y.ch && x.w.lo == y.w.lo &&
                              x.w.hi == y.w.hi,
                          "edge %zu of cipher %zu", e, i);
                    if (sig) {
                        // sigma comes back at its full width, zero-padded past the input's words
                        CHECK(y.s.nbits == 8192 && y.s.w.size() == sw, "sigma width, edge %zu of cipher %zu", e, i);
                        for (uint32_t k = 0; k < sw && !g_fail; ++k)
                            CHECK(y.s.w[k] == (k < x.s.w.size() ? x.s.w[k] : 0ull), "sigma word %u", k);
                    } else {
                        CHECK(y.s.w.empty(), "weights-only edge with a sigma");
                    }
                }
            }
        }
    }
    {   // the pinned arrays' fallback: grow, shrink, swap, release; nothing left registered
        pvac_hip::detail::pinned_batch b;
        b.meta.resize(1 << 20);
        b.meta.resize(1 << 22);
        for (size_t i = 0; i < b.meta.size(); i += 4096) b.meta[i] = i;
        b.meta.resize(16);
        CHECK(b.meta[0] == 0, "contents kept across a grow");
        pvac_hip::detail::pinned_batch c;
        std::swap(b.meta, c.meta);
        CHECK(c.meta.size() == 16 && b.meta.empty(), "swap");
        b.release();
        c.release();
        auto& reg = pvac_hip::detail::pinned_registry::get();
        std::lock_guard<std::mutex> g(reg.mu);
        CHECK(reg.pinned.empty(), "%zu pinned allocations left registered", reg.pinned.size());
    }
    if (g_fail) return 1;
    std::printf("host_arrays_check: ok\n");
    return 0;
}
