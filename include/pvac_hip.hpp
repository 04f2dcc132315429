// pvac_hip.hpp — header-only C++17 adapter: the pvac-hfhe 0.1.0 by-value ciphertext API on top of
// the MI355X C ABI (pvac_hip.h / libpvac_hip.so).
//
// It is templated on the REFERENCE'S OWN types (include/pvac/core/types.hpp:72-139): any Cipher
// with `L` (Layer{rule, seed{ztag, nonce{lo, hi}}, pa, pb}) and `E` (Edge{layer_id, idx, ch,
// w{lo, hi}, s{nbits, w}}) vectors and any PubKey with `prm{B, m_bits, n_bits, h_col_wt,
// x_col_wt, err_wt, edge_budget}`, `canon_tag` and `H` (vector of BitVec columns). Nothing of
// the reference is copied; a maintainer routes the reference's functions here:
//
//   pvac::ct_mul(pk, A, B)  (ops/arithmetic.hpp:47)  -> pvac_hip::ct_mul(pk, A, B)
//   pvac::ct_add(pk, A, B)  (ops/arithmetic.hpp:12)  -> pvac_hip::ct_add(pk, A, B)
//   pvac::ct_sub(pk, A, B)  (ops/arithmetic.hpp:43)  -> pvac_hip::ct_sub(pk, A, B)
//   pvac::ct_scale(pk, A,s) (ops/arithmetic.hpp:33)  -> pvac_hip::ct_scale(pk, A, s)
//   pvac::ct_neg(pk, A)     (ops/arithmetic.hpp:39)  -> pvac_hip::ct_neg(pk, A)
//   pvac::ct_div_const(pk, A, k) (ops/arithmetic.hpp:108) -> pvac_hip::ct_div_const(pk, A, k)
//   pvac::enc_value(pk, sk, v) (ops/encrypt.hpp:289)  -> pvac_hip::enc_value<Cipher>(pk, sk, v)
//   pvac::dec_value(pk, sk, C) (ops/decrypt.hpp:62)  -> pvac_hip::dec_value(pk, sk, C)
//   saveCts / loadCts          (tests/add.cpp:22-155) -> pvac_hip::save_cts_bytes / load_cts_bytes
// plus batched forms (std::vector of pairs in, std::vector out) that keep one launch per batch.
// enc/dec also read pk.H_digest, pk.powg_B, pk.prm.lpn_* and the SecKey's prf_k / lpn_s_bits.
//
// Randomness: like the reference (core/random.hpp:40-110), nonces (2 words per new product
// layer, (la, lb) row-major, lo then hi) and salts (1 word per emitted edge, in emit order) come
// from getrandom(2) one 8-byte draw at a time, in the reference's order for a single ct_mul. A
// caller-supplied source (any callable returning uint64_t) replaces it for reproducible runs.
// Errors: C ABI status codes become pvac_hip::Error (the reference has no error codes and lets
// std::bad_alloc escape, arithmetic.hpp:76).
//
// Build: g++/hipcc -std=c++17 -I<repo>/include -I/opt/rocm/include -D__HIP_PLATFORM_AMD__
//        ... -L<repo>/pvac_hfhe_cppbyv_amd/lib -lpvac_hip -L/opt/rocm/lib -lamdhip64
#ifndef PVAC_HIP_HPP
#define PVAC_HIP_HPP

#include <hip/hip_runtime_api.h>
#include <sys/random.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <exception>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <thread>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "pvac_hip.h"

namespace pvac_hip {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

using RandomSource = std::function<uint64_t()>;

// One 8-byte getrandom per word, as csprng_u64 does (core/random.hpp:106-110).
inline uint64_t os_random_u64() {
    uint64_t v = 0;
    size_t got = 0;
    while (got < sizeof v) {
        const ssize_t r = getrandom(reinterpret_cast<uint8_t*>(&v) + got, sizeof v - got, 0);
        if (r <= 0) throw Error(PVAC_EDEVICE, "getrandom failed");
        got += (size_t)r;
    }
    return v;
}

namespace detail {

inline void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw Error(PVAC_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

// RAII device array of T; alloc() keeps the allocation when it already holds count elements, so
// an engine-owned array reused call after call stops paying hipMalloc / hipFree.
template <class T>
struct dev_array {
    T* p = nullptr;
    size_t n = 0, cap = 0;
    dev_array() = default;
    explicit dev_array(size_t count) { alloc(count); }
    dev_array(const dev_array&) = delete;
    dev_array& operator=(const dev_array&) = delete;
    dev_array(dev_array&& o) noexcept : p(o.p), n(o.n), cap(o.cap) { o.p = nullptr; o.n = o.cap = 0; }
    ~dev_array() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = cap = 0;
    }
    void alloc(size_t count) {
        n = count;
        if (p && count <= cap) return;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = count ? count : 1;
        hip_ok(hipMalloc(&p, cap * sizeof(T)), "hipMalloc");
    }
    void upload(const T* h, size_t count, hipStream_t s) {
        if (count) hip_ok(hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, s), "H2D");
    }
    void download(T* h, size_t count, hipStream_t s) const {
        if (count) hip_ok(hipMemcpyAsync(h, p, count * sizeof(T), hipMemcpyDeviceToHost, s), "D2H");
    }
};

// Host arrays that are filled right after they are sized (by a copy or a conversion loop): default-
// initialised, so sizing a few GB of output does not first zero it on one thread.
template <class T>
struct default_init : std::allocator<T> {
    template <class U>
    struct rebind { using other = default_init<U>; };
    using std::allocator<T>::allocator;
    default_init() noexcept = default;
    template <class U>
    default_init(const default_init<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) { ::new ((void*)p) U; }
    template <class U, class... Args>
    void construct(U* p, Args&&... args) { ::new ((void*)p) U(std::forward<Args>(args)...); }
};
template <class T>
using hvec = std::vector<T, default_init<T>>;

// The same, in page-locked host memory (hipHostMalloc): copies to and from the device run at the
// link's rate instead of through the runtime's pageable staging. Pinning is slow to set up, so only
// engine-owned arrays that are reused call after call use it. When the runtime refuses to pin (a
// locked-memory limit), the array is ordinary pageable memory instead: slower copies, same results.
struct pinned_registry {   // which live allocations are pinned (deallocate frees them the same way)
    std::mutex mu;
    std::set<void*> pinned;
    static pinned_registry& get() {
        static pinned_registry r;
        return r;
    }
};
template <class T>
struct pinned_alloc : default_init<T> {
    using value_type = T;
    template <class U>
    struct rebind { using other = pinned_alloc<U>; };
    pinned_alloc() noexcept = default;
    template <class U>
    pinned_alloc(const pinned_alloc<U>&) noexcept {}
    T* allocate(size_t count) {
        const size_t bytes = (count ? count : 1) * sizeof(T);
        void* q = nullptr;
        if (hipHostMalloc(&q, bytes, hipHostMallocDefault) == hipSuccess && q) {
            pinned_registry& r = pinned_registry::get();
            std::lock_guard<std::mutex> g(r.mu);
            r.pinned.insert(q);
            return static_cast<T*>(q);
        }
        (void)hipGetLastError();   // the refused pin must not surface as a later launch's error
        q = std::malloc(bytes);
        if (!q) throw std::bad_alloc();
        return static_cast<T*>(q);
    }
    void deallocate(T* q, size_t) noexcept {
        bool was_pinned = false;
        {
            pinned_registry& r = pinned_registry::get();
            std::lock_guard<std::mutex> g(r.mu);
            was_pinned = r.pinned.erase((void*)q) != 0;
        }
        if (was_pinned)
            (void)hipHostFree(q);
        else
            std::free(q);
    }
    template <class U>
    bool operator==(const pinned_alloc<U>&) const noexcept { return true; }
    template <class U>
    bool operator!=(const pinned_alloc<U>&) const noexcept { return false; }
};

// Host SoA image of a batch of reference Ciphers + its device copy.
template <bool Pinned>
struct basic_batch {
    template <class T>
    using vec = std::vector<T, typename std::conditional<Pinned, pinned_alloc<T>, default_init<T>>::type>;
    vec<uint64_t> l_off, l_cnt, e_off, e_cnt, meta, w_lo, w_hi, sigma;
    vec<pvac_layer> layers;
    dev_array<uint64_t> d_l_off, d_l_cnt, d_e_off, d_e_cnt, d_meta, d_w_lo, d_w_hi, d_sigma;
    dev_array<pvac_layer> d_layers;
    uint32_t sigma_words = 0;

    // frees every host and device array (an engine-owned batch between calls)
    void release() {
        basic_batch e;
        std::swap(l_off, e.l_off); std::swap(l_cnt, e.l_cnt); std::swap(e_off, e.e_off); std::swap(e_cnt, e.e_cnt);
        std::swap(meta, e.meta); std::swap(w_lo, e.w_lo); std::swap(w_hi, e.w_hi); std::swap(sigma, e.sigma);
        std::swap(layers, e.layers);
        for (auto* d : {&d_l_off, &d_l_cnt, &d_e_off, &d_e_cnt, &d_meta, &d_w_lo, &d_w_hi, &d_sigma}) d->release();
        d_layers.release();
    }

    pvac_ct_batch view(bool with_sigma) {
        pvac_ct_batch b{};
        b.n = l_cnt.size();
        b.l_off = d_l_off.p; b.l_cnt = d_l_cnt.p; b.layers = d_layers.p;
        b.e_off = d_e_off.p; b.e_cnt = d_e_cnt.p;
        b.meta = d_meta.p; b.w_lo = d_w_lo.p; b.w_hi = d_w_hi.p;
        b.sigma = with_sigma ? d_sigma.p : nullptr;
        b.sigma_words = sigma_words;
        return b;
    }
};
using batch = basic_batch<false>;
using pinned_batch = basic_batch<true>;

// Runs f(begin, end) over [0, n) on up to hardware_concurrency() threads (AoS <-> SoA conversion
// of large batches; each cipher is independent).
template <class F>
void parallel_ranges(size_t n, F f) {
    const size_t hw = std::max<size_t>(1, std::thread::hardware_concurrency());
    const size_t nt = std::min<size_t>(std::min<size_t>(hw, 32), n / 256 + 1);
    if (nt <= 1) { f(size_t(0), n); return; }
    std::vector<std::thread> th;
    const size_t per = (n + nt - 1) / nt;
    for (size_t t = 0; t < nt; ++t) {
        const size_t b = t * per, e = std::min(n, b + per);
        if (b < e) th.emplace_back([=, &f]() { f(b, e); });
    }
    for (auto& x : th) x.join();
}

template <class CipherT, class Batch>
void to_host(const std::vector<const CipherT*>& cs, uint32_t sigma_words, bool with_sigma, Batch& b) {
    const size_t n = cs.size();
    b.sigma_words = sigma_words;
    b.l_off.resize(n); b.l_cnt.resize(n); b.e_off.resize(n); b.e_cnt.resize(n);
    uint64_t lo = 0, eo = 0;
    for (size_t i = 0; i < n; ++i) {
        b.l_off[i] = lo; b.l_cnt[i] = cs[i]->L.size(); lo += cs[i]->L.size();
        b.e_off[i] = eo; b.e_cnt[i] = cs[i]->E.size(); eo += cs[i]->E.size();
    }
    b.layers.resize(lo);
    b.meta.resize(eo); b.w_lo.resize(eo); b.w_hi.resize(eo);
    if (with_sigma) b.sigma.assign(eo * sigma_words, 0);
    parallel_ranges(n, [&](size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i) {
            const CipherT* c = cs[i];
            size_t l = b.l_off[i], e = b.e_off[i];
            for (const auto& L : c->L) {
                pvac_layer& y = b.layers[l++];
                y.rule = (uint32_t)L.rule; y.pa = L.pa; y.pb = L.pb; y.pad = 0;
                y.ztag = L.seed.ztag; y.nonce_lo = L.seed.nonce.lo; y.nonce_hi = L.seed.nonce.hi;
            }
            for (const auto& E : c->E) {
                b.meta[e] = (uint64_t)E.layer_id | ((uint64_t)E.idx << 32) | ((uint64_t)E.ch << 48);
                b.w_lo[e] = E.w.lo; b.w_hi[e] = E.w.hi;
                if (with_sigma) {
                    const size_t k = std::min<size_t>(E.s.w.size(), sigma_words);
                    if (k) std::memcpy(&b.sigma[e * sigma_words], E.s.w.data(), k * 8);
                }
                ++e;
            }
        }
    });
}

template <class Batch>
void upload(Batch& b, hipStream_t s, bool with_sigma) {
    b.d_l_off.alloc(b.l_off.size()); b.d_l_off.upload(b.l_off.data(), b.l_off.size(), s);
    b.d_l_cnt.alloc(b.l_cnt.size()); b.d_l_cnt.upload(b.l_cnt.data(), b.l_cnt.size(), s);
    b.d_e_off.alloc(b.e_off.size()); b.d_e_off.upload(b.e_off.data(), b.e_off.size(), s);
    b.d_e_cnt.alloc(b.e_cnt.size()); b.d_e_cnt.upload(b.e_cnt.data(), b.e_cnt.size(), s);
    b.d_layers.alloc(b.layers.size()); b.d_layers.upload(b.layers.data(), b.layers.size(), s);
    b.d_meta.alloc(b.meta.size()); b.d_meta.upload(b.meta.data(), b.meta.size(), s);
    b.d_w_lo.alloc(b.w_lo.size()); b.d_w_lo.upload(b.w_lo.data(), b.w_lo.size(), s);
    b.d_w_hi.alloc(b.w_hi.size()); b.d_w_hi.upload(b.w_hi.data(), b.w_hi.size(), s);
    if (with_sigma) { b.d_sigma.alloc(b.sigma.size()); b.d_sigma.upload(b.sigma.data(), b.sigma.size(), s); }
}

// Output records of capacity layer/edge slots; the per-cipher offset/count arrays were
// allocated before the plan (which writes the offsets) and are kept.
template <class Batch>
void alloc_out(Batch& c, size_t n, uint64_t lslots, uint64_t eslots, uint32_t sigma_words, bool with_sigma) {
    c.sigma_words = sigma_words;
    c.d_layers.alloc(lslots);
    c.d_meta.alloc(eslots); c.d_w_lo.alloc(eslots); c.d_w_hi.alloc(eslots);
    if (with_sigma) c.d_sigma.alloc(eslots * sigma_words);
    c.l_cnt.resize(n);
}

// host SoA image (c.l_off ... c.sigma filled) -> reference Ciphers
template <class CipherT, class Batch>
std::vector<CipherT> convert_host(Batch& c, size_t n, uint32_t m_bits, bool with_sigma) {
    std::vector<CipherT> out(n);
    parallel_ranges(n, [&](size_t i0, size_t i1) {
    for (size_t i = i0; i < i1; ++i) {
        CipherT& C = out[i];
        C.L.resize(c.l_cnt[i]);
        for (size_t l = 0; l < c.l_cnt[i]; ++l) {
            const pvac_layer& y = c.layers[c.l_off[i] + l];
            auto& L = C.L[l];
            L.rule = static_cast<decltype(L.rule)>(y.rule);
            L.pa = y.pa; L.pb = y.pb;
            L.seed.ztag = y.ztag; L.seed.nonce.lo = y.nonce_lo; L.seed.nonce.hi = y.nonce_hi;
        }
        C.E.resize(c.e_cnt[i]);
        for (size_t k = 0; k < c.e_cnt[i]; ++k) {
            const size_t e = c.e_off[i] + k;
            auto& E = C.E[k];
            E.layer_id = (uint32_t)c.meta[e];
            E.idx = (uint16_t)(c.meta[e] >> 32);
            E.ch = (uint8_t)(c.meta[e] >> 48);
            E.w.lo = c.w_lo[e]; E.w.hi = c.w_hi[e];
            // weights-only results (an engine extension: the reference always draws sigma) keep an
            // empty BitVec instead of a zeroed m_bits one (1 KiB per edge); save_cts zero-pads it
            if (with_sigma) {
                E.s.nbits = m_bits;
                E.s.w.assign(&c.sigma[e * c.sigma_words], &c.sigma[e * c.sigma_words] + c.sigma_words);
            }
        }
    }
    });
    return out;
}

// device records of d (lslots / eslots rows) -> host SoA image c, synchronous
template <class Batch, class Dev>
void download(Batch& c, const Dev& d, size_t n, uint64_t lslots, uint64_t eslots, bool with_sigma, hipStream_t s) {
    c.sigma_words = d.sigma_words;
    c.l_off.resize(n); c.l_cnt.resize(n); c.e_off.resize(n); c.e_cnt.resize(n);
    c.layers.resize(lslots); c.meta.resize(eslots); c.w_lo.resize(eslots); c.w_hi.resize(eslots);
    d.d_l_off.download(c.l_off.data(), n, s); d.d_l_cnt.download(c.l_cnt.data(), n, s);
    d.d_e_off.download(c.e_off.data(), n, s); d.d_e_cnt.download(c.e_cnt.data(), n, s);
    d.d_layers.download(c.layers.data(), lslots, s);
    d.d_meta.download(c.meta.data(), eslots, s);
    d.d_w_lo.download(c.w_lo.data(), eslots, s); d.d_w_hi.download(c.w_hi.data(), eslots, s);
    if (with_sigma) {
        c.sigma.resize(eslots * c.sigma_words);
        d.d_sigma.download(c.sigma.data(), c.sigma.size(), s);
    }
    hip_ok(hipStreamSynchronize(s), "sync");
}

template <class CipherT>
std::vector<CipherT> from_device(batch& c, size_t n, uint64_t lslots, uint64_t eslots, uint32_t m_bits,
                                 bool with_sigma, hipStream_t s) {
    download(c, c, n, lslots, eslots, with_sigma, s);
    return convert_host<CipherT>(c, n, m_bits, with_sigma);
}

// small synchronous device -> host copies of a batch view handed to a chain hook (valid only there)
inline hvec<uint64_t> d2h_u64(const uint64_t* p, size_t n, hipStream_t s) {
    hvec<uint64_t> v(n);
    if (n) hip_ok(hipMemcpyAsync(v.data(), p, n * 8, hipMemcpyDeviceToHost, s), "D2H");
    hip_ok(hipStreamSynchronize(s), "sync");
    return v;
}

// the used rows of a capacity-padded device batch view -> reference Ciphers
template <class CipherT>
std::vector<CipherT> from_view(const pvac_ct_batch& v, uint32_t m_bits, hipStream_t s) {
    batch c;
    const size_t n = v.n;
    c.l_off = d2h_u64(v.l_off, n, s); c.l_cnt = d2h_u64(v.l_cnt, n, s);
    c.e_off = d2h_u64(v.e_off, n, s); c.e_cnt = d2h_u64(v.e_cnt, n, s);
    uint64_t nl = 0, ne = 0;
    for (size_t i = 0; i < n; ++i) {
        nl = std::max(nl, c.l_off[i] + c.l_cnt[i]);
        ne = std::max(ne, c.e_off[i] + c.e_cnt[i]);
    }
    const bool sig = v.sigma != nullptr;
    c.sigma_words = v.sigma_words;
    c.layers.resize(nl); c.meta.resize(ne); c.w_lo.resize(ne); c.w_hi.resize(ne);
    if (sig) c.sigma.resize(ne * c.sigma_words);
    auto get = [&](void* dst, const void* src, size_t bytes) {
        if (bytes) hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s), "D2H");
    };
    get(c.layers.data(), v.layers, nl * sizeof(pvac_layer));
    get(c.meta.data(), v.meta, ne * 8); get(c.w_lo.data(), v.w_lo, ne * 8); get(c.w_hi.data(), v.w_hi, ne * 8);
    if (sig) get(c.sigma.data(), v.sigma, c.sigma.size() * 8);
    hip_ok(hipStreamSynchronize(s), "sync");
    return convert_host<CipherT>(c, n, m_bits, sig);
}

}  // namespace detail

// One device context per (device, canon_tag); owns the device copy of pk.H for sigma.
class Engine {
public:
    Engine(int device, const pvac_hip_params& prm) : prm_(prm) {
        const int rc = pvac_hip_ctx_create(device, &prm, &ctx_);
        if (rc) throw Error(rc, "pvac_hip_ctx_create failed (no MI355X / HIP runtime?)");
        stream_ = (hipStream_t)pvac_hip_ctx_stream(ctx_);
    }
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;
    ~Engine() {
        if (stream_) (void)hipStreamSynchronize(stream_);
        mul_a_.release(); mul_b_.release(); mul_c_.release(); mul_p_.release();
        mul_nonces_.release(); mul_salts_.release(); mul_status_.release();
        pvac_hip_ctx_destroy(ctx_);
    }

    template <class PubKeyT>
    static pvac_hip_params params_of(const PubKeyT& pk) {
        pvac_hip_params p{};
        p.B = (uint32_t)pk.prm.B; p.m_bits = (uint32_t)pk.prm.m_bits; p.n_bits = (uint32_t)pk.prm.n_bits;
        p.h_col_wt = (uint32_t)pk.prm.h_col_wt; p.x_col_wt = (uint32_t)pk.prm.x_col_wt;
        p.err_wt = (uint32_t)pk.prm.err_wt; p.edge_budget = (uint64_t)pk.prm.edge_budget;
        p.canon_tag = pk.canon_tag;
        return p;
    }

    pvac_hip_ctx* ctx() const { return ctx_; }
    uint32_t sigma_words() const { return (prm_.m_bits + 63) / 64; }

    // Wall-clock split of the last batched ct_mul, in seconds: host AoS -> SoA, H2D, plan + nonce
    // draws, exec (+ salts, sigma and the device-side pack of the used rows), D2H, SoA -> AoS.
    struct Phases { double to_soa = 0, h2d = 0, plan = 0, exec = 0, d2h = 0, to_aos = 0; };
    const Phases& last_phases() const { return phases_; }

    // Batched ct_mul keeps its host (pinned) and device arrays between calls, sized by the largest
    // batch so far; trim() hands them back.
    void trim() {
        detail::hip_ok(hipStreamSynchronize(stream_), "sync");
        mul_a_.release(); mul_b_.release(); mul_c_.release(); mul_p_.release();
        mul_nonces_.release(); mul_salts_.release(); mul_status_.release();
    }

    // H regenerated on the device from canon_tag (gen_H, crypto/matrix.hpp:191-251); returns the
    // H_digest for comparison with pk.H_digest.
    std::vector<uint8_t> gen_H() {
        std::vector<uint8_t> d(32);
        check(pvac_hip_ctx_gen_H(ctx_, d.data()));
        h_ready_ = true;
        return d;
    }

    // pk.H (dense BitVec columns) -> device sparse columns, once; an empty pk.H (e.g. a key
    // loaded without H) is regenerated on the device from canon_tag.
    template <class PubKeyT>
    void ensure_H(const PubKeyT& pk) {
        if (h_ready_) return;
        if (pk.H.empty()) {
            (void)gen_H();
            return;
        }
        const uint32_t wpc = sigma_words();
        std::vector<uint64_t> dense((size_t)pk.H.size() * wpc, 0);
        for (size_t c = 0; c < pk.H.size(); ++c)
            std::memcpy(&dense[c * wpc], pk.H[c].w.data(), std::min<size_t>(pk.H[c].w.size(), wpc) * 8);
        check(pvac_hip_ctx_set_H(ctx_, dense.data(), (uint32_t)pk.H.size(), wpc));
        h_ready_ = true;
    }

    // Batched ct_mul (ops/arithmetic.hpp:47-106) over pairs (A[i], B[i]). with_sigma needs pk.H.
    template <class PubKeyT, class CipherT>
    std::vector<CipherT> ct_mul(const PubKeyT& pk, const std::vector<const CipherT*>& A,
                                const std::vector<const CipherT*>& B, bool with_sigma, const RandomSource& rnd) {
        if (A.size() != B.size()) throw Error(PVAC_EINVAL, "ct_mul: |A| != |B|");
        const size_t n = A.size();
        if (!n) return {};
        if (with_sigma) ensure_H(pk);
        using clk = std::chrono::steady_clock;
        auto t = clk::now();
        auto lap = [&t](double& into) {
            const auto u = clk::now();
            into = std::chrono::duration<double>(u - t).count();
            t = u;
        };
        // engine-owned (pinned, grow-only) arrays: a steady stream of batches maps, pins and frees nothing
        detail::pinned_batch& a = mul_a_;
        detail::pinned_batch& b = mul_b_;
        detail::pinned_batch& c = mul_c_;
        detail::to_host(A, sigma_words(), false, a);
        detail::to_host(B, sigma_words(), false, b);
        lap(phases_.to_soa);
        detail::upload(a, stream_, false);
        detail::upload(b, stream_, false);
        detail::hip_ok(hipStreamSynchronize(stream_), "sync");
        lap(phases_.h2d);
        pvac_ct_batch va = a.view(false), vb = b.view(false);
        c.d_l_off.alloc(n); c.d_l_cnt.alloc(n); c.d_e_off.alloc(n); c.d_e_cnt.alloc(n);
        pvac_ct_batch vc{};
        vc.l_off = c.d_l_off.p; vc.l_cnt = c.d_l_cnt.p; vc.e_off = c.d_e_off.p; vc.e_cnt = c.d_e_cnt.p;
        pvac_hip_plan plan{};
        check(pvac_hip_ct_mul_plan(ctx_, &va, &vb, &vc, &plan));
        // nonces per pair in the reference's draw order: (la, lb) row-major, lo then hi
        std::vector<uint64_t> loff(n);
        c.d_l_off.download(loff.data(), n, stream_);
        detail::hip_ok(hipStreamSynchronize(stream_), "sync");
        std::vector<uint64_t> nonces(2 * (plan.total_layer_slots ? plan.total_layer_slots : 1), 0);
        for (size_t i = 0; i < n; ++i) {
            const uint64_t LA = A[i]->L.size(), LB = B[i]->L.size();
            const uint64_t s0 = loff[i] + LA + LB;
            for (uint64_t k = 0; k < LA * LB; ++k) {
                nonces[2 * (s0 + k)] = rnd();
                nonces[2 * (s0 + k) + 1] = rnd();
            }
        }
        detail::dev_array<uint64_t>& d_nonces = mul_nonces_;
        d_nonces.alloc(nonces.size());
        d_nonces.upload(nonces.data(), nonces.size(), stream_);
        detail::alloc_out(c, n, plan.total_layer_slots, plan.total_edge_slots, sigma_words(), with_sigma);
        lap(phases_.plan);
        vc = c.view(false);
        vc.n = n;
        check(pvac_hip_ct_mul_exec(ctx_, &plan, &va, &vb, d_nonces.p, nullptr, &vc, 0));
        if (with_sigma) {
            // one salt per emitted edge, drawn after the weights are known (arithmetic.hpp:90-94), in
            // emit order. In the reference hash order (pair status 0) output position k of a pair IS
            // its k-th emit, so sigma_from_H runs over the finished batch (pvac_hip_sigma_batch);
            // a pair in the canonical order (guard_budget) takes its salts in hash order, which the
            // second exec with PVAC_MUL_WITH_SIGMA maps (salt positions)
            std::vector<uint64_t> ecnt(n), eoff(n);
            std::vector<uint32_t> status(n);
            detail::dev_array<uint32_t>& d_status = mul_status_;
            d_status.alloc(n);
            check(pvac_hip_ct_mul_status(ctx_, d_status.p, n));
            c.d_e_cnt.download(ecnt.data(), n, stream_);
            c.d_e_off.download(eoff.data(), n, stream_);
            d_status.download(status.data(), n, stream_);
            detail::hip_ok(hipStreamSynchronize(stream_), "sync");
            std::vector<uint64_t> salts(plan.total_edge_slots ? plan.total_edge_slots : 1, 0);
            bool hash_order = true;
            for (size_t i = 0; i < n; ++i) {
                hash_order &= status[i] != 1u;
                for (uint64_t k = 0; k < ecnt[i]; ++k) salts[eoff[i] + k] = rnd();
            }
            detail::dev_array<uint64_t>& d_salts = mul_salts_;
            d_salts.alloc(salts.size());
            d_salts.upload(salts.data(), salts.size(), stream_);
            vc = c.view(true);
            vc.n = n;
            if (hash_order) {
                check(pvac_hip_sigma_batch(ctx_, &vc, d_salts.p));
            } else {
                check(pvac_hip_ct_mul_plan(ctx_, &va, &vb, &vc, &plan));
                vc = c.view(true);
                vc.n = n;
                check(pvac_hip_ct_mul_exec(ctx_, &plan, &va, &vb, d_nonces.p, d_salts.p, &vc, PVAC_MUL_WITH_SIGMA));
            }
        }
        // only the used rows cross the link: packed on the device first (each pair's output kept its
        // plan capacity), then copied at their exact totals
        detail::pinned_batch& p = mul_p_;
        p.d_l_off.alloc(n); p.d_l_cnt.alloc(n); p.d_e_off.alloc(n); p.d_e_cnt.alloc(n);
        detail::alloc_out(p, n, plan.total_layer_slots, plan.total_edge_slots, sigma_words(), with_sigma);
        vc = c.view(with_sigma);
        vc.n = n;
        pvac_ct_batch vp = p.view(with_sigma);
        uint64_t tot[2] = {0, 0};
        check(pvac_hip_batch_pack(ctx_, &vc, &vp, tot));
        lap(phases_.exec);
        detail::download(c, p, n, tot[0], tot[1], with_sigma, stream_);
        lap(phases_.d2h);
        std::vector<CipherT> out = detail::convert_host<CipherT>(c, n, prm_.m_bits, with_sigma);
        lap(phases_.to_aos);
        return out;
    }

    // Depth chains through pvac_hip_ct_mul_chain (the chain entry point): for every input x of xs,
    // c_0 = x, c_k = ct_mul(pk, c_{k-1}, x) for k = 1..depth (the test_depth / cfg-4 shape of
    // tests/test_main.cpp:289-293's loop); returns every c_depth. Randomness of chain i comes from
    // rnds[i] in the reference's draw order, step after step: 2 words per new product layer (la, lb
    // row-major, lo then hi), then one salt per emitted edge (arithmetic.hpp:64, 93). Only c_depth's
    // sigmas survive a chain, so the intermediate salts are drawn and discarded; with_sigma computes
    // the final step's sigmas (needs pk.H), otherwise the final salts are discarded too. A chain
    // replayed from a reference stream is byte-identical to the reference's c_depth. devices: GPU
    // ordinals to spread the chains over (whole chunks per device; empty = this engine's device);
    // chunk: inputs per worker chunk (with sigma the last step holds 1 KiB per edge: keep it small).
    // ops (optional): per-step operands, ops[d][i] the cipher chain i multiplies by at step d + 1
    // (the reference's own loop, tests/test_main.cpp:291-292, multiplies by a fresh enc_value(2) per
    // step); steps past ops.size() multiply by x. rnds then carry only the ct_mul draws: a caller
    // replaying one interleaved stream encrypts the operands from their own stretches of it.
    template <class PubKeyT, class CipherT>
    std::vector<CipherT> ct_mul_chain(const PubKeyT& pk, const std::vector<const CipherT*>& xs, uint32_t depth,
                                      bool with_sigma, std::vector<RandomSource>& rnds,
                                      const std::vector<int>& devices = {}, uint32_t streams = 2, uint64_t chunk = 16,
                                      const std::vector<std::vector<const CipherT*>>& ops = {}) {
        const size_t n = xs.size();
        if (rnds.size() != n) throw Error(PVAC_EINVAL, "ct_mul_chain: one RandomSource per input");
        if (ops.size() > depth) throw Error(PVAC_EINVAL, "ct_mul_chain: more operand steps than depth");
        for (const auto& y : ops)
            if (y.size() != n) throw Error(PVAC_EINVAL, "ct_mul_chain: one operand per input and step");
        if (!n) return {};
        if (with_sigma) ensure_H(pk);
        detail::batch x;
        detail::to_host(xs, sigma_words(), false, x);
        detail::upload(x, stream_, false);
        std::vector<detail::batch> yb(ops.size());
        std::vector<pvac_ct_batch> yv(ops.size());
        for (size_t d = 0; d < ops.size(); ++d) {
            detail::to_host(ops[d], sigma_words(), false, yb[d]);
            detail::upload(yb[d], stream_, false);
            yv[d] = yb[d].view(false);
        }
        detail::hip_ok(hipStreamSynchronize(stream_), "sync");
        struct state {
            std::vector<RandomSource>* rnds;
            std::vector<CipherT> out;
            uint32_t depth, m_bits;
            bool sigma;
        } stt{&rnds, std::vector<CipherT>(n), depth, prm_.m_bits, with_sigma};
        pvac_chain_opts o{};
        o.depth = depth;
        o.streams = streams;
        o.chunk = chunk;
        o.flags = with_sigma ? PVAC_MUL_WITH_SIGMA : 0u;
        o.user = &stt;
        o.devices = devices.empty() ? nullptr : devices.data();
        o.n_devices = (uint32_t)devices.size();
        o.operands = yv.empty() ? nullptr : yv.data();
        o.n_operands = (uint32_t)yv.size();
        // hooks run on the library's worker threads; chunks (and so their inputs' sources) are disjoint
        o.nonces_at = [](void* u, uint32_t, uint64_t c0, const pvac_ct_batch* A, const pvac_ct_batch* X,
                         const pvac_ct_batch* C, uint64_t* words, uint64_t nw, void* st) -> int {
            try {
                state& S = *(state*)u;
                const hipStream_t s = (hipStream_t)st;
                const auto la = detail::d2h_u64(A->l_cnt, A->n, s), lx = detail::d2h_u64(X->l_cnt, X->n, s);
                const auto lo = detail::d2h_u64(C->l_off, C->n, s);
                std::vector<uint64_t> w(nw, 0);
                for (size_t i = 0; i < A->n; ++i) {
                    RandomSource& r = (*S.rnds)[c0 + i];
                    const uint64_t s0 = lo[i] + la[i] + lx[i];
                    for (uint64_t k = 0; k < la[i] * lx[i]; ++k) {
                        w[2 * (s0 + k)] = r();
                        w[2 * (s0 + k) + 1] = r();
                    }
                }
                detail::hip_ok(hipMemcpyAsync(words, w.data(), nw * 8, hipMemcpyHostToDevice, s), "H2D");
                detail::hip_ok(hipStreamSynchronize(s), "sync");
                return 0;
            } catch (...) {
                return 1;
            }
        };
        o.after_step = [](void* u, uint32_t step, uint64_t c0, const pvac_ct_batch*, const pvac_ct_batch*,
                          const pvac_ct_batch* C, uint64_t*, uint64_t, void* st) -> int {
            try {
                state& S = *(state*)u;
                if (S.sigma && step + 1 == S.depth) return 0;   // salts_at draws these
                const auto ec = detail::d2h_u64(C->e_cnt, C->n, (hipStream_t)st);
                for (size_t i = 0; i < C->n; ++i)
                    for (uint64_t k = 0; k < ec[i]; ++k) (void)(*S.rnds)[c0 + i]();
                return 0;
            } catch (...) {
                return 1;
            }
        };
        o.salts_at = [](void* u, uint32_t, uint64_t c0, const pvac_ct_batch*, const pvac_ct_batch*,
                        const pvac_ct_batch* C, uint64_t* words, uint64_t nw, void* st) -> int {
            try {
                state& S = *(state*)u;
                const hipStream_t s = (hipStream_t)st;
                const auto ec = detail::d2h_u64(C->e_cnt, C->n, s), eo = detail::d2h_u64(C->e_off, C->n, s);
                std::vector<uint64_t> w(nw ? nw : 1, 0);
                for (size_t i = 0; i < C->n; ++i)
                    for (uint64_t k = 0; k < ec[i]; ++k) w[eo[i] + k] = (*S.rnds)[c0 + i]();
                detail::hip_ok(hipMemcpyAsync(words, w.data(), nw * 8, hipMemcpyHostToDevice, s), "H2D");
                detail::hip_ok(hipStreamSynchronize(s), "sync");
                return 0;
            } catch (...) {
                return 1;
            }
        };
        o.on_chunk = [](void* u, uint64_t c0, const pvac_ct_batch* C, void* st) -> int {
            try {
                state& S = *(state*)u;
                auto cs = detail::from_view<CipherT>(*C, S.m_bits, (hipStream_t)st);
                for (size_t i = 0; i < cs.size(); ++i) S.out[c0 + i] = std::move(cs[i]);
                return 0;
            } catch (...) {
                return 1;
            }
        };
        pvac_ct_batch vx = x.view(false);
        pvac_chain_stats st{};
        check(pvac_hip_ct_mul_chain(ctx_, &vx, &o, &st));
        return std::move(stt.out);
    }

    // Batched ct_add / ct_sub (ops/arithmetic.hpp:12-31, 43-45); sigmas carried through.
    template <class CipherT>
    std::vector<CipherT> ct_add(const std::vector<const CipherT*>& A, const std::vector<const CipherT*>& B, bool negate_b) {
        if (A.size() != B.size()) throw Error(PVAC_EINVAL, "ct_add: |A| != |B|");
        const size_t n = A.size();
        if (!n) return {};
        detail::batch a, b, c;
        detail::to_host(A, sigma_words(), true, a);
        detail::to_host(B, sigma_words(), true, b);
        detail::upload(a, stream_, true);
        detail::upload(b, stream_, true);
        pvac_ct_batch va = a.view(true), vb = b.view(true);
        c.d_l_off.alloc(n); c.d_l_cnt.alloc(n); c.d_e_off.alloc(n); c.d_e_cnt.alloc(n);
        pvac_ct_batch vc{};
        vc.l_off = c.d_l_off.p; vc.l_cnt = c.d_l_cnt.p; vc.e_off = c.d_e_off.p; vc.e_cnt = c.d_e_cnt.p;
        pvac_hip_plan plan{};
        check(pvac_hip_ct_add_plan(ctx_, &va, &vb, &vc, &plan));
        detail::alloc_out(c, n, plan.total_layer_slots, plan.total_edge_slots, sigma_words(), true);
        vc = c.view(true);
        vc.n = n;
        check(pvac_hip_ct_add_exec(ctx_, &plan, &va, &vb, negate_b ? 1 : 0, &vc));
        return detail::from_device<CipherT>(c, n, plan.total_layer_slots, plan.total_edge_slots, prm_.m_bits, true,
                                            stream_);
    }

    // Element-wise Fp over host arrays (core/field.hpp:50-71, 209-213), one launch.
    void fp_binop(int op, const uint64_t* a_lo, const uint64_t* a_hi, const uint64_t* b_lo, const uint64_t* b_hi,
                  uint64_t* c_lo, uint64_t* c_hi, size_t n) {
        if (!n) return;
        detail::dev_array<uint64_t> d[6];
        for (auto& x : d) x.alloc(n);
        d[0].upload(a_lo, n, stream_); d[1].upload(a_hi, n, stream_);
        const size_t nb = op == PVAC_FP_SCALE ? 1 : n;
        if (op != PVAC_FP_NEG && op != PVAC_FP_INV) { d[2].upload(b_lo, nb, stream_); d[3].upload(b_hi, nb, stream_); }
        check(pvac_hip_fp_binop(ctx_, op, d[0].p, d[1].p, d[2].p, d[3].p, d[4].p, d[5].p, n));
        d[4].download(c_lo, n, stream_); d[5].download(c_hi, n, stream_);
        detail::hip_ok(hipStreamSynchronize(stream_), "sync");
    }

    // Key material of enc_value / dec_value (core/types.hpp:121-137): pk.H_digest and pk.powg_B
    // from the PubKey, prf_k and lpn_s_bits from the SecKey. Uploaded once; a different SecKey
    // under the same canon_tag replaces the device copy.
    template <class PubKeyT, class SecKeyT>
    void ensure_keys(const PubKeyT& pk, const SecKeyT& sk) {
        // plan_noise's Params fields (core/types.hpp:48-50), read on every call like the reference
        check(pvac_hip_ctx_set_noise(ctx_, (double)pk.prm.noise_entropy_bits, (double)pk.prm.tuple2_fraction,
                                     (double)pk.prm.depth_slope_bits));
        const std::vector<uint64_t> fp = key_fingerprint(sk);
        if (keys_ready_ && fp == key_fp_) return;
        if (!keys_ready_) {
            check(pvac_hip_ctx_set_H_digest(ctx_, pk.H_digest.data()));
            std::vector<uint64_t> pg(2 * pk.powg_B.size());
            for (size_t i = 0; i < pk.powg_B.size(); ++i) { pg[2 * i] = pk.powg_B[i].lo; pg[2 * i + 1] = pk.powg_B[i].hi; }
            check(pvac_hip_ctx_set_powg(ctx_, pg.data(), (uint32_t)pk.powg_B.size()));
        }
        check(pvac_hip_ctx_set_secret(ctx_, sk.prf_k.data(), sk.lpn_s_bits.data(), (uint32_t)pk.prm.lpn_n,
                                      (uint32_t)pk.prm.lpn_t, (uint32_t)pk.prm.lpn_tau_num,
                                      (uint32_t)pk.prm.lpn_tau_den));
        key_fp_ = fp;
        keys_ready_ = true;
    }

    // Batched enc_value (ops/encrypt.hpp:281-290, depth hint 0). Value i takes `stride`
    // (enc_caps draws_hint) consecutive words of rnd, in the reference's draw order, so a single
    // value encrypted from a replayed getrandom stream is byte-identical to the reference's; the
    // source is advanced by the whole stride. A value whose rejection sampling outruns its stride
    // (status 1, never seen in practice) is re-run with its own draws extended, prefix kept.
    // depth_hint > 0: enc_value_depth (encrypt.hpp:281-287); a value of 0 is enc_zero_depth (:293-298).
    template <class PubKeyT, class SecKeyT, class CipherT>
    std::vector<CipherT> enc_value(const PubKeyT& pk, const SecKeyT& sk, const std::vector<uint64_t>& vs,
                                   bool with_sigma, const RandomSource& rnd, int depth_hint = 0) {
        const size_t n = vs.size();
        if (!n) return {};
        ensure_keys(pk, sk);
        if (with_sigma) ensure_H(pk);
        uint32_t lpv = 0, epv = 0, stride = 0;
        check(pvac_hip_enc_caps_depth(ctx_, depth_hint, &lpv, &epv, &stride));
        std::vector<uint64_t> draws((size_t)n * stride);
        for (auto& x : draws) x = rnd();
        std::vector<uint32_t> status;
        std::vector<CipherT> out = enc_run<CipherT>(vs, draws, stride, lpv, epv, with_sigma, status, depth_hint);
        for (uint32_t grow = stride; ; grow *= 2) {
            std::vector<size_t> redo;
            for (size_t i = 0; i < n; ++i) {
                if (status[i] == 2) throw Error(PVAC_EINVAL, "enc_value: a merged edge group cancelled (p ~ 1/p)");
                if (status[i] == 1) redo.push_back(i);
            }
            if (redo.empty()) break;
            if (grow > (1u << 20)) throw Error(PVAC_EINVAL, "enc_value: random source keeps being rejected");
            const uint32_t s2 = stride + grow;
            std::vector<uint64_t> v2(redo.size()), d2((size_t)redo.size() * s2);
            for (size_t k = 0; k < redo.size(); ++k) {
                v2[k] = vs[redo[k]];
                std::memcpy(&d2[k * s2], &draws[redo[k] * stride], (size_t)stride * 8);
                for (uint32_t j = stride; j < s2; ++j) d2[k * s2 + j] = rnd();
            }
            std::vector<uint32_t> st2;
            std::vector<CipherT> o2 = enc_run<CipherT>(v2, d2, s2, lpv, epv, with_sigma, st2, depth_hint);
            // the redone values' draws become their prefix for a further round
            std::vector<uint64_t> nd((size_t)n * s2, 0);
            for (size_t i = 0; i < n; ++i) std::memcpy(&nd[i * s2], &draws[i * stride], (size_t)stride * 8);
            for (size_t k = 0; k < redo.size(); ++k) {
                out[redo[k]] = std::move(o2[k]);
                status[redo[k]] = st2[k];
                std::memcpy(&nd[redo[k] * s2], &d2[k * s2], (size_t)s2 * 8);
            }
            draws.swap(nd);
            stride = s2;
        }
        return out;
    }

    // Batched dec_value (ops/decrypt.hpp:12-89): prf_R of every BASE layer on the device
    // (pvac_hip_base_R), then the R-tree, inverses and weighted sum (pvac_hip_dec_value).
    template <class PubKeyT, class SecKeyT, class CipherT, class FpT>
    std::vector<FpT> dec_value(const PubKeyT& pk, const SecKeyT& sk, const std::vector<const CipherT*>& cs) {
        const size_t n = cs.size();
        if (!n) return {};
        ensure_keys(pk, sk);
        detail::batch x;
        detail::to_host(cs, sigma_words(), false, x);
        detail::upload(x, stream_, false);
        pvac_ct_batch vx = x.view(false);
        detail::dev_array<uint64_t> R(2 * (x.layers.size() ? x.layers.size() : 1)), out(2 * n);
        detail::dev_array<uint32_t> st(n);
        check(pvac_hip_base_R(ctx_, &vx, R.p));
        check(pvac_hip_dec_value(ctx_, &vx, R.p, out.p, st.p));
        std::vector<uint64_t> o(2 * n);
        std::vector<uint32_t> s(n);
        out.download(o.data(), 2 * n, stream_);
        st.download(s.data(), n, stream_);
        detail::hip_ok(hipStreamSynchronize(stream_), "sync");
        std::vector<FpT> r(n);
        for (size_t i = 0; i < n; ++i) {
            if (s[i] == 1) throw Error(PVAC_EINVAL, "dec_value: layer graph has a cycle or a bad parent");
            if (s[i] == 2) throw Error(PVAC_EINVAL, "dec_value: edge references a layer or idx out of range");
            r[i].lo = o[2 * i];
            r[i].hi = o[2 * i + 1];
        }
        return r;
    }

private:
    void check(int rc) {
        if (rc) throw Error(rc, std::string("pvac_hip: ") + pvac_hip_last_error(ctx_));
    }

    template <class SecKeyT>
    static std::vector<uint64_t> key_fingerprint(const SecKeyT& sk) {
        std::vector<uint64_t> f(sk.prf_k.begin(), sk.prf_k.end());
        f.insert(f.end(), sk.lpn_s_bits.begin(), sk.lpn_s_bits.end());
        return f;
    }

    // one pvac_hip_enc_value launch over (vs, draws) with a fixed stride; status per value
    template <class CipherT>
    std::vector<CipherT> enc_run(const std::vector<uint64_t>& vs, const std::vector<uint64_t>& draws, uint32_t stride,
                                 uint32_t lpv, uint32_t epv, bool with_sigma, std::vector<uint32_t>& status,
                                 int depth_hint = 0) {
        const size_t n = vs.size();
        detail::dev_array<uint64_t> d_v(n), d_r(draws.size());
        d_v.upload(vs.data(), n, stream_);
        d_r.upload(draws.data(), draws.size(), stream_);
        detail::batch c;
        c.d_l_off.alloc(n); c.d_l_cnt.alloc(n); c.d_e_off.alloc(n); c.d_e_cnt.alloc(n);
        const uint64_t lslots = (uint64_t)n * lpv, eslots = (uint64_t)n * epv;
        detail::alloc_out(c, n, lslots, eslots, sigma_words(), with_sigma);
        pvac_ct_batch vc = c.view(with_sigma);
        vc.n = n;
        detail::dev_array<uint32_t> st(n);
        check(pvac_hip_enc_value_depth(ctx_, n, d_v.p, d_r.p, stride, depth_hint, &vc,
                                       with_sigma ? PVAC_ENC_WITH_SIGMA : 0, st.p));
        status.resize(n);
        st.download(status.data(), n, stream_);
        return detail::from_device<CipherT>(c, n, lslots, eslots, prm_.m_bits, with_sigma, stream_);
    }

    pvac_hip_params prm_;
    pvac_hip_ctx* ctx_ = nullptr;
    hipStream_t stream_ = nullptr;
    bool h_ready_ = false;
    bool keys_ready_ = false;
    Phases phases_;
    detail::pinned_batch mul_a_, mul_b_, mul_c_, mul_p_;
    detail::dev_array<uint64_t> mul_nonces_, mul_salts_;
    detail::dev_array<uint32_t> mul_status_;
    std::vector<uint64_t> key_fp_;
};

// Process-wide engines keyed by canon_tag (one public key = one context), device 0 unless
// PVAC_HIP_DEVICE is set. Contexts are not shared between threads (C ABI contract).
template <class PubKeyT>
Engine& engine_for(const PubKeyT& pk) {
    thread_local std::map<uint64_t, std::unique_ptr<Engine>> engines;
    auto it = engines.find(pk.canon_tag);
    if (it == engines.end()) {
        const char* d = std::getenv("PVAC_HIP_DEVICE");
        it = engines.emplace(pk.canon_tag, std::make_unique<Engine>(d ? std::atoi(d) : 0, Engine::params_of(pk))).first;
    }
    return *it->second;
}

// ---- drop-in single-op forms (ops/arithmetic.hpp signatures) ------------------------------
template <class PubKeyT, class CipherT>
CipherT ct_mul(const PubKeyT& pk, const CipherT& A, const CipherT& B, const RandomSource& rnd = os_random_u64) {
    return engine_for(pk).ct_mul(pk, std::vector<const CipherT*>{&A}, std::vector<const CipherT*>{&B}, true, rnd)[0];
}

template <class PubKeyT, class CipherT>
CipherT ct_add(const PubKeyT& pk, const CipherT& A, const CipherT& B) {
    return engine_for(pk).ct_add(std::vector<const CipherT*>{&A}, std::vector<const CipherT*>{&B}, false)[0];
}

template <class PubKeyT, class CipherT>
CipherT ct_sub(const PubKeyT& pk, const CipherT& A, const CipherT& B) {
    return engine_for(pk).ct_add(std::vector<const CipherT*>{&A}, std::vector<const CipherT*>{&B}, true)[0];
}

// ct_scale (ops/arithmetic.hpp:33-37): every edge weight times s.
template <class PubKeyT, class CipherT, class FpT>
CipherT ct_scale(const PubKeyT& pk, const CipherT& A, const FpT& s) {
    CipherT C = A;
    const size_t n = C.E.size();
    std::vector<uint64_t> lo(n), hi(n), slo{s.lo}, shi{s.hi};
    for (size_t i = 0; i < n; ++i) { lo[i] = C.E[i].w.lo; hi[i] = C.E[i].w.hi; }
    engine_for(pk).fp_binop(PVAC_FP_SCALE, lo.data(), hi.data(), slo.data(), shi.data(), lo.data(), hi.data(), n);
    for (size_t i = 0; i < n; ++i) { C.E[i].w.lo = lo[i]; C.E[i].w.hi = hi[i]; }
    return C;
}

// ct_neg (ops/arithmetic.hpp:39-41): ct_scale by fp_neg(fp_from_u64(1)) = p - 1.
template <class PubKeyT, class CipherT>
CipherT ct_neg(const PubKeyT& pk, const CipherT& A) {
    std::decay_t<decltype(A.E[0].w)> s{};
    s.lo = ~0ull - 1;
    s.hi = 0x7FFFFFFFFFFFFFFFull;
    return ct_scale(pk, A, s);
}

// ct_div_const (ops/arithmetic.hpp:108-110): ct_scale by fp_inv(k) (core/field.hpp:229-273; the
// inverse is unique, so the device's addition chain, PVAC_FP_INV, gives the reference's value;
// fp_inv(0) = 0 as there).
template <class PubKeyT, class CipherT, class FpT>
CipherT ct_div_const(const PubKeyT& pk, const CipherT& A, const FpT& k) {
    uint64_t lo = k.lo, hi = k.hi;
    engine_for(pk).fp_binop(PVAC_FP_INV, &lo, &hi, nullptr, nullptr, &lo, &hi, 1);
    FpT inv = k;
    inv.lo = lo;
    inv.hi = hi;
    return ct_scale(pk, A, inv);
}

// ---- batched forms ------------------------------------------------------------------------
template <class PubKeyT, class CipherT>
std::vector<CipherT> ct_mul_batch(const PubKeyT& pk, const std::vector<CipherT>& A, const std::vector<CipherT>& B,
                                  bool with_sigma = true, const RandomSource& rnd = os_random_u64) {
    std::vector<const CipherT*> a, b;
    for (auto& x : A) a.push_back(&x);
    for (auto& x : B) b.push_back(&x);
    return engine_for(pk).ct_mul(pk, a, b, with_sigma, rnd);
}

// Multi-device batch: pairs split into contiguous ranges, one per entry of `devices` (an ordinal may
// repeat), each range on its own host thread and context. Draws from rnd stay in the one-device order:
// every pair's nonces first (pair order; their counts, 2 |A.L| |B.L| per pair, are known up front, so
// they are drawn before any device starts), then every pair's salts (pair order: range j draws its
// salts once its own weights are known and ranges < j have drawn theirs). So a replayed stream gives
// the bytes of ct_mul_batch on one device.
template <class PubKeyT, class CipherT>
std::vector<CipherT> ct_mul_batch(const PubKeyT& pk, const std::vector<CipherT>& A, const std::vector<CipherT>& B,
                                  bool with_sigma, const RandomSource& rnd, const std::vector<int>& devices) {
    if (devices.size() <= 1) {
        std::vector<const CipherT*> a, b;
        for (auto& x : A) a.push_back(&x);
        for (auto& x : B) b.push_back(&x);
        if (devices.empty()) return engine_for(pk).ct_mul(pk, a, b, with_sigma, rnd);
        Engine e(devices[0], Engine::params_of(pk));
        return e.ct_mul(pk, a, b, with_sigma, rnd);
    }
    if (A.size() != B.size()) throw Error(PVAC_EINVAL, "ct_mul_batch: |A| != |B|");
    const size_t n = A.size(), D = devices.size();
    std::vector<uint64_t> first(D + 1);
    for (size_t j = 0; j <= D; ++j) first[j] = n * j / D;
    // every nonce word, pair order
    std::vector<std::vector<uint64_t>> nonces(D);
    for (size_t j = 0; j < D; ++j)
        for (size_t i = first[j]; i < first[j + 1]; ++i)
            for (size_t k = 0; k < 2 * A[i].L.size() * B[i].L.size(); ++k) nonces[j].push_back(rnd());
    std::mutex mu;
    std::condition_variable cv;
    size_t turn = 0;   // the range whose salts are drawn next
    std::vector<std::vector<CipherT>> out(D);
    std::vector<std::exception_ptr> err(D);
    std::vector<std::thread> th;
    for (size_t j = 0; j < D; ++j)
        th.emplace_back([&, j] {
            bool my_turn = false;
            try {
                size_t pos = 0;
                // a range's source: its pre-drawn nonces, then (in range order) salts from rnd
                RandomSource src = [&]() -> uint64_t {
                    if (pos < nonces[j].size()) return nonces[j][pos++];
                    if (!my_turn) {
                        std::unique_lock<std::mutex> g(mu);
                        cv.wait(g, [&] { return turn == j; });
                        my_turn = true;
                    }
                    std::lock_guard<std::mutex> g(mu);
                    return rnd();
                };
                std::vector<const CipherT*> a, b;
                for (size_t i = first[j]; i < first[j + 1]; ++i) {
                    a.push_back(&A[i]);
                    b.push_back(&B[i]);
                }
                Engine e(devices[j], Engine::params_of(pk));
                out[j] = e.ct_mul(pk, a, b, with_sigma, src);
            } catch (...) {
                err[j] = std::current_exception();
            }
            {
                // hand the salt turn on (also when this range drew none, or failed)
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return turn == j; });
                ++turn;
            }
            cv.notify_all();
        });
    for (auto& t : th) t.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
    std::vector<CipherT> all;
    all.reserve(n);
    for (auto& v : out)
        for (auto& c : v) all.push_back(std::move(c));
    return all;
}

// Chains through the chain entry point (Engine::ct_mul_chain): one RandomSource per input.
template <class PubKeyT, class CipherT>
std::vector<CipherT> ct_mul_chain(const PubKeyT& pk, const std::vector<CipherT>& xs, uint32_t depth, bool with_sigma,
                                  std::vector<RandomSource>& rnds, const std::vector<int>& devices = {}) {
    std::vector<const CipherT*> x;
    for (auto& c : xs) x.push_back(&c);
    return engine_for(pk).ct_mul_chain(pk, x, depth, with_sigma, rnds, devices);
}

// The reference's loop c_k = ct_mul(c_{k-1}, y_k) with a fresh operand per step (tests/test_main.cpp:
// 289-293): ys[k - 1][i] is chain i's operand at step k (depth = ys.size()).
template <class PubKeyT, class CipherT>
std::vector<CipherT> ct_mul_chain(const PubKeyT& pk, const std::vector<CipherT>& xs,
                                  const std::vector<std::vector<CipherT>>& ys, bool with_sigma,
                                  std::vector<RandomSource>& rnds, const std::vector<int>& devices = {}) {
    std::vector<const CipherT*> x;
    for (auto& c : xs) x.push_back(&c);
    std::vector<std::vector<const CipherT*>> ops(ys.size());
    for (size_t d = 0; d < ys.size(); ++d)
        for (auto& c : ys[d]) ops[d].push_back(&c);
    return engine_for(pk).ct_mul_chain(pk, x, (uint32_t)ys.size(), with_sigma, rnds, devices, 2, 16, ops);
}

template <class PubKeyT, class CipherT>
std::vector<CipherT> ct_add_batch(const PubKeyT& pk, const std::vector<CipherT>& A, const std::vector<CipherT>& B,
                                  bool negate_b = false) {
    std::vector<const CipherT*> a, b;
    for (auto& x : A) a.push_back(&x);
    for (auto& x : B) b.push_back(&x);
    return engine_for(pk).ct_add(a, b, negate_b);
}

// ---- encryption / decryption (ops/encrypt.hpp:289, ops/decrypt.hpp:62) --------------------
template <class CipherT, class PubKeyT, class SecKeyT>
CipherT enc_value(const PubKeyT& pk, const SecKeyT& sk, uint64_t v, const RandomSource& rnd = os_random_u64) {
    return engine_for(pk).template enc_value<PubKeyT, SecKeyT, CipherT>(pk, sk, std::vector<uint64_t>{v}, true, rnd)[0];
}

// enc_value_depth / enc_zero_depth (ops/encrypt.hpp:281-287, 293-298): the noise plan of depth_hint
template <class CipherT, class PubKeyT, class SecKeyT>
CipherT enc_value_depth(const PubKeyT& pk, const SecKeyT& sk, uint64_t v, int depth_hint,
                        const RandomSource& rnd = os_random_u64) {
    return engine_for(pk).template enc_value<PubKeyT, SecKeyT, CipherT>(pk, sk, std::vector<uint64_t>{v}, true, rnd,
                                                                         depth_hint)[0];
}

template <class CipherT, class PubKeyT, class SecKeyT>
CipherT enc_zero_depth(const PubKeyT& pk, const SecKeyT& sk, int depth_hint, const RandomSource& rnd = os_random_u64) {
    return enc_value_depth<CipherT>(pk, sk, 0, depth_hint, rnd);
}

template <class CipherT, class PubKeyT, class SecKeyT>
std::vector<CipherT> enc_value_batch(const PubKeyT& pk, const SecKeyT& sk, const std::vector<uint64_t>& vs,
                                     bool with_sigma = true, const RandomSource& rnd = os_random_u64) {
    return engine_for(pk).template enc_value<PubKeyT, SecKeyT, CipherT>(pk, sk, vs, with_sigma, rnd);
}

template <class PubKeyT, class SecKeyT, class CipherT>
auto dec_value(const PubKeyT& pk, const SecKeyT& sk, const CipherT& C) {
    using FpT = std::decay_t<decltype(C.E[0].w)>;
    return engine_for(pk).template dec_value<PubKeyT, SecKeyT, CipherT, FpT>(pk, sk, std::vector<const CipherT*>{&C})[0];
}

template <class PubKeyT, class SecKeyT, class CipherT>
auto dec_value_batch(const PubKeyT& pk, const SecKeyT& sk, const std::vector<CipherT>& cs) {
    using FpT = std::decay_t<decltype(cs[0].E[0].w)>;
    std::vector<const CipherT*> p;
    for (auto& x : cs) p.push_back(&x);
    return engine_for(pk).template dec_value<PubKeyT, SecKeyT, CipherT, FpT>(pk, sk, p);
}

// ---- .ct files (the reference's tests/add.cpp:22-155 format) through the native codec ------
// Layers of PROD rule come back with zero seeds (the format stores none); sigmas come back as
// stored (nbits 0 and no words when the file carries none).
template <class CipherT>
std::vector<CipherT> load_cts_bytes(const std::vector<uint8_t>& buf) {
    pvac_ct_file_info info{};
    int rc = pvac_ct_scan(buf.data(), buf.size(), &info);
    if (rc) throw Error(rc, "load_cts: malformed .ct image");
    if (info.flags & PVAC_CT_MIXED_SIGMA) throw Error(PVAC_ENOSYS, "load_cts: edges disagree on sigma nbits");
    const size_t n = info.n_ciphers, nl = info.total_layers, ne = info.total_edges;
    const uint32_t sw = info.sigma_words;
    std::vector<uint64_t> l_off(n), l_cnt(n), e_off(n), e_cnt(n), meta(ne), w_lo(ne), w_hi(ne), sig(ne * sw);
    std::vector<pvac_layer> layers(nl);
    pvac_ct_batch X{};
    X.n = n; X.l_off = l_off.data(); X.l_cnt = l_cnt.data(); X.layers = layers.data();
    X.e_off = e_off.data(); X.e_cnt = e_cnt.data(); X.meta = meta.data(); X.w_lo = w_lo.data(); X.w_hi = w_hi.data();
    X.sigma = sw ? sig.data() : nullptr;
    X.sigma_words = sw;
    rc = pvac_ct_parse(buf.data(), buf.size(), &X, 0);
    if (rc) throw Error(rc, "load_cts: parse failed");
    std::vector<CipherT> out(n);
    for (size_t i = 0; i < n; ++i) {
        CipherT& C = out[i];
        C.L.resize(l_cnt[i]);
        for (size_t l = 0; l < l_cnt[i]; ++l) {
            const pvac_layer& y = layers[l_off[i] + l];
            auto& L = C.L[l];
            L.rule = static_cast<decltype(L.rule)>(y.rule);
            L.pa = y.pa; L.pb = y.pb;
            L.seed.ztag = y.ztag; L.seed.nonce.lo = y.nonce_lo; L.seed.nonce.hi = y.nonce_hi;
        }
        C.E.resize(e_cnt[i]);
        for (size_t k = 0; k < e_cnt[i]; ++k) {
            const size_t e = e_off[i] + k;
            auto& E = C.E[k];
            E.layer_id = (uint32_t)meta[e];
            E.idx = (uint16_t)(meta[e] >> 32);
            E.ch = (uint8_t)(meta[e] >> 48);
            E.w.lo = w_lo[e]; E.w.hi = w_hi[e];
            E.s.nbits = info.sigma_bits;
            E.s.w.assign(sig.begin() + e * sw, sig.begin() + (e + 1) * sw);
        }
    }
    return out;
}

// Every edge's sigma is written with nbits = sigma_bits (the reference writes m_bits = 8192).
template <class CipherT>
std::vector<uint8_t> save_cts_bytes(const std::vector<CipherT>& cs, uint32_t sigma_bits = 8192) {
    const uint32_t sw = (sigma_bits + 63) / 64;
    std::vector<const CipherT*> p;
    for (auto& x : cs) p.push_back(&x);
    detail::batch b;
    detail::to_host(p, sw, true, b);
    pvac_ct_batch X{};
    X.n = cs.size(); X.l_off = b.l_off.data(); X.l_cnt = b.l_cnt.data(); X.layers = b.layers.data();
    X.e_off = b.e_off.data(); X.e_cnt = b.e_cnt.data(); X.meta = b.meta.data();
    X.w_lo = b.w_lo.data(); X.w_hi = b.w_hi.data();
    X.sigma = b.sigma.data();
    X.sigma_words = sw;
    uint64_t bytes = 0, written = 0;
    int rc = pvac_ct_serialized_size(&X, sigma_bits, &bytes);
    if (rc) throw Error(rc, "save_cts: size");
    std::vector<uint8_t> out(bytes);
    rc = pvac_ct_write(&X, sigma_bits, out.data(), out.size(), &written, 0);
    if (rc || written != bytes) throw Error(rc ? rc : PVAC_EINVAL, "save_cts: write");
    return out;
}

}  // namespace pvac_hip

#endif  // PVAC_HIP_HPP
