// runtime.cpp — host side of libpvac_hip.so: the extern "C" ABI of include/pvac_hip.h.
//
// Owns per-context device state (stream, libstdc++ bucket-count table, plan scratch,
// sparse H, timing events) and sequences the kernels. Never throws across the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <tuple>
#include <new>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "sigma.hpp"
#include "sha256.hpp"

using namespace pvhip;

namespace {

constexpr uint32_t kNbTableLen = kFreshProdMax + 1;   // bucket counts for |A.E||B.E| in [0, 4096]

struct timer_rec {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    double ms = 0;
    uint64_t launches = 0;
};

// one output batch of a chain worker (pvac_hip_ct_mul_chain): stream-ordered allocations that grow
struct chain_set {
    uint64_t* l_off = nullptr;
    uint64_t* l_cnt = nullptr;
    uint64_t* e_off = nullptr;
    uint64_t* e_cnt = nullptr;
    size_t n_cap = 0;
    pvac_layer* layers = nullptr;
    size_t l_cap = 0;
    uint64_t* meta = nullptr;
    uint64_t* w_lo = nullptr;
    uint64_t* w_hi = nullptr;
    size_t e_cap = 0;
    uint64_t* sigma = nullptr;   // final step with PVAC_MUL_WITH_SIGMA: 1 KiB per edge slot
    size_t s_cap = 0;            // edge slots of sigma
    uint32_t* img = nullptr;     // per pair: 1 = this step's C is a dense image (mul_large_args::C_img)
    size_t img_cap = 0;
};

}  // namespace

struct pvac_hip_ctx {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    pvac_hip_params prm{};
    std::string err;
    // device tables / scratch
    uint32_t* nb_table = nullptr;
    uint64_t* nb_magic = nullptr;
    uint8_t* pair_class = nullptr;
    uint32_t* pair_status = nullptr;
    fresh_rec* fresh_recs = nullptr;   // per-pair header records of the fresh ct_mul path
    std::vector<merge_pair_info> merge_host;   // over-budget ct_add pairs of the latest add plan
    void* merge_scratch = nullptr;
    size_t merge_cap = 0;
    unsigned long long* merge_counters = nullptr;
    uint64_t* powg = nullptr;          // pk.powg_B on the device, B x (lo, hi)
    uint32_t powg_n = 0;
    void* dec_scratch = nullptr;
    size_t dec_cap = 0;
    uint64_t* dec_roff = nullptr;
    size_t dec_roff_cap = 0;
    // LPN PRF key material (SecKey) and pk.H_digest
    uint64_t prf_k[4] = {0, 0, 0, 0};
    uint64_t* lpn_s = nullptr;
    uint32_t lpn_words = 0, lpn_t = 0, tau_num = 0, tau_den = 0;
    bool have_secret = false;
    uint8_t H_digest[32] = {0};
    bool have_digest = false;
    bool aes_tables = false;
    uint8_t* prf_req = nullptr;
    size_t prf_req_cap = 0;
    uint64_t* prf_core = nullptr;
    size_t prf_core_cap = 0;
    uint8_t* enc_arena = nullptr;
    size_t enc_arena_cap = 0;
    uint64_t* large_ids = nullptr;
    uint64_t* large_info = nullptr;
    uint64_t* redo_ids = nullptr;        // fresh-kernel pairs left to the general path (a key sum of 0)
    unsigned int* redo_cnt = nullptr;
    size_t pair_cap = 0;
    // general ct_mul path: host descriptors of the last plan, device copies, scratch arena
    std::vector<large_desc> large_host;
    std::vector<large_desc> large_exec;
    uint32_t plan_stamp = 0;
    uint64_t last_mul_pairs = 0;       // pairs of the last ct_mul_exec (pair_status is valid for these)
    uint64_t redo_total = 0;           // pairs re-run by redo_fresh_pairs since the context was created
    uint64_t path_total[4] = {};       // pair launches: fresh kernel, general path, its iblk order, direct mode
    double noise_bits = 120.0, noise_t2 = 0.55, noise_slope = 16.0;   // Params noise fields (enc plan_noise)
    large_desc* desc_dev = nullptr;
    size_t desc_cap = 0;
    uint32_t* sel_dev = nullptr;       // products: descriptor order per sub-batch (A-layer-major class first)
    size_t sel_cap = 0;
    std::vector<uint32_t> sel_host;
    uint32_t* arena = nullptr;
    size_t arena_words = 0;
    // static bucket-group tables of the last plan (one per distinct bucket count) + build scratch
    uint32_t* grp = nullptr;
    size_t grp_cap = 0;
    uint32_t* grp_tmp = nullptr;
    size_t grp_tmp_cap = 0;
    uint32_t* salt_pos = nullptr;
    size_t salt_cap = 0;
    mul_fresh_args* fresh_args = nullptr;   // device copy of the fresh kernel's arguments
    mul_fresh_args fresh_args_host{};
    bool fresh_args_uploaded = false;       // the device copy holds fresh_args_host
    bool redo_cnt_dirty = true;             // redo_cnt may be nonzero (zeroed before the next exec)
    uint64_t* scan_scratch = nullptr;
    size_t scan_cap = 0;
    plan_stats* stats = nullptr;
    unsigned int* check_buf = nullptr;   // gsum check: 4 layer maxima, then a u64 failure count
    uint8_t* check_scratch = nullptr;    // gsum check: layer tables beyond LDS (global slabs)
    size_t check_scratch_cap = 0;
    unsigned long long* totals = nullptr;   // [2]: &stats->total_layers (layer and edge slot totals)
    void* pin = nullptr;                    // pinned host words for the plan's and exec's read-backs
    sigma_tables H;
    // timing
    bool timing = false;
    std::map<std::string, timer_rec> timers;
    std::vector<hipEvent_t> ev_pool;   // timer events returned by flush_timers, reused (no create per launch)
    // general-path scratch cap in words (0 = half the free HBM): chain workers share the device
    uint64_t arena_cap_words = 0;
    bool large_no_direct = false;   // the redo run: every pair on the full (per-key sums) layout
    // chain steps: per-pair dense-image flags of A (read; cleared where A is turned back into records)
    // and of C (written) for the next exec (mul_large_args::A_img / C_img); null outside the chain
    uint32_t* img_in = nullptr;
    uint32_t* img_out = nullptr;
    unsigned long long* img_count = nullptr;   // chain: pair-steps written as images (chain_stats' last word)
    uint64_t* img_tmp = nullptr;       // image -> records: 3 words per edge of the pairs converted
    size_t img_tmp_cap = 0;
    uint64_t* img_pairs = nullptr;     // [2 n]: pair ids, then their offsets in img_tmp
    size_t img_pairs_cap = 0;
    uint32_t img_grid_y = 65535;       // pairs per image -> records launch (PVAC_CHAIN_IMG_BATCH2: 2)
    uint32_t spin_us = 50000;          // read_back's spin before a blocking wait (chain workers: 200)
    // pvac_hip_ct_mul_chain: worker contexts (own stream / arena), and a worker's own buffers
    std::vector<pvac_hip_ctx*> chain_kids;   // [range j * streams + w] of the last call's layout
    chain_set chain_bufs[2];
    chain_set chain_stage;                   // a worker's staged chunk inputs (another device, or STAGE)
    chain_set chain_stage_op;                // ... and its staged per-step operand (pvac_chain_opts::operands)
    uint64_t* chain_nonces = nullptr;
    size_t chain_nonce_cap = 0;
    uint64_t* chain_salts = nullptr;         // final-step salts (WITH_SIGMA)
    size_t chain_salt_cap = 0;
    uint64_t* chain_out = nullptr;           // digests / counts of a chunk before the copy to X's device
    size_t chain_out_cap = 0;
    unsigned long long* chain_stats = nullptr;   // [2 * PVAC_CHAIN_MAX_DEPTH + 1]: edges / products, image pair-steps
    std::vector<int64_t> chain_layout;          // the last call's (streams, chunk, n_devices, ordinals...)
    uint64_t H_gen = 0;                      // bumped whenever H is set (a worker's copy follows it)
    uint64_t H_from = 0;                     // worker: the parent's H_gen its H copy was taken from
};

namespace {

int fail(pvac_hip_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

int hip_fail(pvac_hip_ctx* c, hipError_t e, const char* where) {
    if (e == hipSuccess) return PVAC_OK;
    std::string m = std::string(where) + ": " + hipGetErrorString(e);
    return fail(c, e == hipErrorOutOfMemory ? PVAC_ENOMEM : PVAC_EDEVICE, m);
}

// libstdc++ bucket count chosen by std::unordered_map::reserve(n) on an empty map: the
// container rehashes to _M_next_bkt(max(1, ceil(n / max_load_factor))) with max load 1.0.
// Asking the policy object directly gives the identical value without allocating.
uint64_t bucket_count_after_reserve(uint64_t n) {
    std::__detail::_Prime_rehash_policy pol(1.0f);
    const uint64_t want = std::max<uint64_t>(1, (uint64_t)pol._M_bkt_for_elements(n));
    return pol._M_next_bkt(want);
}

struct scoped_timer {
    pvac_hip_ctx* c;
    timer_rec* rec = nullptr;
    hipEvent_t a{}, b{};
    scoped_timer(pvac_hip_ctx* ctx, const char* name) : c(ctx) {
        if (!c->timing) return;
        rec = &c->timers[name];
        a = take();
        b = take();
        hipEventRecord(a, c->stream);
    }
    hipEvent_t take() {
        hipEvent_t e{};
        if (!c->ev_pool.empty()) {
            e = c->ev_pool.back();
            c->ev_pool.pop_back();
        } else {
            hipEventCreate(&e);
        }
        return e;
    }
    ~scoped_timer() {
        if (!rec) return;
        hipEventRecord(b, c->stream);
        rec->pending.emplace_back(a, b);
    }
};

void flush_timers(pvac_hip_ctx* c) {
    for (auto& kv : c->timers) {
        for (auto& ev : kv.second.pending) {
            hipEventSynchronize(ev.second);
            float ms = 0;
            hipEventElapsedTime(&ms, ev.first, ev.second);
            kv.second.ms += ms;
            kv.second.launches += 1;
            c->ev_pool.push_back(ev.first);
            c->ev_pool.push_back(ev.second);
        }
        kv.second.pending.clear();
    }
}

#ifndef PVAC_FAST_READBACK   // A/B builds only: pinned read-back words and a spinning wait for them
#define PVAC_FAST_READBACK 1
#endif
// The short host waits of a plan (its totals) and of exec (the redo count): a blocking
// hipStreamSynchronize wakes tens of microseconds after the copy lands, so spin on hipStreamQuery
// (up to spin_us, then block) and read into pinned words (a pageable destination stages the copy).
// A caller's context spins up to 50 ms (one thread, the headline step); the chain's worker contexts
// (several threads per device) spin 200 us and then block, so they do not hold cores and the HIP
// runtime's locks while their kernels run.
hipError_t read_back(pvac_hip_ctx* c, void* dst, const void* src, size_t bytes) {
#if PVAC_FAST_READBACK
    if (c->pin && bytes <= 256) {
        hipError_t e = hipMemcpyAsync(c->pin, src, bytes, hipMemcpyDeviceToHost, c->stream);
        if (e != hipSuccess) return e;
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            e = hipStreamQuery(c->stream);
            if (e != hipErrorNotReady) break;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(c->spin_us)) {
                e = hipStreamSynchronize(c->stream);
                break;
            }
        }
        if (e == hipSuccess) std::memcpy(dst, c->pin, bytes);
        return e;
    }
#endif
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return e;
}

int ensure_scan(pvac_hip_ctx* c, size_t n);

int ensure_pairs(pvac_hip_ctx* c, size_t n) {
    if (n > c->pair_cap) {
        hipFree(c->pair_class);
        hipFree(c->pair_status);
        hipFree(c->large_ids);
        hipFree(c->large_info);
        hipFree(c->redo_ids);
        hipFree(c->fresh_recs);
        c->fresh_recs = nullptr;
        c->redo_ids = nullptr;
        c->pair_class = nullptr;
        c->pair_status = nullptr;
        c->large_ids = nullptr;
        c->large_info = nullptr;
        size_t cap = std::max<size_t>(n, 1024);
        hipError_t e = hipMalloc(&c->pair_class, cap);
        if (e == hipSuccess) e = hipMalloc(&c->pair_status, cap * 4);
        if (e == hipSuccess) e = hipMalloc(&c->large_ids, cap * 8);
        if (e == hipSuccess) e = hipMalloc(&c->large_info, cap * 64);   // 5 (mul) or 8 (add merge) words per pair
        if (e == hipSuccess) e = hipMalloc(&c->fresh_recs, cap * sizeof(fresh_rec));
        if (e == hipSuccess) e = hipMalloc(&c->redo_ids, cap * 8);
        if (e == hipSuccess && !c->redo_cnt) e = hipMalloc(&c->redo_cnt, 16);
        if (e != hipSuccess) { c->pair_cap = 0; return hip_fail(c, e, "alloc pair scratch"); }
        c->pair_cap = cap;
    }
    return ensure_scan(c, n);
}

// the exclusive scans' scratch for n counts
int ensure_scan(pvac_hip_ctx* c, size_t n) {
    const size_t sw = scan_scratch_words(n);
    if (sw > c->scan_cap) {
        hipFree(c->scan_scratch);
        c->scan_scratch = nullptr;
        hipError_t e = hipMalloc(&c->scan_scratch, sw * 8);
        if (e != hipSuccess) { c->scan_cap = 0; return hip_fail(c, e, "alloc scan scratch"); }
        c->scan_cap = sw;
    }
    return PVAC_OK;
}

bool batch_ok(const pvac_ct_batch* X) {
    return X && (X->n == 0 || (X->l_off && X->l_cnt && X->e_off && X->e_cnt));
}

template <typename T>
int ensure_dev(pvac_hip_ctx* c, T*& p, size_t& cap, size_t n, const char* what) {
    if (n <= cap) return PVAC_OK;
    hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(n, 1024);
    hipError_t e = hipMalloc(&p, want * sizeof(T));
    if (e != hipSuccess) return hip_fail(c, e, what);
    cap = want;
    return PVAC_OK;
}

uint32_t ceil_log2(uint64_t x) {
    uint32_t b = 0;
    while ((1ull << b) < x) ++b;
    return b;
}

// Per-A-edge emit order for eligible pairs (large_desc::iblk). A/B builds only (make variant-f, never
// the shipped library): -DPVAC_LARGE_IBLK=0 keeps the n/16 block marks for every pair, and so does
// -DPVAC_LARGE_PRODUCTS_COL26, whose per-task products kernel does not see an A layer's keys in one
// workgroup.
#ifndef PVAC_LARGE_IBLK
#define PVAC_LARGE_IBLK 1
#endif
constexpr bool large_iblk_enabled() {
#ifdef PVAC_LARGE_PRODUCTS_COL26
    return false;
#else
    return PVAC_LARGE_IBLK != 0;
#endif
}
// Direct mode for iblk pairs (large_desc::direct): A/B builds with -DPVAC_LARGE_DIRECT=0 keep every
// iblk pair on the per-key-sums layout
#ifndef PVAC_LARGE_DIRECT
#define PVAC_LARGE_DIRECT 1
#endif

// Scratch layout of one general-path pair (k_mul_large.hip), offsets relative to 0; the
// executor rebases them into the arena. 64-bit arrays on even words, 16-byte arrays on
// multiples of four.
int build_large_desc(large_desc& d, uint64_t pair, uint64_t LA, uint64_t LB, uint64_t nA, uint64_t nB, uint32_t Bm,
                     std::string& why, bool static_grp = false, bool allow_direct = false) {
    d = large_desc{};
    d.pair = pair;
    d.n = nA * nB;
    d.S = LA * LB * Bm;
    d.Lc = LA + LB + LA * LB;
    if (LA > 0xFFFFFFFFull || LB > 0xFFFFFFFFull || nA > 0xFFFFFFFFull || nB > 0xFFFFFFFFull ||
        (nA && d.n / nA != nB) || d.n >= (1ull << 32)) {
        why = "ct_mul: |A.E||B.E| >= 2^32 products in one pair";
        return PVAC_ENOSYS;
    }
    if (d.Lc > kLargeLayersMax) {
        why = "ct_mul: more than " + std::to_string(kLargeLayersMax) + " layers before compaction in one pair";
        return PVAC_ENOSYS;
    }
    if (d.S >= (1ull << 31)) {
        why = "ct_mul: key space |A.L||B.L|B >= 2^31";
        return PVAC_ENOSYS;
    }
    d.LA = (uint32_t)LA; d.LB = (uint32_t)LB; d.nA = (uint32_t)nA; d.nB = (uint32_t)nB;
    d.nblk = (d.n + 15) / 16;
    const uint64_t keys = std::min(d.n, d.S);
    d.capE = 2 * keys;
    d.nbm = make_fastmod64(bucket_count_after_reserve(d.n));
    d.hbits = std::max<uint32_t>(1, ceil_log2(2 * std::max<uint64_t>(keys, 1)));
    d.g_head = d.g_next = kNoGrp;
    // per-A-edge emit order (k_mul_large.hip): static groups and the A-layer-major products kernel
    d.iblk = static_grp && LB <= kLaMaxLB && nA >= 1 && nB >= 1 && nB <= kIblkMaxNB && large_iblk_enabled() ? 1u : 0u;
    // (direct A ids and writer lists pack an A edge with its dense cell: A edges < 2^21, 2 B <= 2^11)
    // (and k_large_products_direct's LDS: the digit table, LB staged B layers and their sums)
    d.direct = d.iblk && allow_direct && PVAC_LARGE_DIRECT && nA < (1ull << 21) && Bm <= 1024u &&
                       large_direct_lds_bytes(Bm, (uint32_t)LB) <= 160u * 1024u
                   ? 1u
                   : 0u;
    d.nb_m = nB ? (1ull << 32) / nB : 0;
    uint64_t o = 0;
    auto even = [&]() { o = (o + 1) & ~1ull; };
    auto quad = [&]() { o = (o + 3) & ~3ull; };
    if (d.direct) {
        // no per-key scratch: cnt | used, the edge lists, per-A-edge counts and masks
        quad();
        d.o_zero = d.o_cnt = o;
        o += kCntWords;
        d.o_hkey = d.o_hhead = d.o_bmask = o;
        d.o_bcnt = d.o_used = o;
        o += d.Lc;
        d.zero_words = o - d.o_zero;
        d.o_tkey = o;
        d.o_lstA = o; o += 2 * LA + nA;
        d.o_lstB = o; o += 2 * LB + nB;
        d.o_neA = o; o += LA;
        d.o_neB = o; o += LB;
        d.o_defer = d.o_info = d.o_sums = d.o_nxt = d.o_tb = d.o_within = d.o_etot = d.o_cpos = d.o_order = d.o_hpos = o;
        const uint64_t ngrp = (nA + 31) / 32;
        quad();
        d.o_icnt = o; o += 8 * ngrp;   // count bytes
        d.o_iwo = o; o += ngrp;
        d.o_wle = o; o += nA;
        d.o_wln = o; o += LA;
        quad();
        d.o_imask = o; o += 4 * nA;
        quad();
        d.words = o;
        return PVAC_OK;
    }
    const uint64_t hcap = static_grp ? 0 : 1ull << d.hbits;   // static groups: no bucket table / chains
    quad();
    d.o_zero = o;
    d.o_cnt = o; o += kCntWords;
    d.o_hkey = o; o += 2 * hcap;
    d.o_hhead = o; o += hcap;
    even();
    d.o_bmask = o; o += 2 * d.nblk;
    d.o_bcnt = o;
    d.o_used = o; o += d.Lc;
    d.zero_words = o - d.o_zero;
    d.o_tkey = o; o += d.S;
    d.o_lstA = o; o += 2 * LA + nA;
    d.o_lstB = o; o += 2 * LB + nB;
    d.o_neA = o; o += LA;
    d.o_neB = o; o += LB;
    d.o_defer = o; o += LA * LB <= kLaMaxLB * LA ? LA * LB : 0;   // A-layer-major pairs only
    d.o_info = o; o += d.S;
    quad();
    d.o_sums = o; o += 8 * d.S;
    d.o_nxt = o; o += static_grp ? 0 : d.S;
    d.o_tb = o; o += d.S;
    d.o_within = o; o += d.S;
    d.o_etot = o; o += d.S;
    d.o_cpos = o; o += d.S;
    d.o_order = o; o += d.capE;
    d.o_hpos = o; o += d.capE;
    d.o_icnt = o; o += d.iblk ? nA : 0;
    quad();
    d.o_imask = o; o += d.iblk ? 4 * nA : 0;
    quad();
    d.o_wle = d.o_wln = d.o_iwo = o;
    d.words = o;
    return PVAC_OK;
}

void rebase_desc(large_desc& d, uint64_t base) {
    uint64_t* f[] = {&d.o_zero, &d.o_cnt, &d.o_hkey, &d.o_hhead, &d.o_bmask, &d.o_bcnt, &d.o_used, &d.o_tkey,
                     &d.o_lstA, &d.o_lstB, &d.o_neA, &d.o_neB, &d.o_defer, &d.o_info, &d.o_sums, &d.o_nxt, &d.o_tb,
                     &d.o_within, &d.o_etot, &d.o_cpos, &d.o_order, &d.o_hpos, &d.o_icnt, &d.o_imask,
                     &d.o_wle, &d.o_wln, &d.o_iwo};
    for (uint64_t* p : f) *p += base;
}

}  // namespace

// ==================================================================== ABI
extern "C" {

int pvac_hip_abi_version(void) { return PVAC_HIP_ABI_VERSION; }

int pvac_hip_ctx_create(int device, const pvac_hip_params* prm, pvac_hip_ctx** out) {
    if (!out || !prm) return PVAC_EINVAL;
    *out = nullptr;
    if (prm->B == 0 || prm->B > 65535 || prm->m_bits == 0 || prm->n_bits == 0) return PVAC_EINVAL;
    pvac_hip_ctx* c = new (std::nothrow) pvac_hip_ctx();
    if (!c) return PVAC_ENOMEM;
    c->device = device;
    c->prm = *prm;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) { delete c; return PVAC_EDEVICE; }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        c->num_cus = cus;
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { delete c; return PVAC_EDEVICE; }
    c->own_stream = true;
    std::vector<uint32_t> nb(kNbTableLen);
    std::vector<uint64_t> mg(kNbTableLen);
    for (uint32_t n = 0; n < kNbTableLen; ++n) {
        nb[n] = (uint32_t)bucket_count_after_reserve(n);
        mg[n] = make_fastmod64(nb[n]).m;
        if (nb[n] == 0 || nb[n] > 0xFFFFu) { delete c; return PVAC_ERANGE; }   // fresh_rec.nbk is u16
    }
    e = hipMalloc(&c->nb_table, nb.size() * 4);
    if (e == hipSuccess) e = hipMemcpy(c->nb_table, nb.data(), nb.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&c->nb_magic, mg.size() * 8);
    if (e == hipSuccess) e = hipMemcpy(c->nb_magic, mg.data(), mg.size() * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&c->stats, sizeof(plan_stats));
    // the scans' two totals are plan_stats' first words: a plan reads stats and totals back in one copy
    if (e == hipSuccess) c->totals = &c->stats->total_layers;
#if PVAC_FAST_READBACK
    if (e == hipSuccess) e = hipHostMalloc(&c->pin, 256, hipHostMallocDefault);
#endif
    if (e != hipSuccess) { pvac_hip_ctx_destroy(c); return PVAC_ENOMEM; }
    *out = c;
    return PVAC_OK;
}

// a chain worker's output batches (stream-ordered frees on its stream; the caller synchronises)
static void free_chain_sets(pvac_hip_ctx* c) {
    for (chain_set* b : {&c->chain_bufs[0], &c->chain_bufs[1], &c->chain_stage, &c->chain_stage_op}) {
        for (void* q : {(void*)b->l_off, (void*)b->l_cnt, (void*)b->e_off, (void*)b->e_cnt, (void*)b->layers,
                        (void*)b->meta, (void*)b->w_lo, (void*)b->w_hi, (void*)b->sigma, (void*)b->img})
            if (q) hipFreeAsync(q, c->stream);
        *b = chain_set{};
    }
}

// everything a chain worker grew during a call (output batches, nonce / salt / result words, image
// scratch, the general-path arena); the caller selected the worker's device
static hipError_t release_chain_worker(pvac_hip_ctx* k) {
    free_chain_sets(k);
    for (void** q : {(void**)&k->chain_nonces, (void**)&k->chain_salts, (void**)&k->chain_out}) {
        if (*q) hipFreeAsync(*q, k->stream);
        *q = nullptr;
    }
    k->chain_nonce_cap = k->chain_salt_cap = k->chain_out_cap = 0;
    const hipError_t e = hipStreamSynchronize(k->stream);
    for (void** q : {(void**)&k->img_tmp, (void**)&k->img_pairs, (void**)&k->arena, (void**)&k->check_scratch}) {
        hipFree(*q);
        *q = nullptr;
    }
    k->img_tmp_cap = k->img_pairs_cap = k->check_scratch_cap = 0;
    k->arena_words = 0;
    return e;
}

int pvac_hip_ctx_destroy(pvac_hip_ctx* c) {
    if (!c) return PVAC_OK;
    int caller_dev = -1;   // the calling thread's device, restored on return
    if (hipGetDevice(&caller_dev) != hipSuccess) caller_dev = -1;
    hipSetDevice(c->device);
    for (pvac_hip_ctx* k : c->chain_kids) pvac_hip_ctx_destroy(k);
    c->chain_kids.clear();
    hipSetDevice(c->device);   // each worker's destroy selected the worker's device
    if (c->stream) hipStreamSynchronize(c->stream);
    flush_timers(c);
    for (hipEvent_t e : c->ev_pool) hipEventDestroy(e);
    c->ev_pool.clear();
    free_chain_sets(c);
    for (void* q : {(void*)c->chain_nonces, (void*)c->chain_salts, (void*)c->chain_out})
        if (q) hipFreeAsync(q, c->stream);
    if (c->stream) hipStreamSynchronize(c->stream);
    hipFree(c->chain_stats);
    hipFree(c->nb_table);
    hipFree(c->nb_magic);
    hipFree(c->pair_class);
    hipFree(c->pair_status);
    hipFree(c->fresh_recs);
    hipFree(c->large_ids);
    hipFree(c->large_info);
    hipFree(c->redo_ids);
    hipFree(c->redo_cnt);
    hipFree(c->img_tmp);
    hipFree(c->img_pairs);
    hipFree(c->desc_dev);
    hipFree(c->sel_dev);
    hipFree(c->arena);
    hipFree(c->grp);
    hipFree(c->grp_tmp);
    hipFree(c->salt_pos);
    hipFree(c->fresh_args);
    hipFree(c->merge_scratch);
    hipFree(c->merge_counters);
    hipFree(c->powg);
    hipFree(c->lpn_s);
    hipFree(c->prf_req);
    hipFree(c->prf_core);
    hipFree(c->enc_arena);
    hipFree(c->dec_scratch);
    hipFree(c->dec_roff);
    hipFree(c->scan_scratch);
    hipFree(c->stats);
    if (c->pin) hipHostFree(c->pin);
    hipFree(c->check_buf);
    hipFree(c->check_scratch);
    sigma_tables_free(c->H);
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    delete c;
    if (caller_dev >= 0) hipSetDevice(caller_dev);
    return PVAC_OK;
}

int pvac_hip_ctx_set_stream(pvac_hip_ctx* c, void* s) {
    if (!c) return PVAC_EINVAL;
    if (c->own_stream && c->stream) {
        hipStreamSynchronize(c->stream);
        hipStreamDestroy(c->stream);
        c->stream = nullptr;
        c->own_stream = false;
    }
    // NULL selects the legacy null stream (torch's default stream is 0): every launch and copy
    // is then ordered with the caller's own work on that stream.
    c->stream = (hipStream_t)s;
    c->own_stream = false;
    return PVAC_OK;
}

void* pvac_hip_ctx_stream(pvac_hip_ctx* c) { return c ? (void*)c->stream : nullptr; }

int pvac_hip_ctx_synchronize(pvac_hip_ctx* c) {
    if (!c) return PVAC_EINVAL;
    return hip_fail(c, hipStreamSynchronize(c->stream), "synchronize");
}

int pvac_hip_ct_mul_redo_count(pvac_hip_ctx* c, uint64_t* out) {
    if (!c || !out) return PVAC_EINVAL;
    *out = c->redo_total;
    return PVAC_OK;
}

int pvac_hip_ctx_set_noise(pvac_hip_ctx* c, double noise_entropy_bits, double tuple2_fraction, double depth_slope_bits) {
    if (!c || !(noise_entropy_bits >= 0.0) || !(tuple2_fraction >= 0.0 && tuple2_fraction <= 1.0) ||
        !(depth_slope_bits >= 0.0) || noise_entropy_bits > 1e6 || depth_slope_bits > 1e6)
        return fail(c, PVAC_EINVAL, "ctx_set_noise: noise_entropy_bits, depth_slope_bits >= 0, tuple2_fraction in [0, 1]");
    c->noise_bits = noise_entropy_bits;
    c->noise_t2 = tuple2_fraction;
    c->noise_slope = depth_slope_bits;
    return PVAC_OK;
}

int pvac_hip_ct_mul_path_count(pvac_hip_ctx* c, uint64_t* out) {
    if (!c || !out) return PVAC_EINVAL;
    for (int k = 0; k < 4; ++k) out[k] = c->path_total[k];
    return PVAC_OK;
}

int pvac_hip_ct_mul_status(pvac_hip_ctx* c, uint32_t* out, size_t n) {
    if (!c || (!out && n)) return fail(c, PVAC_EINVAL, "ct_mul_status: bad arguments");
    if (!n) return PVAC_OK;
    if (n > c->last_mul_pairs) return fail(c, PVAC_EINVAL, "ct_mul_status: more pairs than the last ct_mul_exec held");
    const hipError_t e = hipMemcpyAsync(out, c->pair_status, n * 4, hipMemcpyDeviceToDevice, c->stream);
    return e == hipSuccess ? PVAC_OK : hip_fail(c, e, "ct_mul_status");
}

const char* pvac_hip_last_error(pvac_hip_ctx* c) { return c ? c->err.c_str() : "null context"; }

int pvac_hip_timing_enable(pvac_hip_ctx* c, int on) {
    if (!c) return PVAC_EINVAL;
    c->timing = on != 0;
    // events for the launches to come, created now rather than inside the timed launches
    while (c->timing && c->ev_pool.size() < 256) {
        hipEvent_t e{};
        if (hipEventCreate(&e) != hipSuccess) break;
        c->ev_pool.push_back(e);
    }
    return PVAC_OK;
}

int pvac_hip_timing_get(pvac_hip_ctx* c, const char* name, double* ms, uint64_t* launches) {
    if (!c || !name) return PVAC_EINVAL;
    flush_timers(c);
    auto it = c->timers.find(name);
    if (ms) *ms = it == c->timers.end() ? 0.0 : it->second.ms;
    if (launches) *launches = it == c->timers.end() ? 0 : it->second.launches;
    return PVAC_OK;
}

int pvac_hip_timing_reset(pvac_hip_ctx* c) {
    if (!c) return PVAC_EINVAL;
    flush_timers(c);
    c->timers.clear();
    return PVAC_OK;
}

// ---------------------------------------------------------------- Fp
int pvac_hip_fp_binop(pvac_hip_ctx* c, int op, const uint64_t* a_lo, const uint64_t* a_hi, const uint64_t* b_lo,
                      const uint64_t* b_hi, uint64_t* c_lo, uint64_t* c_hi, size_t n) {
    if (!c) return PVAC_EINVAL;
    if (op < PVAC_FP_ADD || op > PVAC_FP_INV) return fail(c, PVAC_EINVAL, "fp_binop: bad op");
    if (n && (!a_lo || !a_hi || !c_lo || !c_hi)) return fail(c, PVAC_EINVAL, "fp_binop: null array");
    if (n && op != PVAC_FP_NEG && op != PVAC_FP_INV && (!b_lo || !b_hi)) return fail(c, PVAC_EINVAL, "fp_binop: null b");
    scoped_timer t(c, "fp_binop");
    return hip_fail(c, launch_fp_binop(op, a_lo, a_hi, b_lo, b_hi, c_lo, c_hi, n, c->stream), "fp_binop");
}

// ---------------------------------------------------------------- ct_mul
namespace {

// Whether two key slots of [0, S) share a libstdc++ bucket among nb buckets (std::hash<u64> times the
// reference's 0x9E3779B97F4A7C15, arithmetic.hpp:72-77). A pair whose slots can share a bucket is not
// taken in the direct mode (its emit order then needs bucket leaders across A layers): chain step 2
// (|A.L| = 8, bucket counts near 49 K) has hundreds of such buckets, deeper steps none (the structured
// keys (lp << 32) | r spread perfectly there). Memoised per (nb, S, B): chunks of one step repeat them,
// and the slot -> key map depends on B (two contexts with different B can meet the same (nb, S)).
bool slots_share_bucket(uint64_t nb, uint64_t S, uint32_t Bm) {
    static std::mutex mu;
    static std::map<std::tuple<uint64_t, uint64_t, uint32_t>, bool> memo;
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = memo.find({nb, S, Bm});
        if (it != memo.end()) return it->second;
    }
    bool shared = false;
    if (S > nb) {
        shared = true;
    } else {
        std::vector<uint64_t> seen((nb + 63) / 64, 0);
        for (uint64_t s = 0; s < S && !shared; ++s) {
            const uint64_t key = ((s / Bm) << 32) | (s % Bm);
            const uint64_t b = (key * kGolden) % nb;
            const uint64_t m = 1ull << (b & 63);
            shared = (seen[b >> 6] & m) != 0;
            seen[b >> 6] |= m;
        }
    }
    std::lock_guard<std::mutex> g(mu);
    memo[{nb, S, Bm}] = shared;
    return shared;
}

// Pairs whose bucket count is at least twice their key-slot space (dense chain steps: reserve(|A.E||B.E|)
// buckets for |A.L||B.L|B slots) share their bucket groups with every pair of the same bucket count:
// the group of a slot depends only on (slot, B, bucket count). One static table per distinct bucket
// count replaces the per-pair bucket table + chains (k_large_link) and its zeroing; rank walks the
// static group and keeps the slots present in the pair (almost every slot is alone in its bucket).
int plan_static_groups(pvac_hip_ctx* c) {
    constexpr size_t kMaxCfg = 64;
    constexpr uint64_t kMaxWords = 1ull << 28;   // <= 1 GiB of tables
    std::map<uint64_t, uint64_t> cfg;             // bucket count -> max S
    for (const large_desc& d : c->large_host)
        if (d.nbm.d >= 2 * d.S && d.S) {
            uint64_t& m = cfg[d.nbm.d];
            m = std::max(m, d.S);
        }
    uint64_t words = 0, tmp_max = 0;
    for (auto& kv : cfg) {
        words += 2 * kv.second;
        tmp_max = std::max<uint64_t>(tmp_max, 1ull << std::max<uint32_t>(1, ceil_log2(2 * kv.second)));
    }
    if (cfg.empty() || cfg.size() > kMaxCfg || words > kMaxWords) return PVAC_OK;   // dynamic chains
    int rc = ensure_dev(c, c->grp, c->grp_cap, words, "alloc bucket-group tables");
    if (!rc) rc = ensure_dev(c, c->grp_tmp, c->grp_tmp_cap, 3 * tmp_max, "alloc bucket-group scratch");
    if (rc) return rc;
    std::map<uint64_t, uint64_t> off;   // bucket count -> head offset (next = head + S_max)
    uint64_t o = 0;
    for (auto& kv : cfg) {
        const uint64_t Sm = kv.second;
        const uint32_t hb = std::max<uint32_t>(1, ceil_log2(2 * Sm));
        const uint64_t hcap = 1ull << hb;
        unsigned long long* tk = (unsigned long long*)c->grp_tmp;   // [hcap] u64 keys, then [hcap] u32 heads
        uint32_t* th = c->grp_tmp + 2 * hcap;
        hipError_t e = hipMemsetAsync(c->grp_tmp, 0, 3 * hcap * 4, c->stream);
        if (e == hipSuccess)
            e = launch_grp_build(make_fastmod64(kv.first), c->prm.B, Sm, hb, c->grp + o, c->grp + o + Sm, tk, th,
                                 c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "build bucket-group tables");
        off[kv.first] = o;
        o += 2 * Sm;
    }
    for (large_desc& d : c->large_host) {
        auto it = off.find(d.nbm.d);
        if (it == off.end() || d.nbm.d < 2 * d.S || !d.S) continue;
        std::string why;
        large_desc x;
        rc = build_large_desc(x, d.pair, d.LA, d.LB, d.nA, d.nB, c->prm.B, why, true,
                              !c->large_no_direct && c->prm.edge_budget < (1ull << 28) &&   // 8-byte offsets < 2^31
                                  !slots_share_bucket(d.nbm.d, d.S, c->prm.B));
        if (rc) return fail(c, rc, why);
        x.g_head = it->second;
        x.g_next = it->second + cfg[d.nbm.d];
        d = x;
    }
    return PVAC_OK;
}

}  // namespace

int pvac_hip_ct_mul_plan(pvac_hip_ctx* c, const pvac_ct_batch* A, const pvac_ct_batch* B, pvac_ct_batch* C,
                         pvac_hip_plan* plan) {
    if (!c || !plan || !batch_ok(A) || !batch_ok(B) || !C || !C->l_off || !C->e_off)
        return fail(c, PVAC_EINVAL, "ct_mul_plan: bad arguments");
    if (A->n != B->n) return fail(c, PVAC_EINVAL, "ct_mul_plan: |A| != |B|");
    std::memset(plan, 0, sizeof *plan);
    plan->kind = 1;
    plan->n_pairs = A->n;
    C->n = A->n;
    c->large_host.clear();
    // every earlier plan goes stale now; this one is stamped valid only once it has succeeded, so
    // exec rejects a plan whose device work or descriptor build failed
    const uint32_t stamp = ++c->plan_stamp;
    if (!A->n) {
        plan->reserved[0] = stamp;
        return PVAC_OK;
    }
    int rc = ensure_pairs(c, A->n);
    if (rc) return rc;
    hipError_t e = hipMemsetAsync(c->stats, 0, sizeof(plan_stats), c->stream);
    if (e == hipSuccess)
        e = launch_plan_mul(*A, *B, *C, c->pair_class, c->large_ids, c->stats, c->nb_table, kNbTableLen, c->prm.B,
                            c->stream);
    if (e == hipSuccess)
        e = launch_exclusive_scan2_u64(C->l_off, C->e_off, A->n, c->scan_scratch, &c->totals[0], &c->totals[1], c->stream);
    plan_stats st{};
    if (e == hipSuccess) e = read_back(c, &st, c->stats, sizeof st);
    const unsigned long long tot[2] = {st.total_layers, st.total_edges};
    if (e != hipSuccess) return hip_fail(c, e, "ct_mul_plan");
    plan->total_layer_slots = tot[0];
    plan->total_edge_slots = tot[1];
    plan->n_small = A->n - st.n_large;   // k_plan_mul classifies every pair as small or large
    plan->n_large = st.n_large;
    plan->max_keys = st.max_keys;
    plan->max_prod = st.max_prod;
    plan->max_na = st.max_na;
    plan->max_nb = st.max_nb;
    plan->max_buckets = st.max_buckets;
    plan->max_layers = st.max_layers;
    if (st.n_large) {
        // shapes of the general-path pairs -> host descriptors (bucket counts from this libstdc++)
        std::vector<uint64_t> info(5 * st.n_large);
        e = launch_gather_large(*A, *B, c->large_ids, st.n_large, c->large_info, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(info.data(), c->large_info, info.size() * 8, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "ct_mul_plan (large)");
        c->large_host.resize(st.n_large);
        for (uint64_t k = 0; k < st.n_large; ++k) {
            std::string why;
            rc = build_large_desc(c->large_host[k], info[5 * k], info[5 * k + 1], info[5 * k + 2], info[5 * k + 3],
                                  info[5 * k + 4], c->prm.B, why);
            if (rc) {
                c->large_host.clear();
                return fail(c, rc, why);
            }
        }
        // deterministic launch order (the plan kernel appends in arrival order)
        std::sort(c->large_host.begin(), c->large_host.end(),
                  [](const large_desc& x, const large_desc& y) { return x.pair < y.pair; });
        rc = plan_static_groups(c);
        if (rc) {
            c->large_host.clear();
            return rc;
        }
    }
    plan->reserved[0] = stamp;
    return PVAC_OK;
}

namespace {

// A chain step's input held as dense images (ctx img_in, pvac_hip_ct_mul_chain) turned back into
// hash-order records for the pairs given as (pair, |A.E|) before a path that reads A's records (the
// non-direct kernels, the redo run). The device skips pairs whose flag is clear and clears the flags
// of the pairs it converts.
int images_to_records(pvac_hip_ctx* c, const pvac_ct_batch* A, const std::vector<std::pair<uint64_t, uint64_t>>& pn) {
    if (!c->img_in || pn.empty()) return PVAC_OK;
    std::vector<uint64_t> h(2 * pn.size());
    uint64_t tot = 0;
    for (size_t k = 0; k < pn.size(); ++k) {
        h[k] = pn[k].first;
        h[pn.size() + k] = tot;
        tot += pn[k].second;
    }
    int rc = ensure_dev(c, c->img_pairs, c->img_pairs_cap, h.size(), "alloc image pairs");
    if (!rc) rc = ensure_dev(c, c->img_tmp, c->img_tmp_cap, 3 * std::max<uint64_t>(tot, 1), "alloc image scratch");
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(c->img_pairs, h.data(), h.size() * 8, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess)
        e = launch_image_to_records(*A, c->img_in, c->img_pairs, (uint32_t)pn.size(), c->img_tmp, c->prm.B,
                                    c->img_grid_y, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);   // h is read from the host stack
    return e == hipSuccess ? PVAC_OK : hip_fail(c, e, "chain images to records");
}

// Runs the general path over the plan's large pairs in sub-batches that fit the scratch budget.
int run_large(pvac_hip_ctx* c, const pvac_ct_batch* A, const pvac_ct_batch* B, const uint64_t* nonces,
              pvac_ct_batch* C, uint32_t flags, uint32_t* salt_pos) {
    const size_t nl = c->large_host.size();
    int rc = ensure_dev(c, c->desc_dev, c->desc_cap, nl, "alloc large descriptors");
    if (!rc) rc = ensure_dev(c, c->sel_dev, c->sel_cap, nl, "alloc large descriptor order");
    if (rc) return rc;
    c->sel_host.resize(nl);
    // A-layers per workgroup and the XCD-aware grid of k_large_products_la: compile-time A/B knobs
#ifndef PVAC_LA_PER_WG
#define PVAC_LA_PER_WG kLaPerWG
#endif
#ifndef PVAC_LA_XCD
#define PVAC_LA_XCD 0
#endif
    constexpr uint32_t la_per_wg = PVAC_LA_PER_WG, la_xcd = PVAC_LA_XCD;
    static_assert(la_per_wg >= 1 && la_per_wg <= 64, "A layers per products workgroup");
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 8ull << 30;
    uint64_t budget = std::max<uint64_t>((uint64_t)(free_b / 2) / 4 + c->arena_words, 1ull << 24);
    budget = std::min<uint64_t>(budget, 16ull << 30);   // <= 64 GiB of scratch per sub-batch
    // a worker of pvac_hip_ct_mul_chain shares the device with the other workers: its share
    if (c->arena_cap_words) budget = std::min<uint64_t>(budget, std::max<uint64_t>(c->arena_cap_words, c->arena_words));
    c->large_exec = c->large_host;
    size_t i = 0;
    while (i < nl) {
        uint64_t words = 0;
        size_t j = i;
        uint64_t mS = 0, mZ = 0, mT = 0, mE = 0, mL = 0, mTa = 0, mLa = 0, mA = 0;
        bool dyn = false, all_ib = true, any_dir = false, all_dir = true;
        uint32_t mLBd = 0;
        uint64_t n_ib = 0, n_dir = 0;   // path counters, added once the sub-batch has launched
        while (j < nl && (j == i || words + c->large_exec[j].words <= budget) && j - i < 65535) {
            large_desc& d = c->large_exec[j];
            const uint64_t w = d.words;
            rebase_desc(d, words);
            words += w;
            // direct pairs have no per-key scratch: the slot- and edge-sized grids are the others'
            if (!d.direct) {
                mS = std::max(mS, d.S);
                mE = std::max(mE, d.capE);
                mA = std::max<uint64_t>(mA, d.iblk ? d.nA : 0);
            }
            mZ = std::max(mZ, d.zero_words);
            dyn |= d.g_head == kNoGrp;
            all_ib &= d.iblk != 0;
            any_dir |= d.direct != 0;
            all_dir &= d.direct != 0;
            n_ib += d.iblk;
            n_dir += d.direct;
            if (d.direct) mLBd = std::max<uint32_t>(mLBd, d.LB);
            mL = std::max(mL, std::max<uint64_t>(d.Lc, (uint64_t)d.LA + d.LB));
            ++j;
        }
        // products: pairs with few B layers (chain steps) take the A-layer-major kernel
        uint32_t n_la = 0;
        for (size_t k = i; k < j; ++k)
            if (c->large_exec[k].LB <= kLaMaxLB) c->sel_host[i + n_la++] = (uint32_t)(k - i);
        for (size_t k = i, q = n_la; k < j; ++k) {
            const large_desc& d = c->large_exec[k];
            const uint64_t tasks = (uint64_t)d.LA * d.LB;
            mTa = std::max(mTa, tasks);
            if (d.LB <= kLaMaxLB) {
                mLa = std::max<uint64_t>(mLa, (d.LA + la_per_wg - 1) / la_per_wg);
            } else {
                mT = std::max(mT, tasks);
                c->sel_host[i + q++] = (uint32_t)(k - i);
            }
        }
        if (words > c->arena_words) {
            // grow with 1/8 headroom (within the budget): batches of similar pairs differ by a few
            // words, and a free + re-malloc of tens of GB stalls for seconds
            uint64_t grown = std::max<uint64_t>(words, std::min<uint64_t>(words + words / 8, budget));
            hipStreamSynchronize(c->stream);
            const auto t0 = std::chrono::steady_clock::now();
            hipFree(c->arena);
            c->arena = nullptr;
            c->arena_words = 0;
            hipError_t e = hipMalloc(&c->arena, grown * 4);
            if (e == hipErrorOutOfMemory && grown > words) {   // without the headroom
                (void)hipGetLastError();
                grown = words;
                e = hipMalloc(&c->arena, grown * 4);
            }
            if (e == hipErrorOutOfMemory && j - i > 1) {
                // other contexts hold the HBM the budget counted on: split this sub-batch and retry
                (void)hipGetLastError();
                for (size_t k = i; k < j; ++k) c->large_exec[k] = c->large_host[k];
                budget = std::max<uint64_t>(words / 2, 1);
                continue;
            }
            if (e != hipSuccess) return hip_fail(c, e, "alloc ct_mul scratch arena");
            c->arena_words = grown;
            if (std::getenv("PVAC_DEBUG_ARENA"))
                std::fprintf(stderr, "[pvac] arena -> %.2f GB (free %.1f GB, sub-batch %zu pairs): %.1f ms\n",
                             grown * 4e-9, free_b * 1e-9, j - i,
                             std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        }
        hipError_t e = hipMemcpyAsync(c->desc_dev + i, c->large_exec.data() + i, (j - i) * sizeof(large_desc),
                                      hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(c->sel_dev + i, c->sel_host.data() + i, (j - i) * sizeof(uint32_t), hipMemcpyHostToDevice,
                               c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "upload large descriptors");
        mul_large_args a{};
        a.A = *A; a.B = *B; a.C = *C;
        a.nonces = nonces;
        a.pair_status = c->pair_status;
        a.desc = c->desc_dev + i;
        a.scratch = c->arena;
        a.nl = (uint32_t)(j - i);
        a.Bm = c->prm.B;
        a.canon_tag = c->prm.canon_tag;
        a.edge_budget = c->prm.edge_budget;
        a.flags = flags;
        a.salt_pos = salt_pos;
        a.grp = c->grp;
        a.sel = c->sel_dev + i;
        a.n_la = n_la;
        a.max_S = mS; a.max_zero = mZ; a.max_tasks = mT; a.max_capE = mE; a.max_lay = mL;
        a.max_tasks_all = mTa; a.max_la_wg = mLa; a.max_nA = mA;
        a.any_dyn = dyn ? 1u : 0u;
        a.all_iblk = all_ib ? 1u : 0u;
        a.any_direct = any_dir ? 1u : 0u;
        a.all_direct = all_dir ? 1u : 0u;
        a.dir_lb = std::max<uint32_t>(mLBd, 1u);
        a.redo_ids = c->redo_ids;
        a.redo_cnt = c->redo_cnt;
        a.A_img = c->img_in;
        a.C_img = c->img_out;
        a.img_count = c->img_out ? c->img_count : nullptr;
        a.la_per_wg = la_per_wg;
        a.la_xcd = la_xcd;
        e = launch_ct_mul_large(a, c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "ct_mul_large");
        c->path_total[1] += j - i;
        c->path_total[2] += n_ib;
        c->path_total[3] += n_dir;
        i = j;
    }
    return PVAC_OK;
}

// The fresh kernel and the general path's direct mode emit every key cell that received a
// product; a cell whose sum is 0 mod p (cancelling products or a zero weight, arithmetic.hpp:98-99)
// makes them flag the pair instead, and a direct pair that needs the canonical order or shares
// buckets is flagged too. Those pairs are re-run here on the general path's full layout, which
// folds every sum before it orders keys.
int redo_fresh_pairs(pvac_hip_ctx* c, const pvac_ct_batch* A, const pvac_ct_batch* B, const uint64_t* nonces,
                     pvac_ct_batch* C, uint32_t flags, uint32_t* salt_pos) {
    unsigned int cnt = 0;
    hipError_t e = read_back(c, &cnt, c->redo_cnt, sizeof cnt);
    if (e != hipSuccess) return hip_fail(c, e, "ct_mul_exec (redo count)");
    if (!cnt) {
        c->redo_cnt_dirty = false;
        return PVAC_OK;
    }
    std::vector<uint64_t> info(5 * (size_t)cnt);
    e = launch_gather_large(*A, *B, c->redo_ids, cnt, c->large_info, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(info.data(), c->large_info, info.size() * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "ct_mul_exec (redo shapes)");
    std::vector<large_desc> redo(cnt);
    for (size_t k = 0; k < cnt; ++k) {
        std::string why;
        const int rc = build_large_desc(redo[k], info[5 * k], info[5 * k + 1], info[5 * k + 2], info[5 * k + 3],
                                        info[5 * k + 4], c->prm.B, why);
        if (rc) return fail(c, rc, why);
    }
    std::sort(redo.begin(), redo.end(), [](const large_desc& x, const large_desc& y) { return x.pair < y.pair; });
    // a chain step's image inputs become records first; the redo run reads and writes records only
    uint32_t* const img_in = c->img_in;
    uint32_t* const img_out = c->img_out;
    if (img_in) {
        std::vector<std::pair<uint64_t, uint64_t>> pn;
        for (const large_desc& d : redo) pn.emplace_back(d.pair, d.nA);
        const int rc = images_to_records(c, A, pn);
        if (rc) return rc;
    }
    c->img_in = nullptr;
    c->img_out = nullptr;
    struct img_restore {
        pvac_hip_ctx* c;
        uint32_t *in, *out;
        ~img_restore() { c->img_in = in; c->img_out = out; }
    } img_guard{c, img_in, img_out};
    // run them as the context's large-pair set, then restore the plan's own set and its tables
    std::vector<large_desc> plan_set;
    plan_set.swap(c->large_host);
    c->large_host.swap(redo);
    c->large_no_direct = true;   // the exact path: per-key sums, no presence-based positions
    int rc = plan_static_groups(c);
    if (!rc) rc = run_large(c, A, B, nonces, C, flags, salt_pos);
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = hip_fail(c, hipErrorUnknown, "ct_mul_exec (redo)");
    c->large_no_direct = false;
    c->large_host.swap(plan_set);
    if (!rc) {
        c->redo_total += cnt;
        // the plan's own static group tables were replaced by the redo set's: rebuild them
        if (!c->large_host.empty()) rc = plan_static_groups(c);
    }
    // on failure the group tables may still belong to the redo set: no exec may reuse this plan
    if (rc) ++c->plan_stamp;
    return rc;
}

}  // namespace

int pvac_hip_ct_mul_exec(pvac_hip_ctx* c, const pvac_hip_plan* plan, const pvac_ct_batch* A, const pvac_ct_batch* B,
                         const uint64_t* nonces, const uint64_t* salts, pvac_ct_batch* C, uint32_t flags) {
    if (!c || !plan || plan->kind != 1 || !batch_ok(A) || !batch_ok(B) || !batch_ok(C))
        return fail(c, PVAC_EINVAL, "ct_mul_exec: bad arguments");
    if (A->n != plan->n_pairs || B->n != plan->n_pairs) return fail(c, PVAC_EINVAL, "ct_mul_exec: plan mismatch");
    if (!A->n) return PVAC_OK;
    if (plan->reserved[0] != c->plan_stamp || plan->n_large != c->large_host.size())
        return fail(c, PVAC_EINVAL, "ct_mul_exec: plan is not this context's latest ct_mul plan");
    if (!nonces) return fail(c, PVAC_EINVAL, "ct_mul_exec: nonces required");
    if (!C->layers || !C->meta || !C->w_lo || !C->w_hi) return fail(c, PVAC_EINVAL, "ct_mul_exec: output arrays");
    c->last_mul_pairs = 0;   // pair_status is valid again only once this exec has launched its kernels
    const bool with_sigma = (flags & PVAC_MUL_WITH_SIGMA) != 0;
    if (with_sigma && (!salts || !C->sigma || !c->H.ready))
        return fail(c, PVAC_EINVAL, "ct_mul_exec: WITH_SIGMA needs salts, C->sigma and H");
    uint32_t* salt_pos = nullptr;
    if (with_sigma) {
        int rc = ensure_dev(c, c->salt_pos, c->salt_cap, plan->total_edge_slots, "alloc salt positions");
        if (rc) return rc;
        salt_pos = c->salt_pos;
    }
    if (c->redo_cnt_dirty) {   // a read-back of zero leaves it clean: no memset per exec
        const hipError_t e = hipMemsetAsync(c->redo_cnt, 0, sizeof(unsigned int), c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "reset redo count");
    }
    c->redo_cnt_dirty = true;   // until this exec reads back a zero count
    c->path_total[0] += plan->n_small;
    if (plan->n_small) {
        mul_fresh_args a;
        std::memset(&a, 0, sizeof a);   // padding too: the upload below is skipped on equal bytes
        a.A = *A; a.B = *B; a.C = *C;
        a.recs = c->fresh_recs;
        a.nonces = nonces;
        a.pair_class = c->pair_class;
        a.pair_status = c->pair_status;
        a.nb_table = c->nb_table;
        a.nb_magic = c->nb_magic;
        a.salt_pos = salt_pos;
        a.redo_ids = c->redo_ids;
        a.redo_cnt = c->redo_cnt;
        a.canon_tag = c->prm.canon_tag;
        a.edge_budget = c->prm.edge_budget;
        a.Bm = c->prm.B;
        a.flags = flags;
        a.ks_max = std::max<uint32_t>(plan->max_keys, 32u);   // LDS sizing floor (0-key batches)
        a.prod_max = plan->max_prod;
        a.na_max = plan->max_na;
        a.nb_max = plan->max_nb;
        a.buckets_max = plan->max_buckets;
        a.layers_max = plan->max_layers;
        {
            scoped_timer t(c, "mul_layers_fresh");
            hipError_t e = launch_mul_layers_fresh(a, c->stream);
            if (e != hipSuccess) return hip_fail(c, e, "mul_layers_fresh");
        }
        if (!c->fresh_args) {
            hipError_t ea = hipMalloc(&c->fresh_args, sizeof(mul_fresh_args));
            if (ea != hipSuccess) return hip_fail(c, ea, "alloc fresh args");
        }
        // stream-ordered copy from the ctx's host mirror (kept alive until the next exec); a batch
        // exec'd again into the same buffers (the kernels never write their arguments) reuses it
        hipError_t e = hipSuccess;
        if (!c->fresh_args_uploaded || std::memcmp(&c->fresh_args_host, &a, sizeof a) != 0) {
            c->fresh_args_uploaded = false;
            std::memcpy(&c->fresh_args_host, &a, sizeof a);
            e = hipMemcpyAsync(c->fresh_args, &c->fresh_args_host, sizeof a, hipMemcpyHostToDevice, c->stream);
            c->fresh_args_uploaded = e == hipSuccess;
        }
        if (e != hipSuccess) return hip_fail(c, e, "upload fresh args");
        scoped_timer t(c, "ct_mul_fresh");
        e = launch_ct_mul_fresh(a, c->fresh_args, c->num_cus, c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "ct_mul_fresh");
    }
    if (plan->n_large && (flags & PVAC_MUL_ORDER_CANONICAL) &&
        std::any_of(c->large_host.begin(), c->large_host.end(), [](const large_desc& d) { return d.direct != 0; })) {
        // the direct mode emits hash order only: with the canonical order asked for, its pairs would
        // all be redone, so take them on the full layout from the start (descriptors rebuilt once;
        // the plan stays valid, its direct pairs now run the exact path)
        c->large_no_direct = true;
        const int rc = plan_static_groups(c);
        c->large_no_direct = false;
        if (rc) {
            ++c->plan_stamp;
            return rc;
        }
    }
    if (plan->n_large && c->img_in) {   // chain step: image inputs of pairs off the direct mode -> records
        std::vector<std::pair<uint64_t, uint64_t>> pn;
        for (const large_desc& d : c->large_host)
            if (!d.direct) pn.emplace_back(d.pair, d.nA);
        const int rc = images_to_records(c, A, pn);
        if (rc) return rc;
    }
    if (plan->n_large) {
        scoped_timer t(c, "ct_mul_large");
        int rc = run_large(c, A, B, nonces, C, flags, salt_pos);
        if (rc) return rc;
    }
    {
        int rc = redo_fresh_pairs(c, A, B, nonces, C, flags, salt_pos);
        if (rc) return rc;
    }
    c->last_mul_pairs = A->n;
    if (with_sigma) {
        scoped_timer t(c, "sigma");
        hipError_t e = launch_sigma(c->H, c->prm, *C, salts, salt_pos, c->num_cus, c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "sigma");
    }
    return PVAC_OK;
}

int pvac_hip_ct_mul(pvac_hip_ctx* c, const pvac_ct_batch* A, const pvac_ct_batch* B, pvac_ct_batch* C,
                    uint64_t layer_cap, uint64_t edge_cap, const uint64_t* nonces, const uint64_t* salts,
                    uint32_t flags, pvac_hip_plan* plan_out) {
    pvac_hip_plan p{};
    int rc = pvac_hip_ct_mul_plan(c, A, B, C, &p);
    if (plan_out) *plan_out = p;
    if (rc) return rc;
    if (p.total_layer_slots > layer_cap || p.total_edge_slots > edge_cap) {
        ++c->plan_stamp;   // the plan's offsets do not fit C: it is not exec'd
        return fail(c, PVAC_ENOMEM, "ct_mul: output capacity below the plan's totals");
    }
    return pvac_hip_ct_mul_exec(c, &p, A, B, nonces, salts, C, flags);
}

// ---------------------------------------------------------------- ct_add / ct_sub
int pvac_hip_ct_add_plan(pvac_hip_ctx* c, const pvac_ct_batch* A, const pvac_ct_batch* B, pvac_ct_batch* C,
                         pvac_hip_plan* plan) {
    if (!c || !plan || !batch_ok(A) || !batch_ok(B) || !C || !C->l_off || !C->e_off)
        return fail(c, PVAC_EINVAL, "ct_add_plan: bad arguments");
    if (A->n != B->n) return fail(c, PVAC_EINVAL, "ct_add_plan: |A| != |B|");
    std::memset(plan, 0, sizeof *plan);
    plan->kind = 2;
    plan->n_pairs = A->n;
    C->n = A->n;
    if (!A->n) return PVAC_OK;
    int rc = ensure_pairs(c, A->n);
    if (rc) return rc;
    c->merge_host.clear();
    // as in ct_mul_plan: earlier plans go stale now, this one is stamped only once it has succeeded
    const uint32_t stamp = ++c->plan_stamp;
    hipError_t e = hipMemsetAsync(c->stats, 0, sizeof(plan_stats), c->stream);
    if (e == hipSuccess)
        e = launch_plan_add(*A, *B, *C, c->stats, c->pair_class, c->large_ids, c->prm.edge_budget, c->stream);
    if (e == hipSuccess)
        e = launch_exclusive_scan2_u64(C->l_off, C->e_off, A->n, c->scan_scratch, &c->totals[0], &c->totals[1], c->stream);
    plan_stats st{};
    if (e == hipSuccess) e = read_back(c, &st, c->stats, sizeof st);
    const unsigned long long tot[2] = {st.total_layers, st.total_edges};
    if (e != hipSuccess) return hip_fail(c, e, "ct_add_plan");
    plan->total_layer_slots = tot[0];
    plan->total_edge_slots = tot[1];
    plan->max_layers = st.max_layers;
    plan->n_large = st.n_large;
    plan->n_small = A->n - st.n_large;
    if (st.n_large) {   // guard_budget pairs: shapes and offsets for the per-pair merge launches
        std::vector<uint64_t> info(8 * st.n_large);
        e = launch_gather_merge(*A, *B, *C, c->large_ids, st.n_large, c->large_info, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(info.data(), c->large_info, info.size() * 8, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "ct_add_plan (merge)");
        for (uint64_t k = 0; k < st.n_large; ++k) {
            const uint64_t* o = &info[8 * k];
            merge_pair_info m{};
            m.pair = o[0];
            m.LA = (uint32_t)o[1];
            m.L = (uint32_t)(o[1] + o[2]);
            m.nA = o[3];
            m.nB = o[4];
            m.aeo = o[5];
            m.beo = o[6];
            m.ceo = o[7];
            if (m.nA + m.nB >= (1ull << 31) || (uint64_t)m.L * c->prm.B * 2 >= 0xFFFFFFFFull) {
                c->merge_host.clear();
                return fail(c, PVAC_ENOSYS, "ct_add_plan: over-budget pair beyond 2^31 edges or 2^32 keys");
            }
            c->merge_host.push_back(m);
        }
        std::sort(c->merge_host.begin(), c->merge_host.end(),
                  [](const merge_pair_info& x, const merge_pair_info& y) { return x.pair < y.pair; });
    }
    plan->reserved[0] = stamp;
    return PVAC_OK;
}

int pvac_hip_ct_add_exec(pvac_hip_ctx* c, const pvac_hip_plan* plan, const pvac_ct_batch* A, const pvac_ct_batch* B,
                         int negate_b, pvac_ct_batch* C) {
    if (!c || !plan || plan->kind != 2 || !batch_ok(A) || !batch_ok(B) || !batch_ok(C))
        return fail(c, PVAC_EINVAL, "ct_add_exec: bad arguments");
    if (A->n != plan->n_pairs || B->n != plan->n_pairs) return fail(c, PVAC_EINVAL, "ct_add_exec: plan mismatch");
    if (!A->n) return PVAC_OK;
    if (plan->max_layers > 30000) return fail(c, PVAC_ENOSYS, "ct_add_exec: > 30000 layers per cipher");
    if (plan->n_large && (plan->reserved[0] != c->plan_stamp || plan->n_large != c->merge_host.size()))
        return fail(c, PVAC_EINVAL, "ct_add_exec: plan is not this context's latest plan");
    {
        scoped_timer t(c, "ct_add");
        const int rc = hip_fail(c,
                                launch_ct_add(*A, *B, *C, negate_b, plan->max_layers,
                                              plan->n_large ? c->pair_class : nullptr, c->stream),
                                "ct_add");
        if (rc) return rc;
    }
    if (!plan->n_large) return PVAC_OK;
    // guard_budget (encrypt.hpp:106-111): compact_edges + compact_layers per over-budget pair
    scoped_timer t(c, "ct_add_merge");
    if (!c->merge_counters) {
        hipError_t e = hipMalloc(&c->merge_counters, 2 * sizeof(unsigned long long));
        if (e != hipSuccess) return hip_fail(c, e, "alloc merge counters");
    }
    for (const merge_pair_info& m : c->merge_host) {
        const size_t need = merge_scratch_bytes(m.nA + m.nB, m.L);
        if (need > c->merge_cap) {
            hipFree(c->merge_scratch);
            c->merge_scratch = nullptr;
            c->merge_cap = 0;
            hipError_t e = hipMalloc(&c->merge_scratch, need);
            if (e != hipSuccess) return hip_fail(c, e, "alloc merge scratch");
            c->merge_cap = need;
        }
        const int rc = hip_fail(c,
                                launch_add_merge(*A, *B, *C, m.pair, m, c->prm.B, negate_b, c->merge_scratch,
                                                 c->merge_cap, c->merge_counters, c->stream),
                                "ct_add merge");
        if (rc) return rc;
    }
    return PVAC_OK;
}

int pvac_hip_ct_scale(pvac_hip_ctx* c, pvac_ct_batch* X, uint64_t s_lo, uint64_t s_hi) {
    if (!c || !batch_ok(X)) return PVAC_EINVAL;
    scoped_timer t(c, "ct_scale");
    return hip_fail(c, launch_ct_scale(*X, s_lo, s_hi, c->stream), "ct_scale");
}

// ---------------------------------------------------------------- sigma / H
int pvac_hip_ctx_set_H(pvac_hip_ctx* c, const uint64_t* H, uint32_t n_cols, uint32_t wpc) {
    if (!c || !H) return PVAC_EINVAL;
    if (n_cols != c->prm.n_bits || wpc != (c->prm.m_bits + 63) / 64) return fail(c, PVAC_EINVAL, "set_H: shape");
    try {
        const int rc = hip_fail(c, sigma_tables_from_dense(c->H, c->prm, H, c->stream), "set_H");
        if (rc) return rc;
        ++c->H_gen;
        // H_digest = SHA-256("H|v2" || le64 m || le64 n || le64 wt || column bytes) (matrix.hpp:218-250)
        const size_t colbytes = (c->prm.m_bits + 7) / 8;
        std::vector<uint8_t> msg(28 + (size_t)n_cols * colbytes);
        std::memcpy(msg.data(), "H|v2", 4);
        const uint64_t hdr[3] = {c->prm.m_bits, c->prm.n_bits, c->prm.h_col_wt};
        for (int k = 0; k < 3; ++k)
            for (int i = 0; i < 8; ++i) msg[4 + 8 * k + i] = (uint8_t)(hdr[k] >> (8 * i));
        for (uint32_t col = 0; col < n_cols; ++col)
            for (size_t b = 0; b < colbytes; ++b)
                msg[28 + (size_t)col * colbytes + b] = (uint8_t)(H[(size_t)col * wpc + b / 8] >> (8 * (b % 8)));
        sha256_host(msg.data(), msg.size(), c->H_digest);
        c->have_digest = true;
        return PVAC_OK;
    } catch (const std::exception& ex) {
        return fail(c, PVAC_ENOMEM, std::string("set_H: ") + ex.what());
    }
}

int pvac_hip_ctx_gen_H(pvac_hip_ctx* c, uint8_t digest[32]) {
    if (!c) return PVAC_EINVAL;
    try {
        scoped_timer t(c, "gen_H");
        uint8_t d[32];
        const int rc = hip_fail(c, sigma_tables_generate(c->H, c->prm, d, c->stream), "gen_H");
        if (rc) return rc;
        ++c->H_gen;
        std::memcpy(c->H_digest, d, 32);
        c->have_digest = true;
        if (digest) std::memcpy(digest, d, 32);
        return PVAC_OK;
    } catch (const std::exception& ex) {
        return fail(c, PVAC_ENOMEM, std::string("gen_H: ") + ex.what());
    }
}

int pvac_hip_sigma_batch(pvac_hip_ctx* c, pvac_ct_batch* X, const uint64_t* salts) {
    if (!c || !batch_ok(X) || !salts || !X->sigma) return PVAC_EINVAL;
    if (!c->H.ready) return fail(c, PVAC_EINVAL, "sigma_batch: H not set");
    scoped_timer t(c, "sigma");
    return hip_fail(c, launch_sigma(c->H, c->prm, *X, salts, nullptr, c->num_cus, c->stream), "sigma");
}

// ---------------------------------------------------------------- LPN PRF
int pvac_hip_ctx_set_secret(pvac_hip_ctx* c, const uint64_t prf_k[4], const uint64_t* lpn_s_host, uint32_t lpn_n,
                            uint32_t lpn_t, uint32_t tau_num, uint32_t tau_den) {
    if (!c || !prf_k || !lpn_s_host) return fail(c, PVAC_EINVAL, "set_secret: arguments");
    const uint32_t words = (lpn_n + 63) / 64;
    if (lpn_n == 0 || words > 64 || tau_den == 0 || tau_num > tau_den)
        return fail(c, PVAC_EINVAL, "set_secret: lpn_n must be in [1, 4096], 0 <= tau_num <= tau_den, tau_den > 0");
    if (lpn_t < 127) return fail(c, PVAC_ENOSYS, "set_secret: lpn_t < 127 not supported");
    hipFree(c->lpn_s);
    c->lpn_s = nullptr;
    c->have_secret = false;
    hipError_t e = hipMalloc(&c->lpn_s, 64 * 8);
    if (e == hipSuccess) e = hipMemset(c->lpn_s, 0, 64 * 8);
    if (e == hipSuccess) e = hipMemcpy(c->lpn_s, lpn_s_host, (size_t)words * 8, hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(c, e, "set_secret");
    std::memcpy(c->prf_k, prf_k, 32);
    c->lpn_words = words;
    c->lpn_t = lpn_t;
    c->tau_num = tau_num;
    c->tau_den = tau_den;
    c->have_secret = true;
    return PVAC_OK;
}

int pvac_hip_ctx_set_H_digest(pvac_hip_ctx* c, const uint8_t digest[32]) {
    if (!c || !digest) return PVAC_EINVAL;
    std::memcpy(c->H_digest, digest, 32);
    c->have_digest = true;
    return PVAC_OK;
}

namespace {

uint64_t fnv1a(const char* d) {   // lpn.hpp:150-157
    uint64_t h = 0xcbf29ce484222325ull;
    for (const char* p = d; *p; ++p) { h ^= (uint8_t)*p; h *= 0x100000001b3ull; }
    return h;
}

// constants of the key derivation (lpn.hpp:159-186); the first message block is fixed per key
int prf_setup(pvac_hip_ctx* c, prf_consts& k) {
    if (!c->have_secret) return fail(c, PVAC_EINVAL, "prf: secret key not set (pvac_hip_ctx_set_secret)");
    if (!c->have_digest) return fail(c, PVAC_EINVAL, "prf: H_digest unknown (gen_H, set_H or set_H_digest)");
    if (!c->aes_tables) {
        hipError_t e = prf_upload_tables(c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "prf tables");
        c->aes_tables = true;
    }
    uint8_t m[64];
    for (int i = 0; i < 4; ++i)
        for (int b = 0; b < 8; ++b) m[8 * i + b] = (uint8_t)(c->prf_k[i] >> (8 * b));
    for (int b = 0; b < 8; ++b) m[32 + b] = (uint8_t)(c->prm.canon_tag >> (8 * b));
    std::memcpy(m + 40, c->H_digest, 24);
    uint32_t w[16];
    for (int i = 0; i < 16; ++i)
        w[i] = (uint32_t)m[4 * i] << 24 | (uint32_t)m[4 * i + 1] << 16 | (uint32_t)m[4 * i + 2] << 8 | m[4 * i + 3];
    sha_state st;
    sha_init(st);
    sha_compress(st, w);
    std::memcpy(k.mid, st.h, 32);
    uint64_t tail = 0;
    for (int b = 0; b < 8; ++b) tail |= (uint64_t)c->H_digest[24 + b] << (8 * b);
    k.hd_tail = tail;
    static const char* const doms[6] = {"pvac.prf.r.1", "pvac.prf.r.2", "pvac.prf.r.3",
                                        "pvac.prf.noise.1", "pvac.prf.noise.2", "pvac.prf.noise.3"};
    for (int d = 0; d < 6; ++d) k.dom_hash[d] = fnv1a(doms[d]);
    k.toep_hash = fnv1a("pvac.dom.toeplitz");
    k.s_bits = c->lpn_s;
    k.s_words = c->lpn_words;
    k.tau_num = c->tau_num;
    k.tau_den = c->tau_den;
    return PVAC_OK;
}

int ensure_prf_scratch(pvac_hip_ctx* c, uint64_t cores) {
    int rc = ensure_dev(c, c->prf_req, c->prf_req_cap, cores * prf_request_bytes(), "alloc prf requests");
    if (rc) return rc;
    return ensure_dev(c, c->prf_core, c->prf_core_cap, 2 * cores, "alloc prf cores");
}

}  // namespace

int pvac_hip_prf(pvac_hip_ctx* c, int kind, size_t n, const uint64_t* seeds, uint64_t* out) {
    if (!c || kind < 0 || kind > 7 || (n && (!seeds || !out))) return fail(c, PVAC_EINVAL, "prf: arguments");
    if (!n) return PVAC_OK;
    prf_consts k{};
    int rc = prf_setup(c, k);
    if (rc) return rc;
    rc = ensure_prf_scratch(c, 3 * (uint64_t)n);
    if (rc) return rc;
    scoped_timer t(c, "prf");
    return hip_fail(c, launch_prf(k, kind, seeds, n, c->prf_req, c->prf_core, out, c->stream), "prf");
}

// ---------------------------------------------------------------- enc_value
namespace {
// ops/encrypt.hpp:16-27 with the context's noise Params (the reference's defaults: noise_entropy_bits
// 120, tuple2_fraction 0.55, depth_slope_bits 16; pvac_hip_ctx_set_noise); enc_value uses depth_hint 0
void plan_noise(const pvac_hip_ctx* c, int depth, uint32_t& z2, uint32_t& z3) {
    const uint32_t B = c->prm.B;
    const double budget = c->noise_bits + c->noise_slope * std::max(0, depth);
    const double per2 = 2.0 * std::log2((double)B), per3 = 3.0 * std::log2((double)B);
    int a = std::max(0, (int)std::floor((budget * c->noise_t2) / std::max(1e-6, per2)));
    int b = std::max(0, (int)std::floor((budget * (1.0 - c->noise_t2)) / std::max(1e-6, per3)));
    if (a + b == 1) { if (b > 0) ++b; else ++a; }
    z2 = (uint32_t)a;
    z3 = (uint32_t)b;
}
}  // namespace

int pvac_hip_enc_caps(pvac_hip_ctx* c, uint32_t* layers_per_value, uint32_t* edges_per_value, uint32_t* draws_hint) {
    return pvac_hip_enc_caps_depth(c, 0, layers_per_value, edges_per_value, draws_hint);
}

int pvac_hip_enc_caps_depth(pvac_hip_ctx* c, int depth_hint, uint32_t* layers_per_value, uint32_t* edges_per_value,
                            uint32_t* draws_hint) {
    if (!c) return PVAC_EINVAL;
    uint32_t z2, z3;
    plan_noise(c, depth_hint, z2, z3);
    if ((uint64_t)8 + 2ull * z2 + 3ull * z3 > kEncPreMax)
        return fail(c, PVAC_ENOSYS, "enc_caps: noise plan beyond 256 pre-merge edges per half (depth hint > 124 with the default Params)");
    const uint32_t npre = 8 + 2 * z2 + 3 * z3;
    if (layers_per_value) *layers_per_value = 2;
    if (edges_per_value) *edges_per_value = 2 * npre;
    // mask 2 + per half: nonce 2, signal 2*8 + 2*7, salts npre, noise picks/signs/coefficients, shuffle
    if (draws_hint) *draws_hint = 2 + 2 * (2 + 16 + 14 + npre + z2 * 5 + z3 * 10 + npre) + 64;
    return PVAC_OK;
}

int pvac_hip_enc_value(pvac_hip_ctx* c, size_t n, const uint64_t* values, const uint64_t* rnd, uint32_t rnd_stride,
                       pvac_ct_batch* C, uint32_t flags, uint32_t* status) {
    return pvac_hip_enc_value_depth(c, n, values, rnd, rnd_stride, 0, C, flags, status);
}

int pvac_hip_enc_value_depth(pvac_hip_ctx* c, size_t n, const uint64_t* values, const uint64_t* rnd, uint32_t rnd_stride,
                             int depth_hint, pvac_ct_batch* C, uint32_t flags, uint32_t* status) {
    if (!c || !C || (n && (!values || !rnd || !status))) return fail(c, PVAC_EINVAL, "enc_value: arguments");
    if (!C->l_off || !C->l_cnt || !C->layers || !C->e_off || !C->e_cnt || !C->meta || !C->w_lo || !C->w_hi)
        return fail(c, PVAC_EINVAL, "enc_value: output arrays");
    const bool with_sigma = (flags & PVAC_ENC_WITH_SIGMA) != 0;
    if (with_sigma && (!C->sigma || !c->H.ready || C->sigma_words != c->prm.m_bits / 64))
        return fail(c, PVAC_EINVAL, "enc_value: WITH_SIGMA needs C->sigma (m_bits/64 words per edge) and H");
    if (!c->powg) return fail(c, PVAC_EINVAL, "enc_value: powg_B not set (pvac_hip_ctx_set_powg)");
    C->n = n;
    if (!n) return PVAC_OK;
    prf_consts k{};
    int rc = prf_setup(c, k);
    if (rc) return rc;
    enc_plan_args a{};
    a.values = values;
    a.rnd = rnd;
    a.stride = rnd_stride;
    a.B = c->prm.B;
    plan_noise(c, depth_hint, a.Z2, a.Z3);
    a.n = n;
    a.canon = c->prm.canon_tag;
    a.powg = c->powg;
    const uint32_t npre = 8 + 2 * a.Z2 + 3 * a.Z3;
    if ((uint64_t)8 + 2ull * a.Z2 + 3ull * a.Z3 > kEncPreMax)
        return fail(c, PVAC_ENOSYS, "enc_value: noise plan beyond 256 pre-merge edges per half (depth hint > 124 with the default Params)");
    const uint64_t cores = (uint64_t)n * enc_cores_per_value(a.Z2, a.Z3);
    const uint64_t pe = (uint64_t)n * 2 * npre;
    const uint32_t sw = c->prm.m_bits / 64;
    // arena: halves | requests | cores | pre CSR (4 x n) | pre layers | meta, w_lo, w_hi, salt | sigma
    auto al = [](uint64_t b) { return (b + 255) & ~255ull; };
    const uint64_t off_req = al((uint64_t)2 * n * enc_half_bytes(npre));
    const uint64_t off_core = off_req + al(cores * prf_request_bytes());
    const uint64_t off_csr = off_core + al(cores * 16);
    const uint64_t off_lay = off_csr + al((uint64_t)n * 32);
    const uint64_t off_e = off_lay + al((uint64_t)n * 2 * sizeof(pvac_layer));
    const uint64_t off_sig = off_e + al(pe * 32);
    const uint64_t total = off_sig + (with_sigma ? al(pe * sw * 8) : 0);
    if (total > c->enc_arena_cap) {
        hipFree(c->enc_arena);
        c->enc_arena = nullptr;
        c->enc_arena_cap = 0;
        hipError_t e = hipMalloc(&c->enc_arena, total);
        if (e != hipSuccess) return hip_fail(c, e, "alloc enc scratch");
        c->enc_arena_cap = total;
    }
    uint8_t* A = c->enc_arena;
    pvac_ct_batch pre{};
    pre.n = n;
    pre.l_off = (uint64_t*)(A + off_csr);
    pre.l_cnt = pre.l_off + n;
    pre.e_off = pre.l_cnt + n;
    pre.e_cnt = pre.e_off + n;
    pre.layers = (pvac_layer*)(A + off_lay);
    pre.meta = (uint64_t*)(A + off_e);
    pre.w_lo = pre.meta + pe;
    pre.w_hi = pre.w_lo + pe;
    uint64_t* pre_salt = pre.w_hi + pe;
    pre.sigma = with_sigma ? (uint64_t*)(A + off_sig) : nullptr;
    pre.sigma_words = with_sigma ? sw : 0;
    scoped_timer t(c, "enc_value");
    hipError_t e = launch_enc_plan(a, A, (prf_request*)(A + off_req), pre, pre_salt, status, c->stream);
    if (e == hipSuccess) e = launch_prf_cores(k, A + off_req, cores, (uint64_t*)(A + off_core), c->stream);
    if (e == hipSuccess) e = launch_enc_weights(a, A, (const uint64_t*)(A + off_core), pre, c->stream);
    if (e == hipSuccess && with_sigma) e = launch_sigma(c->H, c->prm, pre, pre_salt, nullptr, c->num_cus, c->stream);
    pvac_ct_batch out = *C;
    if (!with_sigma) out.sigma = nullptr;
    if (e == hipSuccess) e = launch_enc_finish(a, A, pre, out, status, c->stream);
    return hip_fail(c, e, "enc_value");
}

int pvac_hip_base_R(pvac_hip_ctx* c, const pvac_ct_batch* X, uint64_t* R_out) {
    if (!c || !batch_ok(X) || (X->n && !R_out)) return fail(c, PVAC_EINVAL, "base_R: arguments");
    if (!X->n) return PVAC_OK;
    prf_consts k{};
    int rc = prf_setup(c, k);
    if (rc) return rc;
    // layer slots are addressed through l_off / l_cnt on the device: gather every slot's seed
    std::vector<uint64_t> lo(X->n), lc(X->n);
    hipError_t e = hipMemcpyAsync(lo.data(), X->l_off, X->n * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(lc.data(), X->l_cnt, X->n * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "base_R (offsets)");
    uint64_t slots = 0;
    for (uint64_t i = 0; i < X->n; ++i) slots = std::max(slots, lo[i] + lc[i]);
    if (!slots) return PVAC_OK;
    rc = ensure_prf_scratch(c, 4 * slots);   // 3 cores per slot + the BASE flags behind them
    if (rc) return rc;
    scoped_timer t(c, "base_R");
    return hip_fail(c, launch_base_R(k, *X, slots, c->prf_req, c->prf_core, R_out, c->stream), "base_R");
}

// ---------------------------------------------------------------- measured ALU ceilings
int pvac_hip_alu_ceiling(pvac_hip_ctx* c, int kind, double* per_s) {
    if (!c || !per_s || kind < 0 || kind > 5) return fail(c, PVAC_EINVAL, "alu_ceiling: bad arguments");
    const hipError_t e = run_alu_probe(kind, c->num_cus, c->stream, per_s);
    return e == hipSuccess ? PVAC_OK : hip_fail(c, e, "alu_ceiling");
}

int pvac_hip_issue_probe(pvac_hip_ctx* c, int op, int waves_per_simd, double* per_s, double* clock_hz) {
    if (!c || !per_s || !clock_hz) return fail(c, PVAC_EINVAL, "issue_probe: bad arguments");
    const hipError_t e = run_issue_probe(op, waves_per_simd, c->num_cus, c->stream, per_s, clock_hz);
    return e == hipSuccess ? PVAC_OK : hip_fail(c, e, "issue_probe");
}

// ---------------------------------------------------------------- gsum invariant
int pvac_hip_check_mul_gsum(pvac_hip_ctx* c, const pvac_ct_batch* A, const pvac_ct_batch* B, const pvac_ct_batch* C,
                            const uint64_t* nonces, uint32_t* status, uint64_t* n_bad) {
    if (!c || !n_bad || !batch_ok(A) || !batch_ok(B) || !batch_ok(C) || !nonces)
        return fail(c, PVAC_EINVAL, "check_mul_gsum: bad arguments");
    if (A->n != B->n || A->n != C->n) return fail(c, PVAC_EINVAL, "check_mul_gsum: batch sizes differ");
    if (!c->powg) return fail(c, PVAC_EINVAL, "check_mul_gsum: powg_B not set (pvac_hip_ctx_set_powg)");
    *n_bad = 0;
    if (!A->n) return PVAC_OK;
    hipError_t e = hipSuccess;
    if (!c->check_buf) e = hipMalloc(&c->check_buf, 32);
    if (e == hipSuccess) e = hipMemsetAsync(c->check_buf, 0, 32, c->stream);
    if (e == hipSuccess) e = launch_check_sizes(*A, *B, *C, c->check_buf, c->stream);
    unsigned int mx[4] = {0, 0, 0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(mx, c->check_buf, sizeof mx, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "check_mul_gsum (sizes)");
    unsigned long long* cnt = (unsigned long long*)(c->check_buf + 4);
    // layer tables beyond one workgroup's LDS (chain depth 9 on): per-workgroup slabs in global memory
    const uint64_t gs = check_gsum_scratch_bytes(c->prm.B, mx, A->n, c->num_cus);
    if (gs) {
        const int rc = ensure_dev(c, c->check_scratch, c->check_scratch_cap, (size_t)gs, "alloc gsum check scratch");
        if (rc) return rc;
    }
    e = launch_check_gsum(*A, *B, *C, nonces, c->powg, c->prm.B, mx, status, cnt, c->num_cus, gs ? c->check_scratch : nullptr,
                          c->stream);
    if (e == hipErrorInvalidValue) return fail(c, PVAC_ERANGE, "check_mul_gsum: no scratch for the layer tables");
    unsigned long long bad = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&bad, cnt, sizeof bad, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "check_mul_gsum");
    *n_bad = bad;
    return PVAC_OK;
}

// ---------------------------------------------------------------- dec_value
int pvac_hip_ctx_set_powg(pvac_hip_ctx* c, const uint64_t* powg_host, uint32_t count) {
    if (!c || !powg_host || count < c->prm.B) return fail(c, PVAC_EINVAL, "set_powg: need B (lo, hi) pairs");
    hipFree(c->powg);
    c->powg = nullptr;
    c->powg_n = 0;
    hipError_t e = hipMalloc(&c->powg, (size_t)count * 16);
    if (e == hipSuccess) e = hipMemcpy(c->powg, powg_host, (size_t)count * 16, hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(c, e, "set_powg");
    c->powg_n = count;
    return PVAC_OK;
}

int pvac_hip_dec_value(pvac_hip_ctx* c, const pvac_ct_batch* X, const uint64_t* R_base, uint64_t* out,
                       uint32_t* status) {
    if (!c || !batch_ok(X) || !out || !status || (X->n && !R_base)) return fail(c, PVAC_EINVAL, "dec_value: arguments");
    if (!c->powg) return fail(c, PVAC_EINVAL, "dec_value: powg_B not set (pvac_hip_ctx_set_powg)");
    if (!X->n) return PVAC_OK;
    int rc = ensure_pairs(c, X->n);
    if (rc) return rc;
    rc = ensure_dev(c, c->dec_roff, c->dec_roff_cap, X->n, "alloc dec offsets");
    if (rc) return rc;
    // dense per-cipher layer offsets (the batch may be capacity-padded)
    hipError_t e = hipMemcpyAsync(c->dec_roff, X->l_cnt, X->n * 8, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess) e = launch_exclusive_scan_u64(c->dec_roff, X->n, c->scan_scratch, &c->totals[0], c->stream);
    unsigned long long total = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&total, &c->totals[0], 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "dec_value (offsets)");
    const size_t need = dec_scratch_bytes(total);
    if (need > c->dec_cap) {
        hipFree(c->dec_scratch);
        c->dec_scratch = nullptr;
        c->dec_cap = 0;
        e = hipMalloc(&c->dec_scratch, need);
        if (e != hipSuccess) return hip_fail(c, e, "alloc dec scratch");
        c->dec_cap = need;
    }
    scoped_timer t(c, "dec_value");
    return hip_fail(c,
                    launch_dec_value(*X, R_base, c->powg, c->prm.B, c->dec_roff, total, c->dec_scratch, out, status,
                                     c->stream),
                    "dec_value");
}

// ---------------------------------------------------------------- synthetic / checks
int pvac_hip_gen_fresh_batch(pvac_hip_ctx* c, uint64_t seed, uint32_t epl, pvac_ct_batch* X) {
    return pvac_hip_gen_fresh_batch_at(c, seed, 0, epl, X);
}

int pvac_hip_gen_fresh_batch_at(pvac_hip_ctx* c, uint64_t seed, uint64_t first_index, uint32_t epl,
                                pvac_ct_batch* X) {
    if (!c || !batch_ok(X) || !X->layers || !X->meta || !X->w_lo || !X->w_hi) return PVAC_EINVAL;
    return hip_fail(c, launch_gen_fresh(seed, first_index, epl, c->prm.B, *X, c->stream), "gen_fresh");
}

int pvac_hip_fill_nonces(pvac_hip_ctx* c, uint64_t seed, uint64_t first_index, const pvac_ct_batch* A,
                         const pvac_ct_batch* B, const pvac_ct_batch* C, uint64_t* out) {
    if (!c || !batch_ok(A) || !batch_ok(B) || !C || !C->l_off || (A->n && !out) || A->n != B->n) return PVAC_EINVAL;
    return hip_fail(c, launch_fill_nonces(seed, first_index, *A, *B, C->l_off, out, c->stream), "fill_nonces");
}

int pvac_hip_fill_random(pvac_hip_ctx* c, uint64_t seed, uint64_t* out, size_t n) {
    if (!c || (n && !out)) return PVAC_EINVAL;
    return hip_fail(c, launch_fill_random(seed, out, n, c->stream), "fill_random");
}

uint64_t pvac_hip_bucket_count(uint64_t n) { return bucket_count_after_reserve(n); }

int pvac_hip_batch_digest(pvac_hip_ctx* c, const pvac_ct_batch* X, uint64_t* out) {
    if (!c || !batch_ok(X) || (X->n && !out)) return PVAC_EINVAL;
    return hip_fail(c, launch_batch_digest(*X, out, c->stream), "batch_digest");
}

int pvac_hip_batch_sumdigest(pvac_hip_ctx* c, const pvac_ct_batch* X, uint64_t* out) {
    if (!c || !batch_ok(X) || (X->n && !out)) return PVAC_EINVAL;
    return hip_fail(c, launch_batch_sumdigest(*X, out, c->stream), "batch_sumdigest");
}

// The used rows of a capacity-padded batch packed back to back (a plan's output keeps every pair's
// capacity): dst's counts = src's, its offsets their exclusive scans, rows (and sigma when both
// carry it) copied by k_stage_rows. totals[0], [1] = the packed layer / edge counts, so a caller
// copies exactly those rows to the host. dst's row arrays must hold the packed rows (src's
// capacity always does); the pair scratch of a pending plan is left alone.
int pvac_hip_batch_pack(pvac_hip_ctx* c, const pvac_ct_batch* src, pvac_ct_batch* dst, uint64_t* totals) {
    if (!c || !batch_ok(src) || !dst || !totals) return fail(c, PVAC_EINVAL, "batch_pack: arguments");
    const uint64_t n = src->n;
    if (n && (!dst->l_off || !dst->l_cnt || !dst->e_off || !dst->e_cnt || !dst->layers || !dst->meta || !dst->w_lo ||
              !dst->w_hi || !src->layers || !src->meta || !src->w_lo || !src->w_hi))
        return fail(c, PVAC_EINVAL, "batch_pack: null arrays");
    if (dst->sigma && (!src->sigma || dst->sigma_words != src->sigma_words))
        return fail(c, PVAC_EINVAL, "batch_pack: dst sigma needs src sigma of the same width");
    dst->n = n;
    totals[0] = totals[1] = 0;
    if (!n) return PVAC_OK;
    int rc = ensure_scan(c, n);
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(dst->l_cnt, src->l_cnt, n * 8, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dst->e_cnt, src->e_cnt, n * 8, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dst->l_off, src->l_cnt, n * 8, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dst->e_off, src->e_cnt, n * 8, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess)
        e = launch_exclusive_scan2_u64(dst->l_off, dst->e_off, n, c->scan_scratch, &c->totals[0], &c->totals[1],
                                       c->stream);
    unsigned long long tot[2] = {0, 0};
    if (e == hipSuccess) e = read_back(c, tot, c->totals, sizeof tot);
    if (e != hipSuccess) return hip_fail(c, e, "batch_pack (offsets)");
    totals[0] = tot[0];
    totals[1] = tot[1];
    return hip_fail(c, launch_stage_rows(*src, *dst, c->stream), "batch_pack (rows)");
}

// ---------------------------------------------------------------- depth chains
}  // extern "C"

namespace {

// grows a stream-ordered device array to at least `need` elements (1/8 headroom); contents are lost
template <typename T>
hipError_t grow_async(T*& p, size_t& cap, size_t need, hipStream_t st) {
    if (need <= cap && p) return hipSuccess;
    if (p) hipFreeAsync(p, st);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(need + need / 8, 64);
    hipError_t e = hipMallocAsync((void**)&p, want * sizeof(T), st);
    if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        e = hipMallocAsync((void**)&p, std::max<size_t>(need, 64) * sizeof(T), st);
        if (e == hipSuccess) cap = std::max<size_t>(need, 64);
    } else if (e == hipSuccess) {
        cap = want;
    }
    return e;
}

// intermediate chain steps as dense images (A/B builds: -DPVAC_CHAIN_IMAGE=0 keeps records throughout)
#ifndef PVAC_CHAIN_IMAGE
#define PVAC_CHAIN_IMAGE 1
#endif

struct chain_range {
    uint64_t end = 0;               // last input (exclusive) of this device range
    std::atomic<uint64_t> next{0};  // next chunk's first input
};

struct chain_shared {
    const pvac_ct_batch* X = nullptr;
    const pvac_chain_opts* o = nullptr;
    uint64_t chunk = 0;
    int x_dev = 0;                  // the device X (and the digest / count outputs) live on
    chain_range* ranges = nullptr;
    std::atomic<int> stop{0};
    std::mutex mu;
    int rc = PVAC_OK;
    std::string err;
    void failed(int code, const std::string& msg) {
        std::lock_guard<std::mutex> g(mu);
        if (rc == PVAC_OK) {
            rc = code;
            err = msg;
        }
        stop.store(1);
    }
};

struct chain_wstats {
    uint64_t gsum_pairs = 0, gsum_failed = 0, chunks = 0;
};

pvac_ct_batch chain_view(const pvac_ct_batch& X, uint64_t c0, uint64_t k) {
    pvac_ct_batch v = X;
    v.n = k;
    v.l_off = X.l_off + c0;
    v.l_cnt = X.l_cnt + c0;
    v.e_off = X.e_off + c0;
    v.e_cnt = X.e_cnt + c0;
    v.sigma = nullptr;
    v.sigma_words = 0;
    return v;
}

// the inputs of one chunk copied into the worker's own buffers (compact CSR): counts by peer
// copy, offsets by an exclusive scan, rows by k_stage_rows (peer reads when X lives elsewhere)
bool stage_chunk(pvac_hip_ctx* k, chain_shared* sh, const pvac_ct_batch& src, pvac_ct_batch& out, chain_set& S) {
    const uint64_t kk = src.n;
    auto hipchk = [&](hipError_t e, const char* where) {
        if (e == hipSuccess) return true;
        sh->failed(e == hipErrorOutOfMemory ? PVAC_ENOMEM : PVAC_EDEVICE,
                   std::string("ct_mul_chain: stage ") + where + ": " + hipGetErrorString(e));
        return false;
    };
    if (kk > S.n_cap) {
        size_t c1 = S.n_cap, c2 = S.n_cap, c3 = S.n_cap, c4 = S.n_cap;
        if (!hipchk(grow_async(S.l_off, c1, kk, k->stream), "alloc") || !hipchk(grow_async(S.l_cnt, c2, kk, k->stream), "alloc") ||
            !hipchk(grow_async(S.e_off, c3, kk, k->stream), "alloc") || !hipchk(grow_async(S.e_cnt, c4, kk, k->stream), "alloc"))
            return false;
        S.n_cap = std::min(std::min(c1, c2), std::min(c3, c4));
    }
    if (ensure_pairs(k, kk)) {
        sh->failed(PVAC_ENOMEM, "ct_mul_chain: stage scratch: " + k->err);
        return false;
    }
    const int sd = sh->x_dev, dd = k->device;
    if (!hipchk(hipMemcpyPeerAsync(S.l_cnt, dd, src.l_cnt, sd, kk * 8, k->stream), "counts") ||
        !hipchk(hipMemcpyPeerAsync(S.e_cnt, dd, src.e_cnt, sd, kk * 8, k->stream), "counts") ||
        !hipchk(hipMemcpyAsync(S.l_off, S.l_cnt, kk * 8, hipMemcpyDeviceToDevice, k->stream), "offsets") ||
        !hipchk(hipMemcpyAsync(S.e_off, S.e_cnt, kk * 8, hipMemcpyDeviceToDevice, k->stream), "offsets") ||
        !hipchk(launch_exclusive_scan_u64(S.l_off, kk, k->scan_scratch, &k->totals[0], k->stream), "scan") ||
        !hipchk(launch_exclusive_scan_u64(S.e_off, kk, k->scan_scratch, &k->totals[1], k->stream), "scan"))
        return false;
    unsigned long long tot[2] = {0, 0};
    if (!hipchk(hipMemcpyAsync(tot, k->totals, sizeof tot, hipMemcpyDeviceToHost, k->stream), "totals") ||
        !hipchk(hipStreamSynchronize(k->stream), "totals"))
        return false;
    if (tot[0] > S.l_cap && !hipchk(grow_async(S.layers, S.l_cap, tot[0], k->stream), "alloc layers")) return false;
    if (tot[1] > S.e_cap) {
        size_t c1 = S.e_cap, c2 = S.e_cap, c3 = S.e_cap;
        if (!hipchk(grow_async(S.meta, c1, tot[1], k->stream), "alloc edges") ||
            !hipchk(grow_async(S.w_lo, c2, tot[1], k->stream), "alloc edges") ||
            !hipchk(grow_async(S.w_hi, c3, tot[1], k->stream), "alloc edges"))
            return false;
        S.e_cap = std::min(c1, std::min(c2, c3));
    }
    out = pvac_ct_batch{};
    out.n = kk;
    out.l_off = S.l_off;
    out.l_cnt = S.l_cnt;
    out.layers = S.layers;
    out.e_off = S.e_off;
    out.e_cnt = S.e_cnt;
    out.meta = S.meta;
    out.w_lo = S.w_lo;
    out.w_hi = S.w_hi;
    return hipchk(launch_stage_rows(src, out, k->stream), "rows");
}

// the final step's sigmas (PVAC_MUL_WITH_SIGMA): salts from salts_at (or splitmix), then sigma_from_H
// per edge over the finished hash-order output; a pair the exec put in the canonical order
// (guard_budget / ORDER_CANONICAL) makes the step run once more with the salts mapped (exec's salt
// positions), as pvac_hip_ct_mul_exec does for a batch
bool chain_final_sigma(pvac_hip_ctx* k, chain_shared* sh, uint32_t d, uint64_t c0, pvac_hip_plan& plan,
                       const pvac_ct_batch& A, const pvac_ct_batch& Xv, pvac_ct_batch& C, chain_set& S,
                       uint32_t mflags) {
    const pvac_chain_opts& o = *sh->o;
    auto hipchk = [&](hipError_t e, const char* where) {
        if (e == hipSuccess) return true;
        sh->failed(e == hipErrorOutOfMemory ? PVAC_ENOMEM : PVAC_EDEVICE,
                   std::string("ct_mul_chain: sigma ") + where + ": " + hipGetErrorString(e));
        return false;
    };
    const uint64_t slots = std::max<uint64_t>(plan.total_edge_slots, 1);
    const uint32_t sw = k->prm.m_bits / 64;
    if (slots > S.s_cap) {
        if (S.sigma) hipFreeAsync(S.sigma, k->stream);
        S.sigma = nullptr;
        S.s_cap = 0;
        if (!hipchk(hipMallocAsync((void**)&S.sigma, slots * sw * 8, k->stream), "alloc (1 KiB per edge: a smaller chunk?)"))
            return false;
        S.s_cap = slots;
    }
    if (!hipchk(grow_async(k->chain_salts, k->chain_salt_cap, slots, k->stream), "alloc salts")) return false;
    if (o.salts_at) {
        if (o.salts_at(o.user, d, c0, &A, &Xv, &C, k->chain_salts, plan.total_edge_slots, (void*)k->stream) != 0) {
            sh->failed(PVAC_EINVAL, "ct_mul_chain: salts_at callback failed");
            return false;
        }
    } else if (!hipchk(launch_fill_random(o.nonce_seed ^ 0x5A175A175A175A17ull ^ (97ull * c0 + d), k->chain_salts, slots,
                                          k->stream),
                       "fill salts")) {
        return false;
    }
    C.sigma = S.sigma;
    C.sigma_words = sw;
    bool hash_order = (mflags & PVAC_MUL_ORDER_CANONICAL) == 0;
    if (hash_order) {
        std::vector<uint32_t> stv(C.n);
        if (!hipchk(hipMemcpyAsync(stv.data(), k->pair_status, C.n * 4, hipMemcpyDeviceToHost, k->stream), "status") ||
            !hipchk(hipStreamSynchronize(k->stream), "status"))
            return false;
        for (uint32_t v : stv) hash_order &= v != 1u;
    }
    if (hash_order) return hipchk(launch_sigma(k->H, k->prm, C, k->chain_salts, nullptr, k->num_cus, k->stream), "launch");
    if (pvac_hip_ct_mul_exec(k, &plan, &A, &Xv, k->chain_nonces, k->chain_salts, &C, mflags | PVAC_MUL_WITH_SIGMA)) {
        sh->failed(PVAC_EDEVICE, "ct_mul_chain: sigma exec: " + k->err);
        return false;
    }
    return true;
}

// one worker: chunks of its device range in input order from the range's counter, depth steps of
// plan + exec each on this context's stream, the final c_depth to the digests / on_chunk
void chain_worker(pvac_hip_ctx* k, chain_shared* sh, chain_range* rg, bool stage, chain_wstats* ws) {
    if (hipSetDevice(k->device) != hipSuccess) {
        sh->failed(PVAC_EDEVICE, "ct_mul_chain: hipSetDevice");
        return;
    }
    const pvac_chain_opts& o = *sh->o;
    const pvac_ct_batch& X = *sh->X;
    const uint32_t mflags = o.flags & PVAC_MUL_ORDER_CANONICAL;
    const bool check = (o.flags & PVAC_CHAIN_CHECK_GSUM) != 0;
    const bool sigma = (o.flags & PVAC_MUL_WITH_SIGMA) != 0;
    const bool remote = k->device != sh->x_dev;
    // intermediate steps hand their C to the next step as dense images (mul_large_args::C_img) unless
    // a caller hook or the gsum check reads every step's records; an image A never meets the fresh
    // kernel, whose pairs have at most kFreshEdgesMax < 2B edges a side
    const bool use_img = PVAC_CHAIN_IMAGE && !check && !o.after_step && 2u * k->prm.B > kFreshEdgesMax;
    auto hipchk = [&](hipError_t e, const char* where) {
        if (e == hipSuccess) return true;
        sh->failed(e == hipErrorOutOfMemory ? PVAC_ENOMEM : PVAC_EDEVICE,
                   std::string("ct_mul_chain: ") + where + ": " + hipGetErrorString(e));
        return false;
    };
    auto rcchk = [&](int rc, const char* where) {
        if (rc == PVAC_OK) return true;
        sh->failed(rc, std::string("ct_mul_chain: ") + where + ": " + k->err);
        return false;
    };
    for (;;) {
        if (sh->stop.load()) return;
        const uint64_t c0 = rg->next.fetch_add(sh->chunk);
        if (c0 >= rg->end) return;
        const uint64_t kk = std::min<uint64_t>(sh->chunk, rg->end - c0);
        pvac_ct_batch Xv = chain_view(X, c0, kk);
        if ((stage || remote) && !stage_chunk(k, sh, chain_view(X, c0, kk), Xv, k->chain_stage)) return;
        const pvac_ct_batch X0 = Xv;   // the chunk's inputs: c_0, and the operand of steps without one
        pvac_ct_batch A = Xv;
        int cur = 0;
        uint32_t* a_img = nullptr;   // the previous step's image flags (A's)
        struct img_reset {
            pvac_hip_ctx* k;
            ~img_reset() { k->img_in = k->img_out = nullptr; }
        } img_guard{k};
        for (uint32_t d = 0; d < o.depth; ++d) {
            if (sh->stop.load()) return;
            // this step's operand: operands[d] (the reference's loop multiplies by a fresh enc_value per
            // step, tests/test_main.cpp:291-292) or the chunk's inputs
            Xv = X0;
            if (d < o.n_operands) {
                Xv = chain_view(o.operands[d], c0, kk);
                if ((stage || remote) && !stage_chunk(k, sh, chain_view(o.operands[d], c0, kk), Xv, k->chain_stage_op))
                    return;
            }
            chain_set& S = k->chain_bufs[cur];
            if (kk > S.n_cap) {
                size_t c1 = S.n_cap, c2 = S.n_cap, c3 = S.n_cap, c4 = S.n_cap;
                if (!hipchk(grow_async(S.l_off, c1, kk, k->stream), "alloc offsets") ||
                    !hipchk(grow_async(S.l_cnt, c2, kk, k->stream), "alloc counts") ||
                    !hipchk(grow_async(S.e_off, c3, kk, k->stream), "alloc offsets") ||
                    !hipchk(grow_async(S.e_cnt, c4, kk, k->stream), "alloc counts"))
                    return;
                S.n_cap = std::min(std::min(c1, c2), std::min(c3, c4));
            }
            pvac_ct_batch C{};
            C.n = kk;
            C.l_off = S.l_off;
            C.l_cnt = S.l_cnt;
            C.e_off = S.e_off;
            C.e_cnt = S.e_cnt;
            pvac_hip_plan plan{};
            if (!rcchk(pvac_hip_ct_mul_plan(k, &A, &Xv, &C, &plan), "plan")) return;
            // an output array that does not fit first takes this worker's scratch arena back (the
            // general path reallocates it within what is left, splitting its sub-batch if needed)
            auto grow_out = [&](auto*& p, size_t& cap, size_t need, const char* what) -> bool {
                hipError_t e = grow_async(p, cap, need, k->stream);
                if (e == hipErrorOutOfMemory && k->arena) {
                    (void)hipGetLastError();
                    e = hipStreamSynchronize(k->stream);
                    hipFree(k->arena);
                    k->arena = nullptr;
                    k->arena_words = 0;
                    if (e == hipSuccess) e = grow_async(p, cap, need, k->stream);
                }
                return hipchk(e, what);
            };
            if (plan.total_layer_slots > S.l_cap && !grow_out(S.layers, S.l_cap, plan.total_layer_slots, "alloc layers"))
                return;
            if (plan.total_edge_slots > S.e_cap) {
                size_t c1 = S.e_cap, c2 = S.e_cap, c3 = S.e_cap;
                if (!grow_out(S.meta, c1, plan.total_edge_slots, "alloc edges") ||
                    !grow_out(S.w_lo, c2, plan.total_edge_slots, "alloc edges") ||
                    !grow_out(S.w_hi, c3, plan.total_edge_slots, "alloc edges"))
                    return;
                S.e_cap = std::min(c1, std::min(c2, c3));
            }
            const size_t nw = 2 * std::max<uint64_t>(plan.total_layer_slots, 1);
            if (!hipchk(grow_async(k->chain_nonces, k->chain_nonce_cap, nw, k->stream), "alloc nonces")) return;
            C.layers = S.layers;
            C.meta = S.meta;
            C.w_lo = S.w_lo;
            C.w_hi = S.w_hi;
            if (o.nonces_at) {
                if (o.nonces_at(o.user, d, c0, &A, &Xv, &C, k->chain_nonces, nw, (void*)k->stream) != 0) {
                    sh->failed(PVAC_EINVAL, "ct_mul_chain: nonces_at callback failed");
                    return;
                }
            } else if (o.fill_nonces) {
                if (o.fill_nonces(o.user, d, c0, nw, k->chain_nonces, (void*)k->stream) != 0) {
                    sh->failed(PVAC_EINVAL, "ct_mul_chain: fill_nonces callback failed");
                    return;
                }
            } else if (!hipchk(launch_fill_random(o.nonce_seed + 97ull * c0 + d, k->chain_nonces, nw, k->stream),
                               "fill nonces")) {
                return;
            }
            uint32_t* c_img = nullptr;
            if (use_img && d + 1 < o.depth) {
                if (kk > S.img_cap && !hipchk(grow_async(S.img, S.img_cap, kk, k->stream), "alloc image flags")) return;
                if (!hipchk(hipMemsetAsync(S.img, 0, kk * 4, k->stream), "image flags")) return;
                c_img = S.img;
            }
            k->img_in = a_img;
            k->img_out = c_img;
            k->img_count = k->chain_stats + 2 * PVAC_CHAIN_MAX_DEPTH;
            if (!rcchk(pvac_hip_ct_mul_exec(k, &plan, &A, &Xv, k->chain_nonces, nullptr, &C, mflags), "exec")) return;
            k->img_out = nullptr;   // the final-step sigma re-run below reads A (img_in), writes records
            if (!hipchk(launch_chain_stats(A, Xv, C, k->chain_stats + 2 * d, k->stream), "stats")) return;
            if (check) {
                uint64_t bad = 0;
                if (!rcchk(pvac_hip_check_mul_gsum(k, &A, &Xv, &C, k->chain_nonces, nullptr, &bad), "gsum check"))
                    return;
                ws->gsum_pairs += kk;
                ws->gsum_failed += bad;
            }
            if (o.after_step && o.after_step(o.user, d, c0, &A, &Xv, &C, nullptr, 0, (void*)k->stream) != 0) {
                sh->failed(PVAC_EINVAL, "ct_mul_chain: after_step callback failed");
                return;
            }
            if (sigma && d + 1 == o.depth && !chain_final_sigma(k, sh, d, c0, plan, A, Xv, C, S, mflags)) return;
            k->img_in = nullptr;
            a_img = c_img;
            A = C;
            cur ^= 1;
        }
        // digests / counts land in the caller's arrays on X's device (through the worker's own
        // buffer and a peer copy when this worker runs on another device)
        auto out_words = [&](uint64_t n_out, uint64_t* dst, int kind) {   // 0 counts, 1 FNV, 2 sum digests
            if (n_out <= c0 || !dst) return true;
            const uint64_t m = std::min<uint64_t>(kk, n_out - c0);
            pvac_ct_batch H = A;
            H.n = m;
            auto put = [&](uint64_t* to) {
                if (kind == 1) return hipchk(launch_batch_digest(H, to, k->stream), "digest");
                if (kind == 2) return hipchk(launch_batch_sumdigest(H, to, k->stream), "sum digest");
                return hipchk(hipMemcpyAsync(to, A.e_cnt, m * 8, hipMemcpyDeviceToDevice, k->stream), "counts");
            };
            if (!remote) return put(dst + c0);
            if (!hipchk(grow_async(k->chain_out, k->chain_out_cap, m, k->stream), "alloc outputs") || !put(k->chain_out))
                return false;
            return hipchk(hipMemcpyPeerAsync(dst + c0, sh->x_dev, k->chain_out, k->device, m * 8, k->stream), "peer copy");
        };
        if (!out_words(o.digest_n, o.digest_out, 1) || !out_words(o.count_n, o.count_out, 0) ||
            !out_words(o.sumdigest_n, o.sumdigest_out, 2))
            return;
        if (o.on_chunk && o.on_chunk(o.user, c0, &A, (void*)k->stream) != 0) {
            sh->failed(PVAC_EINVAL, "ct_mul_chain: on_chunk callback failed");
            return;
        }
        ++ws->chunks;
    }
}

}  // namespace

extern "C" {

int pvac_hip_memcpy(void* dst, const void* src, size_t bytes, void* stream) {
    if (!bytes) return PVAC_OK;
    if (!dst || !src) return PVAC_EINVAL;
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    return e == hipSuccess ? PVAC_OK : PVAC_EDEVICE;
}

int pvac_hip_chain_partition(uint64_t n, uint64_t chunk, uint32_t parts, uint64_t* first) {
    if (!first || parts == 0 || parts > PVAC_CHAIN_MAX_DEVICES) return PVAC_EINVAL;
    if (!chunk) chunk = 1024;
    const uint64_t nch = (n + chunk - 1) / chunk;   // whole chunks, dealt as evenly as possible
    for (uint32_t j = 0; j <= parts; ++j) first[j] = std::min<uint64_t>(n, (nch * j / parts) * chunk);
    return PVAC_OK;
}

int pvac_hip_ct_mul_chain(pvac_hip_ctx* c, const pvac_ct_batch* X, const pvac_chain_opts* o, pvac_chain_stats* st) {
    if (!c || !o || !st || !batch_ok(X)) return fail(c, PVAC_EINVAL, "ct_mul_chain: bad arguments");
    if (o->depth < 1 || o->depth > PVAC_CHAIN_MAX_DEPTH) return fail(c, PVAC_EINVAL, "ct_mul_chain: depth");
    if (o->flags & ~(PVAC_MUL_ORDER_CANONICAL | PVAC_CHAIN_CHECK_GSUM | PVAC_MUL_WITH_SIGMA | PVAC_CHAIN_STAGE_INPUTS |
                     PVAC_CHAIN_IMG_BATCH2))
        return fail(c, PVAC_EINVAL, "ct_mul_chain: flags");
    if (o->n_operands > o->depth || (o->n_operands && !o->operands))
        return fail(c, PVAC_EINVAL, "ct_mul_chain: operands");
    for (uint32_t d = 0; d < o->n_operands; ++d) {
        const pvac_ct_batch& Y = o->operands[d];
        if (!batch_ok(&Y) || Y.n != X->n || (Y.n && (!Y.layers || !Y.meta || !Y.w_lo || !Y.w_hi)))
            return fail(c, PVAC_EINVAL, "ct_mul_chain: operand " + std::to_string(d) + " is not a batch of |X| ciphers");
    }
    if ((o->flags & PVAC_CHAIN_CHECK_GSUM) && !c->powg)
        return fail(c, PVAC_EINVAL, "ct_mul_chain: CHECK_GSUM needs pvac_hip_ctx_set_powg");
    if ((o->flags & PVAC_MUL_WITH_SIGMA) && !c->H.ready)
        return fail(c, PVAC_EINVAL, "ct_mul_chain: WITH_SIGMA needs H (pvac_hip_ctx_set_H / gen_H)");
    if (o->n_devices > PVAC_CHAIN_MAX_DEVICES || (o->n_devices && !o->devices))
        return fail(c, PVAC_EINVAL, "ct_mul_chain: devices");
    if (X->n && (!X->layers || !X->meta || !X->w_lo || !X->w_hi)) return fail(c, PVAC_EINVAL, "ct_mul_chain: input arrays");
    std::memset(st, 0, sizeof *st);
    const auto t0 = std::chrono::steady_clock::now();
    if (!X->n) return PVAC_OK;
    const uint32_t S = o->streams ? std::min<uint32_t>(o->streams, 64) : 4u;
    const uint64_t chunk = o->chunk ? o->chunk : 1024;
    const uint32_t D = o->n_devices ? o->n_devices : 1u;
    std::vector<int> devs(D, c->device);
    for (uint32_t j = 0; j < o->n_devices; ++j) devs[j] = o->devices[j];
    // inputs already enqueued on the caller's stream must be complete before other streams read them
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "ct_mul_chain (caller stream)");
    // a layout change (streams, chunk, the device list) first returns everything the workers grew
    // (output batches, nonce / salt / result words, image scratch, scratch arenas), so the HBM shares
    // below are taken over the device's memory, not over what the previous layout's workers left free
    std::vector<int64_t> layout{(int64_t)S, (int64_t)chunk, (int64_t)D};
    layout.insert(layout.end(), devs.begin(), devs.end());
    if (!c->chain_kids.empty() && layout != c->chain_layout) {
        for (pvac_hip_ctx* k : c->chain_kids) {
            hipSetDevice(k->device);
            e = release_chain_worker(k);
            if (e != hipSuccess) {
                hipSetDevice(c->device);
                return hip_fail(c, e, "ct_mul_chain: worker release");
            }
        }
        hipSetDevice(c->device);
    }
    c->chain_layout = layout;
    // worker contexts: [range j * S + w] on devs[j]; a layout change rebuilds the ones that differ
    if (c->chain_kids.size() > (size_t)D * S) {
        for (size_t w = (size_t)D * S; w < c->chain_kids.size(); ++w) pvac_hip_ctx_destroy(c->chain_kids[w]);
        c->chain_kids.resize((size_t)D * S);
    }
    for (uint32_t j = 0; j < D; ++j) {
        // each worker's general-path scratch: its share of half the HBM free now on its device (the
        // other half holds the workers' ping-pong outputs and the caller's data)
        size_t free_b = 0, total_b = 0;
        if (hipSetDevice(devs[j]) != hipSuccess) {
            hipSetDevice(c->device);
            return fail(c, PVAC_EDEVICE, "ct_mul_chain: device " + std::to_string(devs[j]));
        }
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 8ull << 30;
        const uint32_t same = (uint32_t)std::count(devs.begin(), devs.end(), devs[j]);
        const uint64_t cap_words = std::max<uint64_t>((uint64_t)(free_b / 2) / ((uint64_t)S * same) / 4, 1ull << 24);
        if (devs[j] != c->device) {   // peer reads of X / peer writes of the outputs
            const hipError_t pe = hipDeviceEnablePeerAccess(c->device, 0);
            if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) {
                hipSetDevice(c->device);
                return hip_fail(c, pe, "ct_mul_chain: peer access");
            }
            (void)hipGetLastError();
        }
        for (uint32_t w = 0; w < S; ++w) {
            const size_t slot = (size_t)j * S + w;
            if (slot < c->chain_kids.size() && c->chain_kids[slot]->device != devs[j]) {
                pvac_hip_ctx_destroy(c->chain_kids[slot]);
                c->chain_kids[slot] = nullptr;
            }
            if (slot >= c->chain_kids.size()) c->chain_kids.push_back(nullptr);
            pvac_hip_ctx*& k = c->chain_kids[slot];
            if (!k) {
                const int rc = pvac_hip_ctx_create(devs[j], &c->prm, &k);
                if (rc) {
                    hipSetDevice(c->device);
                    return fail(c, rc, "ct_mul_chain: worker context");
                }
                e = hipMalloc(&k->chain_stats, (2 * PVAC_CHAIN_MAX_DEPTH + 1) * sizeof(unsigned long long));
                if (e != hipSuccess) {
                    hipSetDevice(c->device);
                    return hip_fail(c, e, "ct_mul_chain: worker statistics");
                }
            }
            k->arena_cap_words = cap_words;
            k->prm = c->prm;
            k->spin_us = 200;
            k->img_grid_y = (o->flags & PVAC_CHAIN_IMG_BATCH2) ? 2u : 65535u;
            if (c->powg && (k->powg_n != c->powg_n || !k->powg)) {
                hipFree(k->powg);
                k->powg = nullptr;
                e = hipMalloc(&k->powg, (size_t)c->powg_n * 16);
                if (e != hipSuccess) {
                    hipSetDevice(c->device);
                    return hip_fail(c, e, "ct_mul_chain: worker powg");
                }
                k->powg_n = c->powg_n;
            }
            e = hipSuccess;
            if (c->powg) e = hipMemcpyPeer(k->powg, k->device, c->powg, c->device, (size_t)c->powg_n * 16);
            if (e == hipSuccess && (o->flags & PVAC_MUL_WITH_SIGMA) && (!k->H.ready || k->H_from != c->H_gen)) {
                e = sigma_tables_clone(k->H, c->H, k->device, c->device, k->stream);
                k->H_from = c->H_gen;
            }
            if (e == hipSuccess) e = hipMemsetAsync(k->chain_stats, 0, (2 * PVAC_CHAIN_MAX_DEPTH + 1) * 8, k->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(k->stream);
            if (e != hipSuccess) {
                hipSetDevice(c->device);
                return hip_fail(c, e, "ct_mul_chain: worker setup");
            }
        }
    }
    hipSetDevice(c->device);
    std::vector<uint64_t> first(D + 1);
    pvac_hip_chain_partition(X->n, chunk, D, first.data());
    std::vector<chain_range> ranges(D);
    for (uint32_t j = 0; j < D; ++j) {
        ranges[j].next.store(first[j]);
        ranges[j].end = first[j + 1];
    }
    chain_shared sh;
    sh.X = X;
    sh.o = o;
    sh.chunk = chunk;
    sh.x_dev = c->device;
    sh.ranges = ranges.data();
    const size_t nk = (size_t)D * S;
    std::vector<chain_wstats> ws(nk);
    std::vector<uint64_t> redo0(nk);
    for (size_t w = 0; w < nk; ++w) redo0[w] = c->chain_kids[w]->redo_total;
    std::vector<std::thread> th;
    th.reserve(nk);
    for (uint32_t j = 0; j < D; ++j)
        for (uint32_t w = 0; w < S; ++w)
            th.emplace_back(chain_worker, c->chain_kids[(size_t)j * S + w], &sh, &ranges[j],
                            j > 0 && (o->flags & PVAC_CHAIN_STAGE_INPUTS) != 0, &ws[(size_t)j * S + w]);
    for (std::thread& t : th) t.join();
    for (size_t w = 0; w < nk; ++w) {
        pvac_hip_ctx* k = c->chain_kids[w];
        hipSetDevice(k->device);
        e = hipStreamSynchronize(k->stream);
        if (e != hipSuccess && sh.rc == PVAC_OK) sh.failed(PVAC_EDEVICE, std::string("ct_mul_chain: ") + hipGetErrorString(e));
        unsigned long long v[2 * PVAC_CHAIN_MAX_DEPTH + 1];
        if (hipMemcpy(v, k->chain_stats, sizeof v, hipMemcpyDeviceToHost) == hipSuccess) {
            for (uint32_t d = 0; d < o->depth; ++d) {
                st->edges[d] += v[2 * d];
                st->products[d] += v[2 * d + 1];
            }
            st->image_steps += v[2 * PVAC_CHAIN_MAX_DEPTH];
        }
        st->gsum_pairs += ws[w].gsum_pairs;
        st->gsum_failed += ws[w].gsum_failed;
        st->chunks += ws[w].chunks;
        st->redo += k->redo_total - redo0[w];
    }
    hipSetDevice(c->device);
    st->pair_steps = X->n * o->depth;
    st->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (sh.rc != PVAC_OK) return fail(c, sh.rc, sh.err);
    return PVAC_OK;
}

}  // extern "C"

