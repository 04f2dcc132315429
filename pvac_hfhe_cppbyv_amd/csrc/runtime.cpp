// runtime.cpp — host side of libpvac_hip.so: the extern "C" ABI of include/pvac_hip.h.
//
// Owns per-context device state (stream, libstdc++ bucket-count table, plan scratch,
// sparse H, timing events) and sequences the kernels. Never throws across the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "sigma.hpp"

using namespace pvhip;

namespace {

constexpr uint32_t kNbTableLen = 4097;      // bucket counts for |A.E||B.E| in [0, 4096]
constexpr uint32_t kSmallProdMax = 4096;
constexpr uint32_t kSmallKeysMax = 1536;

struct timer_rec {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    double ms = 0;
    uint64_t launches = 0;
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
    uint8_t* pair_class = nullptr;
    uint32_t* pair_status = nullptr;
    size_t pair_cap = 0;
    uint64_t* scan_scratch = nullptr;
    size_t scan_cap = 0;
    plan_stats* stats = nullptr;
    unsigned long long* totals = nullptr;   // [2]
    sigma_tables H;
    // timing
    bool timing = false;
    std::map<std::string, timer_rec> timers;
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
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a, c->stream);
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
            hipEventDestroy(ev.first);
            hipEventDestroy(ev.second);
        }
        kv.second.pending.clear();
    }
}

int ensure_pairs(pvac_hip_ctx* c, size_t n) {
    if (n > c->pair_cap) {
        hipFree(c->pair_class);
        hipFree(c->pair_status);
        c->pair_class = nullptr;
        c->pair_status = nullptr;
        size_t cap = std::max<size_t>(n, 1024);
        hipError_t e = hipMalloc(&c->pair_class, cap);
        if (e == hipSuccess) e = hipMalloc(&c->pair_status, cap * 4);
        if (e != hipSuccess) { c->pair_cap = 0; return hip_fail(c, e, "alloc pair scratch"); }
        c->pair_cap = cap;
    }
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
    for (uint32_t n = 0; n < kNbTableLen; ++n) nb[n] = (uint32_t)bucket_count_after_reserve(n);
    e = hipMalloc(&c->nb_table, nb.size() * 4);
    if (e == hipSuccess) e = hipMemcpy(c->nb_table, nb.data(), nb.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&c->stats, sizeof(plan_stats));
    if (e == hipSuccess) e = hipMalloc(&c->totals, 2 * sizeof(unsigned long long));
    if (e != hipSuccess) { pvac_hip_ctx_destroy(c); return PVAC_ENOMEM; }
    *out = c;
    return PVAC_OK;
}

int pvac_hip_ctx_destroy(pvac_hip_ctx* c) {
    if (!c) return PVAC_OK;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    flush_timers(c);
    hipFree(c->nb_table);
    hipFree(c->pair_class);
    hipFree(c->pair_status);
    hipFree(c->scan_scratch);
    hipFree(c->stats);
    hipFree(c->totals);
    sigma_tables_free(c->H);
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    delete c;
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

const char* pvac_hip_last_error(pvac_hip_ctx* c) { return c ? c->err.c_str() : "null context"; }

int pvac_hip_timing_enable(pvac_hip_ctx* c, int on) {
    if (!c) return PVAC_EINVAL;
    c->timing = on != 0;
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
    if (op < PVAC_FP_ADD || op > PVAC_FP_SCALE) return fail(c, PVAC_EINVAL, "fp_binop: bad op");
    if (n && (!a_lo || !a_hi || !c_lo || !c_hi)) return fail(c, PVAC_EINVAL, "fp_binop: null array");
    if (n && op != PVAC_FP_NEG && (!b_lo || !b_hi)) return fail(c, PVAC_EINVAL, "fp_binop: null b");
    scoped_timer t(c, "fp_binop");
    return hip_fail(c, launch_fp_binop(op, a_lo, a_hi, b_lo, b_hi, c_lo, c_hi, n, c->stream), "fp_binop");
}

// ---------------------------------------------------------------- ct_mul
int pvac_hip_ct_mul_plan(pvac_hip_ctx* c, const pvac_ct_batch* A, const pvac_ct_batch* B, pvac_ct_batch* C,
                         pvac_hip_plan* plan) {
    if (!c || !plan || !batch_ok(A) || !batch_ok(B) || !C || !C->l_off || !C->e_off)
        return fail(c, PVAC_EINVAL, "ct_mul_plan: bad arguments");
    if (A->n != B->n) return fail(c, PVAC_EINVAL, "ct_mul_plan: |A| != |B|");
    std::memset(plan, 0, sizeof *plan);
    plan->kind = 1;
    plan->n_pairs = A->n;
    C->n = A->n;
    if (!A->n) return PVAC_OK;
    int rc = ensure_pairs(c, A->n);
    if (rc) return rc;
    hipError_t e = hipMemsetAsync(c->stats, 0, sizeof(plan_stats), c->stream);
    if (e == hipSuccess)
        e = launch_plan_mul(*A, *B, *C, c->pair_class, c->stats, c->nb_table, kNbTableLen, c->prm.B, kSmallKeysMax,
                            kSmallProdMax, c->stream);
    if (e == hipSuccess) e = launch_exclusive_scan_u64(C->l_off, A->n, c->scan_scratch, &c->totals[0], c->stream);
    if (e == hipSuccess) e = launch_exclusive_scan_u64(C->e_off, A->n, c->scan_scratch, &c->totals[1], c->stream);
    plan_stats st{};
    unsigned long long tot[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(&st, c->stats, sizeof st, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(tot, c->totals, sizeof tot, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "ct_mul_plan");
    plan->total_layer_slots = tot[0];
    plan->total_edge_slots = tot[1];
    plan->n_small = st.n_small;
    plan->n_large = st.n_large;
    plan->max_keys = st.max_keys;
    plan->max_prod = st.max_prod;
    plan->max_na = st.max_na;
    plan->max_nb = st.max_nb;
    plan->max_buckets = st.max_buckets;
    plan->max_layers = st.max_layers;
    return PVAC_OK;
}

int pvac_hip_ct_mul_exec(pvac_hip_ctx* c, const pvac_hip_plan* plan, const pvac_ct_batch* A, const pvac_ct_batch* B,
                         const uint64_t* nonces, const uint64_t* salts, pvac_ct_batch* C, uint32_t flags) {
    if (!c || !plan || plan->kind != 1 || !batch_ok(A) || !batch_ok(B) || !batch_ok(C))
        return fail(c, PVAC_EINVAL, "ct_mul_exec: bad arguments");
    if (A->n != plan->n_pairs || B->n != plan->n_pairs) return fail(c, PVAC_EINVAL, "ct_mul_exec: plan mismatch");
    if (!A->n) return PVAC_OK;
    if (!nonces) return fail(c, PVAC_EINVAL, "ct_mul_exec: nonces required");
    if (!C->layers || !C->meta || !C->w_lo || !C->w_hi) return fail(c, PVAC_EINVAL, "ct_mul_exec: output arrays");
    if (plan->n_large)
        return fail(c, PVAC_ENOSYS, "ct_mul_exec: pairs beyond the fresh-shape kernel need the layer-dense path");
    const bool with_sigma = (flags & PVAC_MUL_WITH_SIGMA) != 0;
    if (with_sigma && (!salts || !C->sigma || !c->H.ready))
        return fail(c, PVAC_EINVAL, "ct_mul_exec: WITH_SIGMA needs salts, C->sigma and H");
    if (plan->n_small) {
        mul_small_args a{};
        a.A = *A; a.B = *B; a.C = *C;
        a.nonces = nonces;
        a.salt_pos = nullptr;
        a.pair_class = c->pair_class;
        a.pair_status = c->pair_status;
        a.nb_table = c->nb_table;
        a.canon_tag = c->prm.canon_tag;
        a.edge_budget = c->prm.edge_budget;
        a.Bm = c->prm.B;
        a.flags = flags;
        a.ks_max = plan->max_keys;
        a.prod_max = plan->max_prod;
        a.na_max = plan->max_na;
        a.nb_max = plan->max_nb;
        a.buckets_max = plan->max_buckets;
        a.layers_max = plan->max_layers;
        int blocks = 0;
        scoped_timer t(c, "ct_mul_small");
        hipError_t e = launch_ct_mul_small(a, c->num_cus, c->stream, &blocks);
        if (e != hipSuccess) return hip_fail(c, e, "ct_mul_small");
    }
    if (with_sigma) {
        scoped_timer t(c, "sigma");
        hipError_t e = launch_sigma(c->H, c->prm, *C, salts, nullptr, c->num_cus, c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "sigma");
    }
    return PVAC_OK;
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
    hipError_t e = hipMemsetAsync(c->stats, 0, sizeof(plan_stats), c->stream);
    if (e == hipSuccess) e = launch_plan_add(*A, *B, *C, c->stats, c->stream);
    if (e == hipSuccess) e = launch_exclusive_scan_u64(C->l_off, A->n, c->scan_scratch, &c->totals[0], c->stream);
    if (e == hipSuccess) e = launch_exclusive_scan_u64(C->e_off, A->n, c->scan_scratch, &c->totals[1], c->stream);
    plan_stats st{};
    unsigned long long tot[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(&st, c->stats, sizeof st, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(tot, c->totals, sizeof tot, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "ct_add_plan");
    plan->total_layer_slots = tot[0];
    plan->total_edge_slots = tot[1];
    plan->max_layers = st.max_layers;
    plan->n_small = A->n;
    return PVAC_OK;
}

int pvac_hip_ct_add_exec(pvac_hip_ctx* c, const pvac_hip_plan* plan, const pvac_ct_batch* A, const pvac_ct_batch* B,
                         int negate_b, pvac_ct_batch* C) {
    if (!c || !plan || plan->kind != 2 || !batch_ok(A) || !batch_ok(B) || !batch_ok(C))
        return fail(c, PVAC_EINVAL, "ct_add_exec: bad arguments");
    if (A->n != plan->n_pairs || B->n != plan->n_pairs) return fail(c, PVAC_EINVAL, "ct_add_exec: plan mismatch");
    if (!A->n) return PVAC_OK;
    if (plan->max_layers > 30000) return fail(c, PVAC_ENOSYS, "ct_add_exec: > 30000 layers per cipher");
    // guard_budget: pairs whose |A.E|+|B.E| exceed edge_budget need compact_edges (layer-dense path)
    scoped_timer t(c, "ct_add");
    return hip_fail(c, launch_ct_add(*A, *B, *C, negate_b, plan->max_layers, c->stream), "ct_add");
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
        return hip_fail(c, sigma_tables_from_dense(c->H, c->prm, H, c->stream), "set_H");
    } catch (const std::exception& ex) {
        return fail(c, PVAC_ENOMEM, std::string("set_H: ") + ex.what());
    }
}

int pvac_hip_ctx_gen_H(pvac_hip_ctx* c, uint8_t digest[32]) {
    if (!c) return PVAC_EINVAL;
    try {
        scoped_timer t(c, "gen_H");
        return hip_fail(c, sigma_tables_generate(c->H, c->prm, digest, c->stream), "gen_H");
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

// ---------------------------------------------------------------- synthetic / checks
int pvac_hip_gen_fresh_batch(pvac_hip_ctx* c, uint64_t seed, uint32_t epl, pvac_ct_batch* X) {
    if (!c || !batch_ok(X) || !X->layers || !X->meta || !X->w_lo || !X->w_hi) return PVAC_EINVAL;
    return hip_fail(c, launch_gen_fresh(seed, epl, c->prm.B, *X, c->stream), "gen_fresh");
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

}  // extern "C"
