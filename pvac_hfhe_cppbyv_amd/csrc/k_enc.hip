// k_enc.hip — batched enc_value (reference ops/encrypt.hpp:114-291) on CDNA4.
//
// enc_value(v) = combine_ciphers(enc_fp_depth(v + mask), enc_fp_depth(-mask)), mask =
// rand_fp_nonzero(). Every random choice comes from csprng_u64 in a fixed order, so a value's
// output is a function of its draw stream (the ABI input). The order the reference consumes it:
//   mask (2 words, rejection on 0), then enc_fp_depth(-mask) — GCC evaluates combine_ciphers'
//   second argument first (pinned by the reference's fixtures) — then enc_fp_depth(v + mask).
// Per enc_fp_depth: nonce (2), 8 signal (idx distinct by rejection, ch) pairs, r_0..r_6
// (rand_fp_nonzero), 8 salts (one per make_edge), Z2 pair groups (i, j != i, s1, r_i, 2 salts),
// Z3 triple groups (i, j, k distinct, s1..s3, a, b, 3 salts), then shuffle_edges (n - 1 draws)
// over the compact_edges output. The PRF values (prf_R, prf_noise_delta) and the weights do not
// draw, so one thread per value replays the whole stream first (k_enc_plan): it records every
// choice, the compact_edges groups ((idx, ch) order — keys alone decide them) and the shuffle
// permutation, and queues the PRF cores. k_prf_core evaluates them, k_enc_weights solves the
// signal / noise equations (ops/encrypt.hpp:185-252) and k_enc_finish folds each merged group
// (fp_add chain in creation order, sigma XOR) in shuffled order.
//
// A merged group whose weight and sigma both vanish is dropped by the reference, which then
// shuffles one edge fewer; that needs an exact cancellation (probability ~1/p) and is reported
// as status 2 instead of being reproduced.
#include "common.hpp"
#include "sha256.hpp"

namespace pvhip {
namespace {

constexpr int kEB = 64;

template <uint32_t CAP>   // pre-edge capacity: kEncPreSmall or kEncPreMax (group ids fit a byte)
struct enc_half {
    static_assert(CAP <= 256, "group ids and slots are bytes");
    uint64_t nlo, nhi, ztag;
    uint64_t vlo, vhi;            // the value this half encrypts (v + mask or -mask)
    uint32_t npre, nout;
    uint32_t key[CAP];            // idx | ch << 16, creation order
    uint64_t salt[CAP];
    uint64_t rlo[CAP], rhi[CAP];  // coefficients; solved ones filled by k_enc_weights
    uint8_t grp[CAP];             // compact_edges group of each pre-edge ((idx, P < M) order)
    uint8_t slot[CAP];            // output slot -> group (after shuffle_edges)
};

struct rstream {
    const uint64_t* p;
    uint32_t n, i;
    bool over;
    __device__ uint64_t next() {
        if (i < n) return p[i++];
        over = true;
        return 0;
    }
};

__device__ fp rand_fp_nonzero(rstream& rs) {   // core/types.hpp:145-155
    for (;;) {
        const uint64_t lo = rs.next();
        const uint64_t hi = rs.next() & kM63;
        const fp x = fp_from_words(lo, hi);
        if ((x.lo | x.hi) || rs.over) return x;
    }
}

__device__ __forceinline__ fp powg_at(const uint64_t* g, uint32_t i) { return fp{g[2 * i], g[2 * i + 1]}; }

// one enc_fp_depth draw replay (ops/encrypt.hpp:162-258, no PRF / weights)
template <uint32_t CAP>
__device__ void plan_half(const enc_plan_args& a, rstream& rs, const fp& v, enc_half<CAP>& H) {
    const uint32_t B = a.B;
    H.nlo = rs.next();
    H.nhi = rs.next();
    H.ztag = layer_ztag(a.canon, H.nlo, H.nhi);   // prg_layer_ztag (crypto/matrix.hpp:254-264)
    H.vlo = v.lo;
    H.vhi = v.hi;
    uint32_t idx[8], ch[8];
    for (int j = 0; j < 8; ++j) {   // pick_unique_idx (encrypt.hpp:130-135), then the sign
        uint32_t x;
        bool dup;
        do {
            x = (uint32_t)(rs.next() % B);
            dup = false;
            for (int q = 0; q < j; ++q) dup |= idx[q] == x;
        } while (dup && !rs.over);
        idx[j] = x;
        ch[j] = (uint32_t)(rs.next() & 1);
    }
    for (int j = 0; j < 7; ++j) {
        const fp r = rand_fp_nonzero(rs);
        H.rlo[j] = r.lo;
        H.rhi[j] = r.hi;
    }
    H.rlo[7] = 0;
    H.rhi[7] = 0;
    for (int j = 0; j < 8; ++j) {   // make_edge draws the salt (encrypt.hpp:150-153)
        H.key[j] = idx[j] | (ch[j] << 16);
        H.salt[j] = rs.next();
    }
    uint32_t np = 8;
    for (uint32_t t = 0; t < a.Z2; ++t) {   // encrypt.hpp:212-229
        const uint32_t i = (uint32_t)(rs.next() % B);
        uint32_t j;
        do { j = (uint32_t)(rs.next() % B); } while (j == i && !rs.over);
        const uint32_t s1 = (uint32_t)(rs.next() & 1), s2 = s1 ^ 1;
        const fp ri = rand_fp_nonzero(rs);
        H.key[np] = i | (s1 << 16); H.rlo[np] = ri.lo; H.rhi[np] = ri.hi; H.salt[np] = rs.next(); ++np;
        H.key[np] = j | (s2 << 16); H.rlo[np] = 0; H.rhi[np] = 0; H.salt[np] = rs.next(); ++np;
    }
    for (uint32_t t = 0; t < a.Z3; ++t) {   // encrypt.hpp:231-252
        const uint32_t i = (uint32_t)(rs.next() % B);
        uint32_t j, k;
        do { j = (uint32_t)(rs.next() % B); } while (j == i && !rs.over);
        do { k = (uint32_t)(rs.next() % B); } while ((k == i || k == j) && !rs.over);
        const uint32_t s1 = (uint32_t)(rs.next() & 1), s2 = (uint32_t)(rs.next() & 1), s3 = (uint32_t)(rs.next() & 1);
        const fp fa = rand_fp_nonzero(rs), fb = rand_fp_nonzero(rs);
        H.key[np] = i | (s1 << 16); H.rlo[np] = fa.lo; H.rhi[np] = fa.hi; H.salt[np] = rs.next(); ++np;
        H.key[np] = j | (s2 << 16); H.rlo[np] = fb.lo; H.rhi[np] = fb.hi; H.salt[np] = rs.next(); ++np;
        H.key[np] = k | (s3 << 16); H.rlo[np] = 0; H.rhi[np] = 0; H.salt[np] = rs.next(); ++np;
    }
    H.npre = np;
    // compact_edges (encrypt.hpp:39-71) output order: (layer, idx, P before M) over distinct keys.
    // First occurrences marked in slot[] (reused for the order below), then each pre-edge's group is
    // the number of distinct keys below its own: O(np^2)
    auto sk = [&](uint32_t e) { return (H.key[e] & 0xFFFFu) * 2u + (H.key[e] >> 16); };
    uint32_t ng = 0;
    for (uint32_t e = 0; e < np; ++e) {
        const uint32_t k = sk(e);
        bool first = true;
        for (uint32_t q = 0; q < e; ++q) first &= sk(q) != k;
        H.slot[e] = first ? 1u : 0u;
        ng += first ? 1u : 0u;
    }
    for (uint32_t e = 0; e < np; ++e) {
        const uint32_t k = sk(e);
        uint32_t rank = 0;
        for (uint32_t f = 0; f < np; ++f) rank += (H.slot[f] && sk(f) < k) ? 1u : 0u;
        H.grp[e] = (uint8_t)rank;
    }
    // shuffle_edges (encrypt.hpp:155-160) on the ng compacted entries, in place in slot[]
    for (uint32_t g = 0; g < ng; ++g) H.slot[g] = (uint8_t)g;
    for (uint32_t i = ng > 1 ? ng - 1 : 0; i > 0; --i) {
        const uint32_t j = (uint32_t)(rs.next() % (uint64_t)(i + 1));
        const uint8_t t = H.slot[i];
        H.slot[i] = H.slot[j];
        H.slot[j] = t;
    }
    H.nout = ng;
}

// prf requests of one half: prf_R's three cores (seed = the layer seed) and, for every group but
// the last, prf_noise_delta's three cores on the derived seed (encrypt.hpp:113-128, 205-210)
template <class HALF>
__device__ void half_requests(const enc_plan_args& a, const HALF& H, prf_request* req) {
    for (uint32_t c = 0; c < 3; ++c) req[c] = prf_request{H.ztag, H.nlo, H.nhi, c, 0};
    const uint32_t G = a.Z2 + a.Z3;
    for (uint32_t g = 0; g + 1 < G; ++g) {
        const uint64_t gg = (uint64_t)g + 1, kk = (uint64_t)(g < a.Z2 ? 0 : 1) + 1;
        uint64_t lo = H.nlo ^ (0x9e3779b97f4a7c15ull * gg), hi = H.nhi ^ (0x94d049bb133111ebull * gg);
        uint64_t z = H.ztag ^ (0x517cc1b727220a95ull * gg);
        lo ^= kk;
        hi ^= kk << 32;
        z ^= kk << 48;
        for (uint32_t c = 0; c < 3; ++c) req[3 + 3 * g + c] = prf_request{z, lo, hi, 3 + c, 0};
    }
}

template <uint32_t CAP>
__global__ __launch_bounds__(kEB) void k_enc_plan(enc_plan_args a, enc_half<CAP>* halves, prf_request* req,
                                                  pvac_ct_batch pre, uint64_t* pre_salt, uint32_t* status) {
    const uint64_t i = (uint64_t)blockIdx.x * kEB + threadIdx.x;
    if (i >= a.n) return;
    rstream rs{a.rnd + i * a.stride, a.stride, 0, false};
    const fp mask = rand_fp_nonzero(rs);
    const fp va = fp_add(fp{a.values[i], 0}, mask), vb = fp_neg(mask);
    enc_half<CAP>& A = halves[2 * i];       // output layer 0: enc_fp_depth(v + mask)
    enc_half<CAP>& Bh = halves[2 * i + 1];  // output layer 1: enc_fp_depth(-mask), drawn first
    plan_half(a, rs, vb, Bh);
    plan_half(a, rs, va, A);
    status[i] = rs.over ? 1u : 0u;
    const uint32_t per_half = 3 * max(a.Z2 + a.Z3, 1u);
    half_requests(a, A, req + i * 2 * per_half);
    half_requests(a, Bh, req + i * 2 * per_half + per_half);
    // pre-merge batch for sigma_from_H: 2 BASE layers, the halves' edges in creation order
    const uint32_t npre = 8 + 2 * a.Z2 + 3 * a.Z3;
    pre.l_off[i] = 2 * i;
    pre.l_cnt[i] = 2;
    pre.e_off[i] = i * 2 * npre;
    pre.e_cnt[i] = 2 * npre;
    for (int h = 0; h < 2; ++h) {
        const enc_half<CAP>& H = h ? Bh : A;
        pvac_layer y{};
        y.ztag = H.ztag;
        y.nonce_lo = H.nlo;
        y.nonce_hi = H.nhi;
        pre.layers[2 * i + h] = y;
        for (uint32_t e = 0; e < npre; ++e) {
            const uint64_t s = i * 2 * npre + (uint64_t)h * npre + e;
            pre.meta[s] = make_meta((uint32_t)h, H.key[e] & 0xFFFFu, H.key[e] >> 16);
            pre_salt[s] = H.salt[e];
        }
    }
}

template <uint32_t CAP>
__global__ __launch_bounds__(kEB) void k_enc_weights(enc_plan_args a, enc_half<CAP>* halves, const uint64_t* cores,
                                                     pvac_ct_batch pre) {
    const uint64_t hi_ = (uint64_t)blockIdx.x * kEB + threadIdx.x;
    if (hi_ >= 2 * a.n) return;
    enc_half<CAP>& H = halves[hi_];
    const uint32_t G = a.Z2 + a.Z3;
    const uint32_t per_half = 3 * max(G, 1u);
    const uint64_t* c = cores + 2 * hi_ * per_half;
    auto core = [&](uint32_t q) { return fp{c[2 * q], c[2 * q + 1]}; };
    const fp R = fp_mul(fp_mul(core(0), core(1)), core(2));   // prf_R (lpn.hpp:263-268)
    auto rr = [&](uint32_t e) { return fp{H.rlo[e], H.rhi[e]}; };
    auto idx = [&](uint32_t e) { return H.key[e] & 0xFFFFu; };
    auto chn = [&](uint32_t e) { return H.key[e] >> 16; };
    // signal (encrypt.hpp:184-193): the last coefficient solves sum(+/- r_j g^idx_j) = v
    fp sumg{0, 0};
    for (uint32_t j = 0; j < 7; ++j) {
        const fp term = fp_mul(rr(j), powg_at(a.powg, idx(j)));
        sumg = chn(j) == 0 ? fp_add(sumg, term) : fp_sub(sumg, term);
    }
    const fp rl = fp_mul(fp_sub(fp{H.vlo, H.vhi}, sumg), fp_inv(powg_at(a.powg, idx(7))));
    const fp r7 = chn(7) == 0 ? rl : fp_neg(rl);
    H.rlo[7] = r7.lo;
    H.rhi[7] = r7.hi;
    // noise groups: Delta_g = prf_noise_delta for all but the last, which takes -(their sum)
    fp dacc{0, 0};
    uint32_t gid = 0;
    auto delta = [&]() {
        if (G - gid <= 1) return fp_neg(dacc);
        const uint32_t q = 3 + 3 * gid;
        const fp d = fp_mul(fp_mul(core(q), core(q + 1)), core(q + 2));   // prf_R_noise
        dacc = fp_add(dacc, d);
        return d;
    };
    uint32_t e = 8;
    for (uint32_t t = 0; t < a.Z2; ++t, ++gid, e += 2) {   // encrypt.hpp:212-229
        const fp D = delta();
        const fp Dp = chn(e) == 0 ? D : fp_neg(D);
        const fp rj = fp_mul(fp_sub(fp_mul(rr(e), powg_at(a.powg, idx(e))), Dp), fp_inv(powg_at(a.powg, idx(e + 1))));
        H.rlo[e + 1] = rj.lo;
        H.rhi[e + 1] = rj.hi;
    }
    for (uint32_t t = 0; t < a.Z3; ++t, ++gid, e += 3) {   // encrypt.hpp:231-252
        const fp D = delta();
        fp t1 = fp_mul(rr(e), powg_at(a.powg, idx(e)));
        fp t2 = fp_mul(rr(e + 1), powg_at(a.powg, idx(e + 1)));
        if (chn(e)) t1 = fp_neg(t1);
        if (chn(e + 1)) t2 = fp_neg(t2);
        const fp gk = chn(e + 2) == 0 ? powg_at(a.powg, idx(e + 2)) : fp_neg(powg_at(a.powg, idx(e + 2)));
        const fp cc = fp_mul(fp_sub(D, fp_add(t1, t2)), fp_inv(gk));
        H.rlo[e + 2] = cc.lo;
        H.rhi[e + 2] = cc.hi;
    }
    // weights w = r * R (make_edge arguments)
    const uint64_t i = hi_ >> 1, h = hi_ & 1;
    const uint32_t npre = 8 + 2 * a.Z2 + 3 * a.Z3;
    for (uint32_t q = 0; q < H.npre; ++q) {
        const fp w = fp_mul(rr(q), R);
        const uint64_t s = i * 2 * npre + h * npre + q;
        pre.w_lo[s] = w.lo;
        pre.w_hi[s] = w.hi;
    }
}

// one wave per value: merged groups in shuffled order; lanes XOR sigma words
template <uint32_t CAP>
__global__ __launch_bounds__(kEB) void k_enc_finish(enc_plan_args a, const enc_half<CAP>* halves, pvac_ct_batch pre,
                                                    pvac_ct_batch C, uint32_t* status) {
    const uint64_t i = blockIdx.x;
    if (i >= a.n) return;
    const int lane = threadIdx.x;
    const uint32_t npre = 8 + 2 * a.Z2 + 3 * a.Z3;
    const uint64_t lo = 2 * i, eo = i * 2 * npre;
    C.l_off[i] = lo;
    C.l_cnt[i] = 2;
    C.e_off[i] = eo;
    uint32_t pos = 0;
    bool vanished = false;
    for (int h = 0; h < 2; ++h) {
        const enc_half<CAP>& H = halves[2 * i + h];
        if (lane == 0) {
            pvac_layer y{};
            y.ztag = H.ztag;
            y.nonce_lo = H.nlo;
            y.nonce_hi = H.nhi;
            C.layers[lo + h] = y;
        }
        for (uint32_t s = 0; s < H.nout; ++s) {
            const uint32_t g = H.slot[s];
            fp w{0, 0};
            uint32_t key = 0;
            uint64_t any = 0;
            // compact_edges: fp_add chain in creation order from 0, sigma XOR (encrypt.hpp:45-58)
            for (uint32_t e = 0; e < H.npre; ++e) {
                if (H.grp[e] != g) continue;
                const uint64_t src = eo + (uint64_t)h * npre + e;
                w = fp_add(w, fp{pre.w_lo[src], pre.w_hi[src]});
                key = H.key[e];
            }
            const uint64_t dst = eo + pos + s;
            if (pre.sigma && C.sigma) {
                for (uint32_t wd = lane; wd < C.sigma_words; wd += 64) {
                    uint64_t x = 0;
                    for (uint32_t e = 0; e < H.npre; ++e)
                        if (H.grp[e] == g) x ^= pre.sigma[(eo + (uint64_t)h * npre + e) * pre.sigma_words + wd];
                    C.sigma[dst * C.sigma_words + wd] = x;
                    any |= x;
                }
            }
            const bool sig_nz = __ballot(any != 0) != 0;
            vanished |= !(w.lo | w.hi) && !sig_nz;
            if (lane == 0) {
                C.meta[dst] = make_meta((uint32_t)h, key & 0xFFFFu, key >> 16);
                C.w_lo[dst] = w.lo;
                C.w_hi[dst] = w.hi;
            }
        }
        pos += H.nout;
    }
    if (lane == 0) {
        C.e_cnt[i] = pos;
        if (vanished && status[i] == 0) status[i] = 2;
    }
}

}  // namespace

static bool enc_small(uint32_t npre) { return npre <= kEncPreSmall; }

size_t enc_half_bytes(uint32_t npre) {
    return enc_small(npre) ? sizeof(enc_half<kEncPreSmall>) : sizeof(enc_half<kEncPreMax>);
}

uint32_t enc_cores_per_value(uint32_t Z2, uint32_t Z3) { return 2u * 3u * std::max(Z2 + Z3, 1u); }

hipError_t launch_enc_plan(const enc_plan_args& a, void* halves, prf_request* req, pvac_ct_batch& pre,
                           uint64_t* pre_salt, uint32_t* status, hipStream_t st) {
    if (!a.n) return hipSuccess;
    const uint32_t npre = 8 + 2 * a.Z2 + 3 * a.Z3;
    if (npre > kEncPreMax || a.B == 0 || a.B > 65536) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((a.n + kEB - 1) / kEB));
    if (enc_small(npre))
        hipLaunchKernelGGL(k_enc_plan<kEncPreSmall>, grid, dim3(kEB), 0, st, a, (enc_half<kEncPreSmall>*)halves, req, pre,
                           pre_salt, status);
    else
        hipLaunchKernelGGL(k_enc_plan<kEncPreMax>, grid, dim3(kEB), 0, st, a, (enc_half<kEncPreMax>*)halves, req, pre,
                           pre_salt, status);
    return hipGetLastError();
}

hipError_t launch_enc_weights(const enc_plan_args& a, void* halves, const uint64_t* cores, pvac_ct_batch& pre,
                              hipStream_t st) {
    if (!a.n) return hipSuccess;
    const dim3 grid((unsigned)((2 * a.n + kEB - 1) / kEB));
    if (enc_small(8 + 2 * a.Z2 + 3 * a.Z3))
        hipLaunchKernelGGL(k_enc_weights<kEncPreSmall>, grid, dim3(kEB), 0, st, a, (enc_half<kEncPreSmall>*)halves, cores,
                           pre);
    else
        hipLaunchKernelGGL(k_enc_weights<kEncPreMax>, grid, dim3(kEB), 0, st, a, (enc_half<kEncPreMax>*)halves, cores, pre);
    return hipGetLastError();
}

hipError_t launch_enc_finish(const enc_plan_args& a, const void* halves, const pvac_ct_batch& pre, pvac_ct_batch& C,
                             uint32_t* status, hipStream_t st) {
    if (!a.n) return hipSuccess;
    if (a.n > 0x7FFFFFFFull) return hipErrorInvalidValue;
    if (enc_small(8 + 2 * a.Z2 + 3 * a.Z3))
        hipLaunchKernelGGL(k_enc_finish<kEncPreSmall>, dim3((unsigned)a.n), dim3(kEB), 0, st, a,
                           (const enc_half<kEncPreSmall>*)halves, pre, C, status);
    else
        hipLaunchKernelGGL(k_enc_finish<kEncPreMax>, dim3((unsigned)a.n), dim3(kEB), 0, st, a,
                           (const enc_half<kEncPreMax>*)halves, pre, C, status);
    return hipGetLastError();
}

}  // namespace pvhip
