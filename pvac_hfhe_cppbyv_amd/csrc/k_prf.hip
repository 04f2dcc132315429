// k_prf.hip — the LPN PRF prf_R_core (reference crypto/lpn.hpp:159-268) on CDNA4.
//
// prf_R_core(seed, dom):
//   key, nonce   = SHA-256(prf_k || canon || H_digest || ztag || nonce_lo || nonce_hi || fnv(dom)),
//                  nonce = fnv(dom) ^ nonce_lo                                   (lpn.hpp:159-186)
//   y bit r      = parity(64 keystream words & s) ^ [bounded(tau_den) < tau_num]  (lpn.hpp:188-224)
//   top          = the Toeplitz key's keystream (key/nonce from dom "pvac.dom.toeplitz", nonce ^ fnv(dom))
//   R            = hash_to_fp_nonzero(low 127 bits of y * top over GF(2))        (toeplitz.hpp, lpn.hpp:25-37)
// Only rows 0..126 and the first 127 bits of top reach the output: coefficient j < 127 of a
// carry-less product involves coefficients <= j of both factors. The reference loops all lpn_t
// (16384) rows; 127 rows give the identical value (pinned: tests/test_oracle_enc.py,
// tests/test_gpu_enc.py), ≈4.1 K AES-256 blocks per call instead of ≈532 K.
//
// One wave per request. The 104-byte key-derivation message's first block is fixed per key: its
// SHA-256 midstate comes from the host, so each derivation is one compression. Lane l evaluates
// rows l and l + 64 (33 AES blocks each; row r's 64 words start at keystream word 65 r because
// every row consumes 64 words plus one bounded draw). A bounded draw that would be rejected
// (probability ~tau_den / 2^64 per row) shifts every later row: such a request is recomputed by
// an exact sequential walk instead.
#include "common.hpp"
#include "aes256.hpp"
#include "sha256.hpp"

namespace pvhip {
namespace {

constexpr int kPB = 256;   // 4 requests per block

__constant__ aes_ttables c_aes;

__device__ __forceinline__ uint32_t bswap32d(uint32_t x) { return __builtin_bswap32(x); }

// block 2 of the derivation message (bytes 64..127): H_digest[24..32) | ztag | nlo | nhi | dom | pad
__device__ __forceinline__ void derive(const prf_consts& k, uint64_t ztag, uint64_t nlo, uint64_t nhi, uint64_t dh,
                                       uint32_t key[8]) {
    uint32_t w[16];
    const uint64_t le[5] = {k.hd_tail, ztag, nlo, nhi, dh};
#pragma unroll
    for (int i = 0; i < 5; ++i) {   // little-endian u64 bytes as big-endian message words
        w[2 * i] = bswap32d((uint32_t)le[i]);
        w[2 * i + 1] = bswap32d((uint32_t)(le[i] >> 32));
    }
    w[10] = 0x80000000u;
#pragma unroll
    for (int i = 11; i < 15; ++i) w[i] = 0;
    w[15] = 104u * 8u;
    sha_state s;
#pragma unroll
    for (int i = 0; i < 8; ++i) s.h[i] = k.mid[i];
    sha_compress(s, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) key[i] = bswap32d(s.h[i]);   // digest bytes -> little-endian key words
}

// T0 only, replicated kTCopies times in a bank-per-lane layout: entry x of copy c is LDS word
// x * kTCopies + c, and lane l reads copy l % kTCopies, so the 64 lanes of a lookup hit at most two
// words per bank (one per lane half) instead of colliding at random; T1..T3 are byte rotations.
constexpr uint32_t kTCopies = 32;

__device__ __forceinline__ uint32_t tlook(const uint32_t* T, uint32_t x) {
    return T[(x * kTCopies) | (threadIdx.x & (kTCopies - 1))];
}

__device__ __forceinline__ void ctr_block(uint64_t ctr, const uint32_t* T, const uint32_t* rk, uint64_t& lo,
                                          uint64_t& hi) {
    uint32_t w0 = (uint32_t)ctr, w1 = (uint32_t)(ctr >> 32), w2 = 0, w3 = 0;
    aes256_encrypt(w0, w1, w2, w3,
                   [&](int t, uint32_t x) {
                       const uint32_t v = tlook(T, x);
                       return t == 0 ? v : __builtin_amdgcn_alignbit(v, v, 32 - 8 * t);   // rotl(v, 8t)
                   },
                   [&](int i) { return rk[i]; });
    lo = ((uint64_t)w1 << 32) | w0;
    hi = ((uint64_t)w3 << 32) | w2;
}

__device__ void expand_key(const uint32_t key[8], uint32_t* rk, const uint32_t* T) {
    uint32_t r[60];
    aes256_expand(key, r, [&](uint32_t x) { return (tlook(T, x) >> 8) & 0xFFu; });
    for (int i = threadIdx.x & 63; i < 60; i += 64) rk[i] = r[i];
}

__device__ __forceinline__ uint64_t wave_xor_u64(uint64_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x ^= (uint64_t)__shfl_xor((long long)x, d, 64);
    return x;
}

__global__ __launch_bounds__(kPB, 4) void k_prf_core(prf_consts k, const prf_request* req, uint64_t n, uint64_t* out) {
    __shared__ uint32_t T[256 * kTCopies];
    __shared__ uint64_t S[64];
    __shared__ uint32_t RK[kPB / 64][2][60];
    for (int i = threadIdx.x; i < 256 * (int)kTCopies; i += kPB) T[i] = c_aes.T[0][i / kTCopies];
    for (int i = threadIdx.x; i < 64; i += kPB) S[i] = i < (int)k.s_words ? k.s_bits[i] : 0ull;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t q = (uint64_t)blockIdx.x * (kPB / 64) + wave;
    if (q >= n) return;   // wave-uniform; no block barrier below
    const prf_request rq = req[q];
    const uint64_t dh = k.dom_hash[rq.dom];
    uint32_t key[8];
    derive(k, rq.ztag, rq.nonce_lo, rq.nonce_hi, dh, key);
    uint32_t* rk = RK[wave][0];
    uint32_t* rkt = RK[wave][1];
    expand_key(key, rk, T);
    derive(k, rq.ztag, rq.nonce_lo, rq.nonce_hi, k.toep_hash, key);
    expand_key(key, rkt, T);
    __builtin_amdgcn_wave_barrier();
    const uint64_t nonce = dh ^ rq.nonce_lo;
    const uint64_t tnonce = (k.toep_hash ^ rq.nonce_lo) ^ dh;
    const uint64_t lim = ~0ull - (~0ull % (uint64_t)k.tau_den);
    const uint32_t sw = k.s_words;           // 64 for lpn_n = 4096
    const uint64_t row_words = sw + 1ull;    // 64 row words + one bounded draw
    // rows lane and lane + 64
    uint32_t ybit[2] = {0, 0};
    bool rejected = false;
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
        const uint32_t r = (uint32_t)lane + 64u * h;
        if (r >= 127u) continue;
        const uint64_t w0 = row_words * r;           // first keystream word of the row
        const uint64_t b0 = w0 >> 1, b1 = (w0 + sw) >> 1;
        uint64_t acc = 0, x = 0;
        for (uint64_t b = b0; b <= b1; ++b) {
            uint64_t lo, hi;
            ctr_block(nonce + b, T, rk, lo, hi);
            const uint64_t qlo = 2 * b, qhi = 2 * b + 1;
            if (qlo >= w0 && qlo < w0 + sw) acc ^= lo & S[qlo - w0];
            if (qhi >= w0 && qhi < w0 + sw) acc ^= hi & S[qhi - w0];
            if (qlo == w0 + sw) x = lo;
            if (qhi == w0 + sw) x = hi;
        }
        rejected |= x >= lim;
        const uint32_t e = (x % (uint64_t)k.tau_den) < (uint64_t)k.tau_num ? 1u : 0u;
        ybit[h] = (uint32_t)__builtin_parityll(acc) ^ e;
    }
    uint64_t y0 = __ballot(ybit[0] != 0), y1 = __ballot(ybit[1] != 0) & 0x7FFFFFFFFFFFFFFFull;
    if (__ballot(rejected)) {
        // exact sequential walk with the reference's rejection loop (AesCtr256::bounded)
        y0 = 0; y1 = 0;
        if (lane == 0) {
            uint64_t p = 0;   // keystream word index
            auto word = [&](uint64_t i) {
                uint64_t lo, hi;
                ctr_block(nonce + (i >> 1), T, rk, lo, hi);
                return (i & 1) ? hi : lo;
            };
            for (uint32_t r = 0; r < 127; ++r) {
                uint64_t acc = 0;
                for (uint32_t w = 0; w < sw; ++w) acc ^= word(p++) & S[w];
                uint64_t x;
                do { x = word(p++); } while (x >= lim);
                const uint32_t e = (x % (uint64_t)k.tau_den) < (uint64_t)k.tau_num ? 1u : 0u;
                const uint64_t bit = (uint64_t)(__builtin_parityll(acc) ^ e);
                if (r < 64) y0 |= bit << r; else y1 |= bit << (r - 64);
            }
        }
        y0 = (uint64_t)__shfl((long long)y0, 0, 64);
        y1 = (uint64_t)__shfl((long long)y1, 0, 64);
    }
    // Toeplitz: low 127 bits of y * top (top = the first two words of the Toeplitz keystream)
    uint64_t t0, t1;
    ctr_block(tnonce, T, rkt, t0, t1);
    uint64_t lo = 0, hi = 0;
    const uint32_t i = (uint32_t)lane;
    if ((y0 >> i) & 1) {   // y bit i: top << i
        lo ^= t0 << i;
        hi ^= i ? (t1 << i) | (t0 >> (64 - i)) : t1;
    }
    if (i < 63 && ((y1 >> i) & 1)) hi ^= t0 << i;   // y bit 64 + i: (top << 64) << i
    lo = wave_xor_u64(lo);
    hi = wave_xor_u64(hi) & 0x7FFFFFFFFFFFFFFFull;
    if (lane == 0) {
        fp r = fp_from_words(lo, hi);   // hash_to_fp_nonzero
        if (!(r.lo | r.hi)) r = fp{1, 0};
        out[2 * q] = r.lo;
        out[2 * q + 1] = r.hi;
    }
}

// out[i] = in[3i] * in[3i+1] * in[3i+2] (prf_R / prf_R_noise from their three cores)
__global__ __launch_bounds__(kPB) void k_prf_triple(const uint64_t* in, uint64_t n, uint64_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * kPB + threadIdx.x;
    if (i >= n) return;
    const fp a{in[6 * i], in[6 * i + 1]}, b{in[6 * i + 2], in[6 * i + 3]}, c{in[6 * i + 4], in[6 * i + 5]};
    const fp r = fp_mul(fp_mul(a, b), c);
    out[2 * i] = r.lo;
    out[2 * i + 1] = r.hi;
}

// kind 0..5: one core per seed; 6 / 7: prf_R / prf_R_noise (three cores per seed)
__global__ __launch_bounds__(kPB) void k_prf_requests(const uint64_t* seeds, uint64_t n, int kind, prf_request* req) {
    const uint64_t i = (uint64_t)blockIdx.x * kPB + threadIdx.x;
    if (i >= n) return;
    const int per = kind >= 6 ? 3 : 1;
    for (int c = 0; c < per; ++c) {
        prf_request r{};
        r.ztag = seeds[3 * i];
        r.nonce_lo = seeds[3 * i + 1];
        r.nonce_hi = seeds[3 * i + 2];
        r.dom = kind >= 6 ? (uint32_t)(3 * (kind - 6) + c) : (uint32_t)kind;
        req[per * i + c] = r;
    }
}

// BASE-layer requests for base_R: slot s of cipher i -> 3 cores (doms 0..2); PROD slots get a
// dummy request whose result is ignored (zeroed by k_base_R_out)
__global__ __launch_bounds__(kPB) void k_base_R_requests(pvac_ct_batch X, uint64_t n_slots, prf_request* req,
                                                         uint8_t* is_base) {
    const uint64_t c = blockIdx.x;
    if (c >= X.n) return;
    const uint64_t lo = X.l_off[c], lc = X.l_cnt[c];
    for (uint64_t l = threadIdx.x; l < lc; l += kPB) {
        const uint64_t s = lo + l;
        if (s >= n_slots) continue;
        const pvac_layer y = X.layers[s];
        for (uint32_t d = 0; d < 3; ++d) req[3 * s + d] = prf_request{y.ztag, y.nonce_lo, y.nonce_hi, d, 0};
        is_base[s] = y.rule == 0 ? 1 : 0;
    }
}

__global__ __launch_bounds__(kPB) void k_base_R_out(const uint64_t* cores, const uint8_t* is_base, uint64_t n_slots,
                                                    uint64_t* R) {
    const uint64_t s = (uint64_t)blockIdx.x * kPB + threadIdx.x;
    if (s >= n_slots) return;
    fp r{0, 0};
    if (is_base[s]) {
        const fp a{cores[6 * s], cores[6 * s + 1]}, b{cores[6 * s + 2], cores[6 * s + 3]},
            c{cores[6 * s + 4], cores[6 * s + 5]};
        r = fp_mul(fp_mul(a, b), c);
    }
    R[2 * s] = r.lo;
    R[2 * s + 1] = r.hi;
}

}  // namespace

hipError_t prf_upload_tables(hipStream_t st) {
    static const aes_ttables t = aes_make_tables();
    return hipMemcpyToSymbolAsync(HIP_SYMBOL(c_aes), &t, sizeof t, 0, hipMemcpyHostToDevice, st);
}

size_t prf_request_bytes() { return sizeof(prf_request); }

hipError_t launch_prf_cores(const prf_consts& k, const void* req, uint64_t n, uint64_t* out, hipStream_t st) {
    if (!n) return hipSuccess;
    const uint64_t blocks = (n + kPB / 64 - 1) / (kPB / 64);
    if (blocks > 0x7FFFFFFFull || k.s_words > 64 || k.tau_den == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_prf_core, dim3((unsigned)blocks), dim3(kPB), 0, st, k, (const prf_request*)req, n, out);
    return hipGetLastError();
}

hipError_t launch_prf(const prf_consts& k, int kind, const uint64_t* seeds, uint64_t n, void* req_scratch,
                      uint64_t* core_scratch, uint64_t* out, hipStream_t st) {
    if (!n) return hipSuccess;
    const unsigned blocks = (unsigned)((n + kPB - 1) / kPB);
    hipLaunchKernelGGL(k_prf_requests, dim3(blocks), dim3(kPB), 0, st, seeds, n, kind, (prf_request*)req_scratch);
    const uint64_t cores = kind >= 6 ? 3 * n : n;
    hipError_t e = launch_prf_cores(k, req_scratch, cores, kind >= 6 ? core_scratch : out, st);
    if (e != hipSuccess || kind < 6) return e;
    hipLaunchKernelGGL(k_prf_triple, dim3(blocks), dim3(kPB), 0, st, core_scratch, n, out);
    return hipGetLastError();
}

hipError_t launch_base_R(const prf_consts& k, const pvac_ct_batch& X, uint64_t n_slots, void* req_scratch,
                         uint64_t* core_scratch, uint64_t* R_out, hipStream_t st) {
    if (!X.n || !n_slots) return hipSuccess;
    if (X.n > 0x7FFFFFFFull) return hipErrorInvalidValue;
    prf_request* req = (prf_request*)req_scratch;
    // requests for slots not covered by any cipher stay as they were: mark them non-BASE first
    uint8_t* is_base = (uint8_t*)(core_scratch + 6 * n_slots);   // scratch tail (caller sized 8 n_slots words)
    hipError_t e = hipMemsetAsync(is_base, 0, n_slots, st);
    if (e == hipSuccess) e = hipMemsetAsync(req, 0, n_slots * 3 * sizeof(prf_request), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_base_R_requests, dim3((unsigned)X.n), dim3(kPB), 0, st, X, n_slots, req, is_base);
    e = launch_prf_cores(k, req, 3 * n_slots, core_scratch, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_base_R_out, dim3((unsigned)((n_slots + kPB - 1) / kPB)), dim3(kPB), 0, st, core_scratch,
                       is_base, n_slots, R_out);
    return hipGetLastError();
}

}  // namespace pvhip
