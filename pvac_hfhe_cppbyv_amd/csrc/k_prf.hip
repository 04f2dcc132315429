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

constexpr int kPB = 256;   // 4 requests per block (utility kernels)
constexpr int kCB = 512;   // k_prf_core: 8 requests per block share the 64 KB table (two blocks per CU)

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

// T0 with one private copy per lane: entry x of copy c at LDS byte (x << 8) | (c << 2) (64 copies of
// 1 KB), so no two lanes of a lookup share a bank, and a lookup's address is one v_perm of the state
// word: byte k of w into address byte 1, the lane's copy offset (lane * 4) in byte 0. T1..T3 are
// byte rotations of T0.
constexpr uint32_t kTBytes = 256u * 256u;

struct ttab {
    const uint8_t* b;   // LDS table
    uint32_t c4;        // lane * 4
    __device__ __forceinline__ uint32_t at(uint32_t addr) const { return *(const uint32_t*)(b + addr); }
    // T0[byte k of w]
    __device__ __forceinline__ uint32_t t0(uint32_t w, uint32_t k) const {
        return at(__builtin_amdgcn_perm(w, c4, 0x0C0C0000u | ((4u + k) << 8)));
    }
    __device__ __forceinline__ uint32_t sbox(uint32_t x) const { return (at((x << 8) | c4) >> 8) & 0xFFu; }
};

__device__ __forceinline__ uint32_t rotl(uint32_t v, int s) { return __builtin_amdgcn_alignbit(v, v, 32 - s); }

// one AES-256 round column: T0[w0.b0] ^ T1[w1.b1] ^ T2[w2.b2] ^ T3[w3.b3] ^ key (aes256_encrypt's order)
__device__ __forceinline__ uint32_t col(const ttab& T, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t key) {
    return T.t0(w0, 0) ^ rotl(T.t0(w1, 1), 8) ^ rotl(T.t0(w2, 2), 16) ^ rotl(T.t0(w3, 3), 24) ^ key;
}
// last-round column: the S-box bytes (byte 1 of T0) of w0.b0, w1.b1, w2.b2, w3.b3, packed by v_perm
__device__ __forceinline__ uint32_t col_last(const ttab& T, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                             uint32_t key) {
    const uint32_t v0 = T.t0(w0, 0), v1 = T.t0(w1, 1), v2 = T.t0(w2, 2), v3 = T.t0(w3, 3);
    const uint32_t lo = __builtin_amdgcn_perm(v1, v0, 0x0C0C0501u);   // [v0.b1, v1.b1, 0, 0]
    const uint32_t hi = __builtin_amdgcn_perm(v3, v2, 0x0C0C0501u);   // [v2.b1, v3.b1, 0, 0]
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u) ^ key;          // [lo.b0, lo.b1, hi.b0, hi.b1]
}

// AES-256 of counter blocks (ctr, 0) under the round keys rk (LDS, 60 words), NB blocks side by side
// (independent round chains for the scheduler to overlap); out: the two u64 halves of each block
template <int NB>
__device__ __forceinline__ void ctr_blocks(const uint64_t* ctr, const ttab& T, const uint32_t* rk, uint64_t* lo,
                                           uint64_t* hi) {
    uint32_t w[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        w[b][0] = (uint32_t)ctr[b] ^ rk[0];
        w[b][1] = (uint32_t)(ctr[b] >> 32) ^ rk[1];
        w[b][2] = rk[2];
        w[b][3] = rk[3];
    }
#pragma unroll
    for (int r = 1; r < 14; ++r) {
        const uint32_t k0 = rk[4 * r], k1 = rk[4 * r + 1], k2 = rk[4 * r + 2], k3 = rk[4 * r + 3];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const uint32_t n0 = col(T, w[b][0], w[b][1], w[b][2], w[b][3], k0);
            const uint32_t n1 = col(T, w[b][1], w[b][2], w[b][3], w[b][0], k1);
            const uint32_t n2 = col(T, w[b][2], w[b][3], w[b][0], w[b][1], k2);
            const uint32_t n3 = col(T, w[b][3], w[b][0], w[b][1], w[b][2], k3);
            w[b][0] = n0; w[b][1] = n1; w[b][2] = n2; w[b][3] = n3;
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const uint32_t n0 = col_last(T, w[b][0], w[b][1], w[b][2], w[b][3], rk[56]);
        const uint32_t n1 = col_last(T, w[b][1], w[b][2], w[b][3], w[b][0], rk[57]);
        const uint32_t n2 = col_last(T, w[b][2], w[b][3], w[b][0], w[b][1], rk[58]);
        const uint32_t n3 = col_last(T, w[b][3], w[b][0], w[b][1], w[b][2], rk[59]);
        lo[b] = ((uint64_t)n1 << 32) | n0;
        hi[b] = ((uint64_t)n3 << 32) | n2;
    }
}

__device__ __forceinline__ void ctr_block(uint64_t ctr, const ttab& T, const uint32_t* rk, uint64_t& lo, uint64_t& hi) {
    ctr_blocks<1>(&ctr, T, rk, &lo, &hi);
}

__device__ void expand_key(const uint32_t key[8], uint32_t* rk, const ttab& T) {
    uint32_t r[60];
    aes256_expand(key, r, [&](uint32_t x) { return T.sbox(x); });
    for (int i = threadIdx.x & 63; i < 60; i += 64) rk[i] = r[i];
}

__device__ __forceinline__ uint64_t wave_xor_u64(uint64_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x ^= (uint64_t)__shfl_xor((long long)x, d, 64);
    return x;
}

__global__ __launch_bounds__(kCB) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_prf_core(prf_consts k, const prf_request* req, uint64_t n, uint64_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t Tb[kTBytes];
    __shared__ uint64_t S[64];
    __shared__ uint32_t RK[kCB / 64][2][60];
    for (int i = threadIdx.x; i < (int)(kTBytes / 4); i += kCB) ((uint32_t*)Tb)[i] = c_aes.T[0][i >> 6];
    for (int i = threadIdx.x; i < 64; i += kCB) S[i] = i < (int)k.s_words ? k.s_bits[i] : 0ull;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const ttab T{Tb, (uint32_t)lane << 2};
    const uint64_t q = (uint64_t)blockIdx.x * (kCB / 64) + wave;
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
    // rows lane and lane + 64, their AES blocks interleaved: two independent round chains per lane
    // keep two sets of T-table lookups in flight (each chain alone waits on its LDS reads). Every
    // row spans the same number of blocks, (w0 + sw) / 2 - w0 / 2 + 1; lane 63's second row (127)
    // does not exist and is computed and dropped.
    uint32_t ybit[2] = {0, 0};
    bool rejected = false;
    {
        const uint64_t wa = row_words * (uint32_t)lane, wb = row_words * ((uint32_t)lane + 64u);
        const uint64_t ba = wa >> 1, bb = wb >> 1;
        const uint64_t nb = ((wa + sw) >> 1) - ba + 1;   // = for row lane + 64 (row_words odd or even alike)
        uint64_t acc[2] = {0, 0}, x[2] = {0, 0};
        const uint64_t w0s[2] = {wa, wb}, b0s[2] = {ba, bb};
        for (uint64_t kb = 0; kb < nb; ++kb) {
            uint64_t lo[2], hi[2];
            const uint64_t ctr[2] = {nonce + ba + kb, nonce + bb + kb};
            ctr_blocks<2>(ctr, T, rk, lo, hi);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint64_t w0 = w0s[h], b = b0s[h] + kb;
                const uint64_t qlo = 2 * b, qhi = 2 * b + 1;
                if (qlo >= w0 && qlo < w0 + sw) acc[h] ^= lo[h] & S[qlo - w0];
                if (qhi >= w0 && qhi < w0 + sw) acc[h] ^= hi[h] & S[qhi - w0];
                if (qlo == w0 + sw) x[h] = lo[h];
                if (qhi == w0 + sw) x[h] = hi[h];
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if ((uint32_t)lane + 64u * h >= 127u) continue;
            rejected |= x[h] >= lim;
            const uint32_t e = (x[h] % (uint64_t)k.tau_den) < (uint64_t)k.tau_num ? 1u : 0u;
            ybit[h] = (uint32_t)__builtin_parityll(acc[h]) ^ e;
        }
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
    const uint64_t blocks = (n + kCB / 64 - 1) / (kCB / 64);
    if (blocks > 0x7FFFFFFFull || k.s_words > 64 || k.tau_den == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_prf_core, dim3((unsigned)blocks), dim3(kCB), 0, st, k, (const prf_request*)req, n, out);
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
