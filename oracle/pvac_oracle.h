/* pvac_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the pvac-hfhe 0.1.0 hot path (reference: /root/reference/include/pvac),
 * used exclusively as the CHECKER by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg. The product (libpvac_hip.so) never links, loads or calls this library.
 *
 * Parity status: PINNED — every function here is checked in tests/test_oracle.py against
 * golden vectors minted by the unmodified reference (oracle/ref_harness.cpp ->
 * tests/golden/ref/, tests/golden/bounty/).
 *
 * Cipher views use the same flat layout as the engine ABI (include/pvac_hip.h):
 *   layer record 40 B {u32 rule, u32 pa, u32 pb, u32 pad, u64 ztag, u64 nonce_lo, u64 nonce_hi}
 *   edge meta u64  = layer_id | (u64)idx << 32 | (u64)ch << 48   (the .ct edge header bytes)
 *   weights        = separate w_lo[], w_hi[] u64 arrays
 *   sigma          = sigma_words u64 per edge (nullable)
 */
#ifndef PVAC_ORACLE_H
#define PVAC_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_layer {
    uint32_t rule, pa, pb, pad;
    uint64_t ztag, nonce_lo, nonce_hi;
} orc_layer;

typedef struct orc_params {
    uint32_t B, m_bits, n_bits, h_col_wt, x_col_wt, err_wt;
    uint64_t edge_budget;
    uint64_t canon_tag;
} orc_params;

typedef struct orc_cipher {
    uint64_t nL, nE;          /* counts (in) / counts written (out) */
    uint64_t capL, capE;      /* capacities (out only) */
    orc_layer* layers;
    uint64_t* meta;
    uint64_t* w_lo;
    uint64_t* w_hi;
    uint64_t* sigma;          /* nullable */
    uint32_t sigma_words;
} orc_cipher;

/* secret-key material of the LPN PRF (crypto/lpn.hpp; SecKey core/types.hpp:134-137) */
typedef struct orc_secret {
    uint64_t prf_k[4];
    const uint64_t* lpn_s;   /* ceil(lpn_n / 64) words */
    uint32_t lpn_n, lpn_t, tau_num, tau_den;
    uint8_t H_digest[32];
} orc_secret;

/* ---- Fp over p = 2^127-1 (core/field.hpp) ---- */
void orc_fp_from_words(const uint64_t* lo, const uint64_t* hi, uint64_t* olo, uint64_t* ohi, size_t n);
void orc_fp_add(const uint64_t* alo, const uint64_t* ahi, const uint64_t* blo, const uint64_t* bhi,
                uint64_t* olo, uint64_t* ohi, size_t n);
void orc_fp_sub(const uint64_t* alo, const uint64_t* ahi, const uint64_t* blo, const uint64_t* bhi,
                uint64_t* olo, uint64_t* ohi, size_t n);
void orc_fp_neg(const uint64_t* alo, const uint64_t* ahi, uint64_t* olo, uint64_t* ohi, size_t n);
void orc_fp_mul(const uint64_t* alo, const uint64_t* ahi, const uint64_t* blo, const uint64_t* bhi,
                uint64_t* olo, uint64_t* ohi, size_t n);
void orc_fp_inv(const uint64_t* alo, const uint64_t* ahi, uint64_t* olo, uint64_t* ohi, size_t n);
void orc_fp_pow(const uint64_t* alo, const uint64_t* ahi, const uint64_t* e, uint64_t* olo, uint64_t* ohi, size_t n);
/* multi-threaded element-wise timing helper for the cpu_baseline leg: returns seconds */
double orc_fp_binop_timed(int op, const uint64_t* alo, const uint64_t* ahi, const uint64_t* blo,
                          const uint64_t* bhi, uint64_t* olo, uint64_t* ohi, size_t n, int threads);

/* ---- hashing / PRG (core/hash.hpp, crypto/matrix.hpp) ---- */
void orc_sha256(const uint8_t* msg, size_t n, uint8_t out[32]);
uint64_t orc_layer_ztag(uint64_t canon_tag, uint64_t nonce_lo, uint64_t nonce_hi);
int orc_prg_choose_k(int k, int N, const char* label, const uint64_t* words, int nwords, int32_t* out);
/* dense H: n_bits columns x ceil(m_bits/64) words; returns H_digest */
int orc_gen_H(const orc_params* prm, uint64_t* H_dense, uint8_t digest[32]);
void orc_sigma_from_H(const orc_params* prm, const uint64_t* H_dense, uint64_t ztag, uint64_t nonce_lo,
                      uint64_t nonce_hi, uint32_t idx, uint32_t ch, uint64_t salt, uint64_t* out_words);

/* ---- ciphertext ops (ops/arithmetic.hpp, ops/encrypt.hpp) ----
 * H_dense == NULL  => weights-only (sigma not produced / copied as given).
 * return 0 ok, <0 error (capacity). */
int orc_ct_add(const orc_params* prm, const orc_cipher* A, const orc_cipher* B, int negate_b, orc_cipher* C);
int orc_ct_mul(const orc_params* prm, const uint64_t* H_dense, const orc_cipher* A, const orc_cipher* B,
               const uint64_t* nonces, const uint64_t* salts, orc_cipher* C);
/* capacities an output of ct_mul may need */
void orc_ct_mul_caps(const orc_params* prm, const orc_cipher* A, const orc_cipher* B, uint64_t* capL, uint64_t* capE);
void orc_commit_ct(const orc_params* prm, const uint8_t H_digest[32], const orc_cipher* C, uint8_t out[32]);
/* dec_value with caller-provided BASE-layer R values (ops/decrypt.hpp:12-89) */
void orc_dec_value(const orc_params* prm, const uint64_t* powg /*B x 2*/, const orc_cipher* C,
                   const uint64_t* R_base /* nL x 2, PROD entries ignored */, uint64_t out[2]);
/* ---- LPN PRF and encryption (crypto/lpn.hpp, ops/encrypt.hpp) ----
 * dom: 0..5 = pvac.prf.r.1..3, pvac.prf.noise.1..3. full_rows = 0 evaluates the 127 LPN rows that
 * reach toep_127's output, 1 all lpn_t rows (the reference's loop). */
void orc_prf_core(const orc_secret* sk, uint64_t canon, uint64_t ztag, uint64_t nlo, uint64_t nhi, int dom,
                  int full_rows, uint64_t out[2]);
void orc_prf_R(const orc_secret* sk, uint64_t canon, uint64_t ztag, uint64_t nlo, uint64_t nhi, int noise,
               uint64_t out[2]);
void orc_prf_noise_delta(const orc_secret* sk, uint64_t canon, uint64_t ztag, uint64_t nlo, uint64_t nhi,
                         uint32_t group, uint32_t kind, uint64_t out[2]);
/* enc_value (ops/encrypt.hpp:281-287) driven by `stream` (the csprng_u64 draws, in order). H_dense
 * NULL: weights only. order: 0 = combine_ciphers' first argument is evaluated first, 1 = second.
 * Returns 0 ok, -1 stream exhausted, -2 capacity. *consumed = draws used. */
int orc_enc_value(const orc_params* prm, const orc_secret* sk, const uint64_t* H_dense, const uint64_t* powg,
                  uint64_t v, const uint64_t* stream, size_t stream_len, int order, orc_cipher* out,
                  size_t* consumed);
/* enc_value_depth(v, depth_hint) (ops/encrypt.hpp:281-287): the noise plan of depth_hint
 * (plan_noise, encrypt.hpp:16-27); v = 0 gives enc_zero_depth (:293-298) exactly. */
/* plan_noise's Params fields (process-wide; defaults 120, 0.55, 16) */
void orc_set_noise(double noise_entropy_bits, double tuple2_fraction, double depth_slope_bits);
int orc_enc_value_depth(const orc_params* prm, const orc_secret* sk, const uint64_t* H_dense, const uint64_t* powg,
                        uint64_t v, int depth_hint, const uint64_t* stream, size_t n, int order, orc_cipher* out,
                        size_t* consumed);
/* libstdc++ bucket count after unordered_map::reserve(n) (the emit-order pin) */
uint64_t orc_bucket_count_after_reserve(uint64_t n);

/* ---- batched weights-only ct_mul over a packed batch (cpu_baseline leg) ----
 * Batch layout = engine ABI batch with dense CSR offsets; outputs per-pair edge counts and an
 * order-sensitive FNV-1a digest over all emitted (meta,w_lo,w_hi). Returns seconds. */
double orc_ct_mul_batch_timed(const orc_params* prm, uint64_t npairs,
                              const uint64_t* a_loff, const orc_layer* a_layers, const uint64_t* a_eoff,
                              const uint64_t* a_meta, const uint64_t* a_wlo, const uint64_t* a_whi,
                              const uint64_t* b_loff, const orc_layer* b_layers, const uint64_t* b_eoff,
                              const uint64_t* b_meta, const uint64_t* b_wlo, const uint64_t* b_whi,
                              int threads, uint64_t* out_counts, uint64_t* out_digests);
/* batched weights-only ct_add (negate_b = 0) / ct_sub (1) over packed pairs; per-pair edge counts
 * and FNV-1a edge digests. Returns seconds. */
double orc_ct_add_batch_timed(const orc_params* prm, uint64_t npairs, const uint64_t* a_loff, const orc_layer* a_layers,
                              const uint64_t* a_eoff, const uint64_t* a_meta, const uint64_t* a_wlo,
                              const uint64_t* a_whi, const uint64_t* b_loff, const orc_layer* b_layers,
                              const uint64_t* b_eoff, const uint64_t* b_meta, const uint64_t* b_wlo,
                              const uint64_t* b_whi, int negate_b, int threads, uint64_t* out_counts,
                              uint64_t* out_digests);
/* cfg 4: depth-`depth` chains c_k = ct_mul(c_{k-1}, x_i) per input of a packed batch (weights
 * only); final edge counts / FNV-1a edge digests per input, per-step edge totals. Returns seconds. */
double orc_ct_mul_chain_timed(const orc_params* prm, uint64_t ninputs, const uint64_t* loff, const orc_layer* layers,
                              const uint64_t* eoff, const uint64_t* meta, const uint64_t* wlo, const uint64_t* whi,
                              int depth, int threads, uint64_t* out_counts, uint64_t* out_digests,
                              uint64_t* step_edges);
/* The same with per-step operands for steps 1..nops: c_k = ct_mul(c_{k-1}, ops[(k-1) * ninputs + i])
 * (a packed batch of nops * ninputs ciphers, step-major), x_i after that. */
double orc_ct_mul_chain_ops_timed(const orc_params* prm, uint64_t ninputs, const uint64_t* loff, const orc_layer* layers,
                                  const uint64_t* eoff, const uint64_t* meta, const uint64_t* wlo, const uint64_t* whi,
                                  int depth, int nops, const uint64_t* oloff, const orc_layer* olayers,
                                  const uint64_t* oeoff, const uint64_t* ometa, const uint64_t* owlo,
                                  const uint64_t* owhi, int threads, uint64_t* out_counts, uint64_t* out_digests,
                                  uint64_t* step_edges);

#ifdef __cplusplus
}
#endif
#endif
