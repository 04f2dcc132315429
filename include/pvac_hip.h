/* pvac_hip.h — C ABI of the MI355X (gfx950) batched ciphertext-arithmetic engine.
 *
 * Drop-in boundary for the pvac-hfhe 0.1.0 hot path (reference: include/pvac/...). The
 * reference exposes a header-only, by-value C++ API and no FFI; every entry point below
 * names the reference function it replaces. The C++ adapter include/pvac_hip.hpp is
 * templated on the reference's own pvac::Cipher / PubKey types (it does not restate them) and
 * routes batched calls through these entry points; INTEGRATION.md §2 is the patch a
 * maintainer adds to the reference's ops/arithmetic.hpp to dispatch ct_mul & co. through it.
 *
 * Conventions
 *  - All functions are noexcept, never throw, and return int status: 0 = ok, <0 = error
 *    (PVAC_E*); pvac_hip_last_error(ctx) gives a message.
 *  - Pointers inside batches/arrays are DEVICE pointers (hipMalloc / torch CUDA tensors)
 *    unless a parameter says "host". Work is enqueued on the ctx stream; functions that
 *    must return sizes to the host synchronise that stream (documented per function).
 *  - One thread per ctx. Contexts are independent (one per device / per host thread).
 *  - Fp values are p = 2^127-1 field elements as two u64 limbs (lo, hi) in SoA arrays.
 *  - Randomness is an explicit input: the reference draws nonces/salts from getrandom(2)
 *    inside ct_mul (core/random.hpp:40-110); here the caller passes those words, which
 *    makes outputs reproducible and testable. The C++ adapter fills them from getrandom.
 */
#ifndef PVAC_HIP_H
#define PVAC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PVAC_HIP_ABI_VERSION 3

/* status codes */
#define PVAC_OK 0
#define PVAC_EINVAL (-22)
#define PVAC_ENOMEM (-12)
#define PVAC_ENOSYS (-38)
#define PVAC_EDEVICE (-5)
#define PVAC_ERANGE (-34)

/* fp binop codes (core/field.hpp:50-71,209-213; ops/arithmetic.hpp:33-37 for SCALE) */
#define PVAC_FP_ADD 0
#define PVAC_FP_SUB 1
#define PVAC_FP_MUL 2
#define PVAC_FP_NEG 3   /* b ignored */
#define PVAC_FP_SCALE 4 /* b is ONE element, broadcast: c[i] = a[i] * b[0] */
#define PVAC_FP_INV 5   /* fp_inv (field.hpp:229-273) = a^(p-2), inv(0) = 0; b ignored */

/* ct_mul flags */
#define PVAC_MUL_WITH_SIGMA 0x1u      /* also generate per-edge sigma (crypto/matrix.hpp:267-303) */
#define PVAC_MUL_ORDER_CANONICAL 0x2u /* emit (layer, idx, P<M) sorted instead of the reference hash order */

typedef struct pvac_hip_ctx pvac_hip_ctx;

/* Mirrors the subset of pvac::Params + PubKey that the hot path reads
 * (core/types.hpp:36-70, 121-129). */
typedef struct pvac_hip_params {
    uint32_t B;          /* 337 */
    uint32_t m_bits;     /* 8192: sigma bits */
    uint32_t n_bits;     /* 16384: H columns */
    uint32_t h_col_wt;   /* 192 */
    uint32_t x_col_wt;   /* 128 */
    uint32_t err_wt;     /* 128 */
    uint64_t edge_budget;/* 1200000 (guard_budget, ops/encrypt.hpp:106-111) */
    uint64_t canon_tag;  /* pk.canon_tag */
} pvac_hip_params;

/* pvac::Layer (core/types.hpp:96-101) as a 40-byte record. rule: 0 = BASE, 1 = PROD. */
typedef struct pvac_layer {
    uint32_t rule, pa, pb, pad;
    uint64_t ztag, nonce_lo, nonce_hi;
} pvac_layer;

/* A batch of n ciphers (pvac::Cipher, core/types.hpp:116-119), SoA with per-cipher
 * (offset, count) ranges so both dense CSR and capacity-padded outputs are expressible.
 * Edge meta packs pvac::Edge{layer_id, idx, ch} exactly like the .ct edge header:
 *   meta = layer_id | (u64)idx << 32 | (u64)ch << 48.
 * sigma (nullable) holds sigma_words u64 per edge slot (edge slot e -> sigma[e*sigma_words]). */
typedef struct pvac_ct_batch {
    uint64_t n;
    uint64_t* l_off;   /* [n] first layer slot of cipher i */
    uint64_t* l_cnt;   /* [n] layers of cipher i */
    pvac_layer* layers;
    uint64_t* e_off;   /* [n] first edge slot of cipher i */
    uint64_t* e_cnt;   /* [n] edges of cipher i */
    uint64_t* meta;
    uint64_t* w_lo;
    uint64_t* w_hi;
    uint64_t* sigma;
    uint32_t sigma_words;
    uint32_t pad;
} pvac_ct_batch;

/* Output sizing of a batched ct_mul / ct_add (filled by the *_plan calls). */
typedef struct pvac_hip_plan {
    uint64_t total_layer_slots;   /* sum of per-pair layer capacities */
    uint64_t total_edge_slots;    /* sum of per-pair edge capacities */
    uint64_t n_pairs;
    uint64_t n_small;             /* pairs served by the LDS-resident fresh-shape kernel */
    uint64_t n_large;             /* pairs served by the layer-dense path */
    uint64_t n_invalid;           /* reserved, always 0: rejections are per pair, see pvac_hip_ct_mul_status */
    uint32_t max_keys, max_prod, max_na, max_nb, max_buckets, max_layers;  /* launch sizing */
    uint32_t kind;                /* 1 = mul, 2 = add, 3 = sub */
    uint32_t reserved[5];
} pvac_hip_plan;

/* ---------------------------------------------------------------- context */
int pvac_hip_abi_version(void);
/* Create a context on `device`. Replaces the implicit PubKey plumbing of the reference. */
int pvac_hip_ctx_create(int device, const pvac_hip_params* prm, pvac_hip_ctx** out);
int pvac_hip_ctx_destroy(pvac_hip_ctx* ctx);
/* Run on the caller's stream (e.g. torch.cuda.current_stream().cuda_stream); NULL = the legacy
 * null stream. A fresh context starts on a private non-blocking stream of its own. */
int pvac_hip_ctx_set_stream(pvac_hip_ctx* ctx, void* hip_stream);
void* pvac_hip_ctx_stream(pvac_hip_ctx* ctx);
int pvac_hip_ctx_synchronize(pvac_hip_ctx* ctx);
/* The noise fields of the reference's Params (core/types.hpp:48-50: noise_entropy_bits 120,
 * tuple2_fraction 0.55, depth_slope_bits 16 by default), used by enc_value / enc_value_depth's
 * plan_noise (ops/encrypt.hpp:16-27). A plan above 256 pre-merge edges per half is PVAC_ENOSYS. */
int pvac_hip_ctx_set_noise(pvac_hip_ctx* ctx, double noise_entropy_bits, double tuple2_fraction, double depth_slope_bits);
const char* pvac_hip_last_error(pvac_hip_ctx* ctx);
/* Upload the public parity matrix H (pk.H, crypto/matrix.hpp:191-251) from a HOST dense
 * array of n_bits columns x ceil(m_bits/64) words; stored on device as per-column sparse
 * row lists. Required only for PVAC_MUL_WITH_SIGMA / pvac_hip_sigma_batch. Synchronous. */
int pvac_hip_ctx_set_H(pvac_hip_ctx* ctx, const uint64_t* H_dense_host, uint32_t n_cols, uint32_t words_per_col);
/* Regenerate H on the device from params.canon_tag (gen_H, crypto/matrix.hpp:191-251) and
 * return its H_digest (host, 32 bytes). */
int pvac_hip_ctx_gen_H(pvac_hip_ctx* ctx, uint8_t digest_out[32]);

/* Measured integer-ALU ceilings of this device for the roofline report (k_ubench.hip), per second:
 * kind 0 = wave64 integer VALU instructions (v_mad_u64_u32 / v_add_co_u32 / v_alignbit_b32 mix),
 * 1 = lazy fp_mul_fold1 products, 2 = full fp_mul products, 3 = column-accumulated products
 * (col26_mac, the general path's dense loop), 4 = wave64 single-pass 32-bit VALU instructions
 * (v_add_u32 / v_xor_b32 / v_alignbit_b32: the issue ceiling of a mostly 32-bit VALU stream),
 * 5 = general-path dense-mode products on the matrix cores (v_mfma_i32_32x32x32_i8 rate x 64).
 * Synchronous. */
int pvac_hip_alu_ceiling(pvac_hip_ctx* ctx, int kind, double* per_s);
/* Per-opcode VALU issue probe (k_ubench.hip): one opcode alone on 16 independent accumulators per
 * lane, waves_per_simd (1..8) waves on every SIMD. Returns wave64 instructions per second chip-wide
 * and the shader clock the SIMDs ran at during the same launch (s_memtime ticks per s_memrealtime
 * tick x 100 MHz, median over workgroups), so cycles per instruction = SIMDs x clock / per_s.
 * op: 0 v_add_u32, 1 v_xor_b32, 2 v_alignbit_b32, 3 v_lshlrev_b32, 4 v_min_u32, 5 v_add3_u32,
 * 6 v_pk_add_u16, 7 v_fma_f32, 8 v_mul_lo_u32, 9 v_mul_hi_u32, 10 v_cndmask_b32, 11 v_bfe_u32,
 * 12 v_add_co_u32, 13 v_and_or_b32, 14 v_pk_min_u16, 15 v_bitop3_b32, 16 v_mad_u64_u32,
 * 17 v_cndmask_b32_e64 (SGPR-pair mask), 18 v_lshl_add_u32, 19 v_mov_b32 DPP row_shr, 20 v_perm_b32,
 * 21 v_mul_u32_u24, 22 v_sub_u32, 23 v_max3_u32, 24 v_cmp (VCC) + VOP2 v_cndmask_b32 pairs, 25 v_cndmask_b32_e64
 * reading VCC, 26 VOP2 v_addc_co_u32 (VCC carry), 27 v_addc_co_u32_e64 (SGPR carry), 28 v_cmp_e64 + v_cndmask_b32_e64
 * (SGPR mask) pairs, 29 v_min_u32_e64, 30 v_add_u32_e64, 31 v_and_b32, 32 v_or_b32, 33 v_lshrrev_b32,
 * 34 v_mov_b32, 35 v_max_u32, 36 v_add_u32_sdwa (byte source), 37 / 38 v_lshlrev_b32_sdwa (byte shifted / byte
 * shift count), 39 v_xor_b32_e64, 40 v_mad_u32_u24.
 * Measurement only (never used by an op). Synchronous. */
int pvac_hip_issue_probe(pvac_hip_ctx* ctx, int op, int waves_per_simd, double* per_s, double* clock_hz);
/* Per-kernel device timing (HIP events on the ctx stream) for the roofline report. */
int pvac_hip_timing_enable(pvac_hip_ctx* ctx, int on);
/* kernel_name: "fp_binop", "ct_mul_small", "ct_mul_large", "ct_add", "sigma", ... ; returns
 * accumulated milliseconds and launch count since the last reset (synchronises). */
int pvac_hip_timing_get(pvac_hip_ctx* ctx, const char* kernel_name, double* ms, uint64_t* launches);
int pvac_hip_timing_reset(pvac_hip_ctx* ctx);

/* ---------------------------------------------------------------- element-wise Fp
 * Replaces fp_add / fp_sub / fp_mul / fp_neg (core/field.hpp:50-71, 209-213) applied over
 * arrays; results are bit-identical to the reference including its quirks for non-canonical
 * inputs (fp_add truncates the high-word carry, field.hpp:53-55). In-place (c == a) allowed. */
int pvac_hip_fp_binop(pvac_hip_ctx* ctx, int op, const uint64_t* a_lo, const uint64_t* a_hi, const uint64_t* b_lo,
                      const uint64_t* b_hi, uint64_t* c_lo, uint64_t* c_hi, size_t n);

/* ---------------------------------------------------------------- batched ciphertext ops
 * ct_mul (ops/arithmetic.hpp:47-106) over n independent pairs C[i] = A[i] * B[i].
 * Two-phase sizing:
 *   1. pvac_hip_ct_mul_plan: writes C->l_off / C->e_off (device) with per-pair capacities
 *      (layers |A.L|+|B.L|+|A.L||B.L|, edges 2*min(|A.E||B.E|, |A.L||B.L|B)), zeroes C->l_cnt /
 *      C->e_cnt when given, and fills *plan (synchronises the stream once to read totals back).
 *   2. caller allocates C->layers (total_layer_slots), C->meta/w_lo/w_hi (total_edge_slots),
 *      optional C->sigma, then pvac_hip_ct_mul_exec writes C->l_cnt/e_cnt and the records.
 * Randomness (replaces the getrandom draws of arithmetic.hpp:59-70,90-94):
 *   nonces: 2 words per OUTPUT layer slot (device, parallel to C->layers): for the product
 *           layer of (la, lb) at slot l_off+|A.L|+|B.L|+la*|B.L|+lb, words [2s]=lo, [2s+1]=hi.
 *   salts : 1 word per OUTPUT edge slot (device, parallel to C->meta), in emit order; used only
 *           with PVAC_MUL_WITH_SIGMA (nullable otherwise).
 * Output edge order is the reference's std::unordered_map iteration order (bit-exact), unless
 * PVAC_MUL_ORDER_CANONICAL. guard_budget/compact_layers semantics are applied per pair.
 * exec synchronises the stream once at its end: a fresh-shape pair with a key sum of 0 mod p
 * (cancelling products, zero weights) is re-run on the general path before it returns. */
int pvac_hip_ct_mul_plan(pvac_hip_ctx* ctx, const pvac_ct_batch* A, const pvac_ct_batch* B, pvac_ct_batch* C,
                         pvac_hip_plan* plan);
int pvac_hip_ct_mul_exec(pvac_hip_ctx* ctx, const pvac_hip_plan* plan, const pvac_ct_batch* A, const pvac_ct_batch* B,
                         const uint64_t* nonces, const uint64_t* salts, pvac_ct_batch* C, uint32_t flags);
/* plan + exec in one call, into output arrays the caller sized once (for a stream of batches of
 * one shape, no host round trip between the two): C->l_off / e_off / l_cnt / e_cnt hold A->n,
 * C->layers layer_cap slots, C->meta / w_lo / w_hi (and C->sigma) edge_cap slots. When this plan
 * needs more, nothing is launched after it and the call returns PVAC_ENOMEM with *plan (nullable)
 * holding the sizes to allocate (the plan has rewritten C's offset and count arrays by then; C's
 * rows are untouched). nonces / salts as for pvac_hip_ct_mul_exec (the nonce slots are
 * C's planned layer slots, so they are valid only while the plan's offsets are: batches of one
 * shape plan the same offsets). */
int pvac_hip_ct_mul(pvac_hip_ctx* ctx, const pvac_ct_batch* A, const pvac_ct_batch* B, pvac_ct_batch* C,
                    uint64_t layer_cap, uint64_t edge_cap, const uint64_t* nonces, const uint64_t* salts,
                    uint32_t flags, pvac_hip_plan* plan);
/* Pairs that ct_mul_exec re-ran on the general path (see above) since the context was created. */
int pvac_hip_ct_mul_redo_count(pvac_hip_ctx* ctx, uint64_t* out);
/* Pair launches by path since the context was created (diagnostics and tests): out[0] the
 * LDS-resident fresh-shape kernel, out[1] the general path (redo launches included), out[2] of
 * those the per-A-edge emit order, out[3] the direct mode (positions from key presence). */
int pvac_hip_ct_mul_path_count(pvac_hip_ctx* ctx, uint64_t* out);
/* Per-pair outcome of the last ct_mul_exec, copied (stream-ordered) to the DEVICE array out[n]:
 * 0 = reference hash order, 1 = canonical (layer, idx, P<M) order (guard_budget or
 * PVAC_MUL_ORDER_CANONICAL), 2 = rejected. Rejection is stricter than the reference: an edge with
 * layer_id >= |X.L| (undefined behaviour there: C.L[lid] out of range), idx >= B or ch > 1
 * (defined there, out of the Cipher contract: dec_value indexes powg_B[idx]) makes the pair's
 * output empty (l_cnt = e_cnt = 0) instead. */
int pvac_hip_ct_mul_status(pvac_hip_ctx* ctx, uint32_t* out, size_t n);
/* The reference's ct_mul invariant check_mul_gsum_all (utils/metrics.hpp:88-113) on every pair of
 * a batch: gsum(C, product layer of (la, lb)) == gsum(A, la) * gsum(B, lb) with
 * gsum(X, l) = sum of +/- w * powg_B[idx] over X's edges in layer l (metrics.hpp:70-86). C is a
 * ct_mul_exec output of (A, B) with `nonces`: a product layer is identified by the nonce it
 * carries (compact_layers renumbers C's layers); a dropped product layer must have a zero product.
 * Needs pvac_hip_ctx_set_powg. status (nullable, DEVICE, n u32): 0 holds, 1 violated, 2 an edge
 * idx >= B, 3 a cipher of more than 2^21 edges (not checked). *n_bad (host) = pairs with status != 0.
 * Synchronous. */
int pvac_hip_check_mul_gsum(pvac_hip_ctx* ctx, const pvac_ct_batch* A, const pvac_ct_batch* B, const pvac_ct_batch* C,
                            const uint64_t* nonces, uint32_t* status, uint64_t* n_bad);

/* ---------------------------------------------------------------- depth chains
 * c_0 = X[i], c_k = ct_mul(c_{k-1}, X[i]) for k = 1..depth, for every input i of X: the reference's
 * chain workload (tests/test_main.cpp:289-295, c = ct_mul(pk, c, x) in a loop) over a batch of
 * independent inputs. The library cuts X into chunks of `chunk` inputs and runs them on `streams`
 * worker threads, each with its own HIP stream, scratch arena and output buffers (child contexts
 * kept by ctx between calls), chunks handed out in input order. One chunk's host planning (the
 * plan's shape read-back) and its short dependent launches overlap other chunks' kernels, so a
 * single caller thread gets the concurrency. Synchronous: returns when every chunk is done.
 * Memory: each worker holds two output batches sized for its chunk's largest step (24 B per edge
 * slot; a depth-8 chain of enc_value inputs ends near 345 K edges, ~8.3 MB) plus a scratch arena
 * of at most half the free HBM over streams (an output array that does not fit takes the worker's
 * arena back first); streams x chunk beyond the device's HBM fails with PVAC_ENOMEM ("alloc edges"). A call whose (streams, n_devices, chunk) differ from the previous
 * call's first releases the workers' buffers and arenas.
 * Each step is exactly pvac_hip_ct_mul_plan + pvac_hip_ct_mul_exec (weights only, reference hash
 * order unless flags has PVAC_MUL_ORDER_CANONICAL). With PVAC_MUL_WITH_SIGMA the FINAL step also
 * gets its sigmas (sigma_from_H per output edge, arithmetic.hpp:90-94; the context needs H): the
 * reference draws one salt per emitted edge at every step, but only c_depth's sigmas survive (an
 * output sigma depends on its layer seed, idx, ch and salt alone), so intermediate steps stay
 * weights-only and a caller replaying a reference stream skips their salts (after_step gives the
 * counts). The final chunk buffer then holds 1 KiB of sigma per edge: size `chunk` for it.
 * Nonces: fill_nonces(user, step, first_input, n_words, dev_words, stream) when given (called on
 * the worker thread; fill n_words device words on `stream`, the 2-words-per-output-layer-slot
 * array of pvac_hip_ct_mul_exec), else splitmix64 words: pvac_hip_fill_random with seed
 * nonce_seed + 97 * first_input + step (step counted from 0).
 * Outputs are streamed: on_chunk(user, first_input, C, stream) receives each chunk's final
 * c_depth (device batch, capacity-padded CSR) valid until it returns; digest_out (DEVICE, nullable)
 * receives pvac_hip_batch_digest of c_depth for inputs [0, digest_n) (FNV-1a: serial over a cipher's
 * edges, ~0.2 s for a chunk of depth-8 chains), count_out (DEVICE, nullable) |E| of c_depth for
 * inputs [0, count_n).
 * PVAC_CHAIN_CHECK_GSUM runs the reference's gsum invariant (pvac_hip_check_mul_gsum) on every pair
 * of every step (needs pvac_hip_ctx_set_powg). A callback's nonzero return stops the chain with
 * PVAC_EINVAL.
 * Step hooks (all optional, called on the worker thread with the worker's stream; A = c_{step},
 * X = the chunk's inputs, C = c_{step+1}, all device batches valid during the call):
 *   (with per-step operands, below, X is the step's operand)
 *   nonces_at  before step `step`'s exec: fill dev_words[0, n_words) (2 words per layer slot of C,
 *              product layer (la, lb) of pair i at C.l_off[i] + |A_i.L| + |X_i.L| + la |X_i.L| + lb,
 *              lo then hi). Replaces fill_nonces.
 *   after_step after step `step`'s exec (C's weights, counts and layers are final; dev_words null).
 *   salts_at   WITH_SIGMA, final step, after its weights: fill dev_words[0, n_words) (n_words = C's
 *              edge slots): dev_words[C.e_off[i] + k] is the salt of pair i's k-th emitted edge in
 *              the reference's emit order (hash order; a pair in the canonical order still takes its
 *              salts in hash order, as pvac_hip_ct_mul_exec does).
 * Intermediate layout: without an after_step hook or the gsum check, a step from the third on whose
 * C is dense (every cell of every product layer present, under 2^21 edges) hands C to the next step
 * as a dense image instead of hash-order records: C's counts, offsets and layer records are final,
 * but edge slot s of pair i holds the weight of cell s mod 2B of its s / 2B-th product layer, and
 * 32-bit word s of the pair's meta region holds that edge's hash-order position | cell << 21
 * (stats.image_steps counts such pair-steps). The
 * next step reads it in place (no per-layer edge gathers); a pair that leaves the direct mode gets
 * its records back first. So nonces_at / salts_at may see A in that layout: read its counts and
 * layers only. c_depth (on_chunk, digests) is always records.
 * Devices: with n_devices > 0 the inputs are split into n_devices contiguous ranges of whole chunks
 * (by global input index; a range never splits a chunk, so every chunk, its nonce seeds and its
 * results are those of a one-device run) and each range runs on `streams` worker threads on
 * devices[j] (an ordinal may repeat). A worker whose device is not X's (or every worker of a range
 * j > 0 with PVAC_CHAIN_STAGE_INPUTS) first copies its chunk's inputs into worker-local buffers
 * (peer reads over xGMI when the devices differ); digests and counts are written to the caller's
 * arrays on X's device. ctx keeps the worker contexts of every device between calls. */
#define PVAC_CHAIN_CHECK_GSUM 0x100u
#define PVAC_CHAIN_STAGE_INPUTS 0x200u   /* ranges j > 0 stage their chunks even on X's device (tests) */
#define PVAC_CHAIN_IMG_BATCH2 0x400u     /* image -> records conversions in launches of 2 pairs (tests) */
#define PVAC_CHAIN_MAX_DEVICES 64
typedef int (*pvac_chain_step_fn)(void* user, uint32_t step, uint64_t first_input, const pvac_ct_batch* A,
                                  const pvac_ct_batch* X, const pvac_ct_batch* C, uint64_t* dev_words,
                                  uint64_t n_words, void* stream);
#define PVAC_CHAIN_MAX_DEPTH 32
typedef struct pvac_chain_opts {
    uint32_t depth;        /* 1 .. PVAC_CHAIN_MAX_DEPTH */
    uint32_t streams;      /* worker streams, 0 = 4 */
    uint64_t chunk;        /* inputs per chunk, 0 = 1024 */
    uint64_t nonce_seed;
    uint32_t flags;        /* PVAC_MUL_ORDER_CANONICAL | PVAC_MUL_WITH_SIGMA | PVAC_CHAIN_CHECK_GSUM |
                              PVAC_CHAIN_STAGE_INPUTS */
    uint32_t pad;
    uint64_t digest_n;     /* leading inputs whose final digests are written */
    uint64_t* digest_out;  /* DEVICE [digest_n], nullable */
    uint64_t count_n;      /* leading inputs whose final edge counts are written */
    uint64_t* count_out;   /* DEVICE [count_n], nullable */
    int (*fill_nonces)(void* user, uint32_t step, uint64_t first_input, uint64_t n_words, uint64_t* dev_words,
                       void* stream);
    int (*on_chunk)(void* user, uint64_t first_input, const pvac_ct_batch* C, void* stream);
    void* user;
    pvac_chain_step_fn nonces_at;    /* step hooks (above), nullable */
    pvac_chain_step_fn after_step;
    pvac_chain_step_fn salts_at;
    const int* devices;              /* HOST [n_devices] GPU ordinals; null / 0 = ctx's device */
    uint32_t n_devices;              /* 0 .. PVAC_CHAIN_MAX_DEVICES */
    uint32_t pad2;
    uint64_t* sumdigest_out;         /* DEVICE [sumdigest_n], nullable: pvac_hip_batch_sumdigest of c_depth */
    uint64_t sumdigest_n;            /* leading inputs whose sum digests are written (reads their whole c_depth) */
    /* Per-step operands (nullable): HOST [n_operands] batch descriptors of DEVICE arrays on X's device,
     * each of X->n ciphers. Step d (from 0) computes c_{d+1} = ct_mul(c_d, operands[d]) for d <
     * n_operands and ct_mul(c_d, x) after that, so the reference's own loop
     *   chain = enc_value(pk, sk, 2); for i in 1..N-1: chain = ct_mul(pk, chain, enc_value(pk, sk, 2))
     * (tests/test_main.cpp:289-293) is X = the first encryptions and operands = the later ones. The
     * step hooks' X argument is the step's operand. n_operands <= depth. */
    const pvac_ct_batch* operands;
    uint32_t n_operands;
    uint32_t pad3;
} pvac_chain_opts;
typedef struct pvac_chain_stats {
    uint64_t pair_steps;                        /* inputs x depth */
    uint64_t edges[PVAC_CHAIN_MAX_DEPTH];       /* sum over inputs of |c_k.E|, step k = index + 1 */
    uint64_t products[PVAC_CHAIN_MAX_DEPTH];    /* sum over inputs of |c_{k-1}.E| |x.E| */
    uint64_t gsum_pairs;                        /* pair-steps checked (PVAC_CHAIN_CHECK_GSUM) */
    uint64_t gsum_failed;                       /* pair-steps whose invariant failed */
    uint64_t redo;                              /* pairs re-run on the general path (ct_mul_exec) */
    uint64_t chunks;
    double seconds;                             /* wall time of the call */
    uint64_t image_steps;                       /* pair-steps whose C went to the next step as a dense
                                                   image (intermediate steps, no after_step hook or
                                                   gsum check): the layout the next step reads back */
} pvac_chain_stats;
int pvac_hip_ct_mul_chain(pvac_hip_ctx* ctx, const pvac_ct_batch* X, const pvac_chain_opts* opts,
                          pvac_chain_stats* stats);
/* Copy `bytes` between any host / device pointers (hipMemcpyDefault) ordered on `stream` (a chain
 * hook's stream, or null for the legacy stream) and wait for it: lets an FFI caller (ctypes, cgo, JNI)
 * that does not link the HIP runtime read a hook's batch view or fill its words. */
int pvac_hip_memcpy(void* dst, const void* src, size_t bytes, void* stream);
/* First input of range j of n_inputs inputs split over `parts` device ranges of whole chunks (the
 * split pvac_hip_ct_mul_chain uses): first[j] for j = 0 .. parts (first[parts] = n_inputs). */
int pvac_hip_chain_partition(uint64_t n_inputs, uint64_t chunk, uint32_t parts, uint64_t* first);

/* ct_add / ct_sub (ops/arithmetic.hpp:12-31, 43-45; combine_ciphers ops/encrypt.hpp:260-279).
 * negate_b != 0 gives ct_sub (B's weights scaled by p-1). Dense CSR output: the plan writes
 * C->l_off/e_off as exclusive scans of |A.L|+|B.L| and |A.E|+|B.E|. Sigmas are carried when
 * A, B and C all have sigma != NULL. */
int pvac_hip_ct_add_plan(pvac_hip_ctx* ctx, const pvac_ct_batch* A, const pvac_ct_batch* B, pvac_ct_batch* C,
                         pvac_hip_plan* plan);
int pvac_hip_ct_add_exec(pvac_hip_ctx* ctx, const pvac_hip_plan* plan, const pvac_ct_batch* A, const pvac_ct_batch* B,
                         int negate_b, pvac_ct_batch* C);

/* ct_scale / ct_neg (ops/arithmetic.hpp:33-41): in-place w <- w * s over every edge of the
 * batch (s host scalar). */
int pvac_hip_ct_scale(pvac_hip_ctx* ctx, pvac_ct_batch* X, uint64_t s_lo, uint64_t s_hi);

/* sigma_from_H for every edge of a batch (crypto/matrix.hpp:267-303): sigma of edge slot e
 * from its layer's (ztag, nonce), idx, ch and salts[e]. Requires H (set_H / gen_H). */
int pvac_hip_sigma_batch(pvac_hip_ctx* ctx, pvac_ct_batch* X, const uint64_t* salts);

/* ---------------------------------------------------------------- synthetic inputs / checks
 * Fresh-shaped cipher generator used by bench.py (SURVEY §8(d) cfg 3 generator): per cipher
 * 2 BASE layers (random ztag/nonce), per layer `edges_per_layer` distinct (idx, ch), uniform
 * nonzero canonical weights, edges grouped by layer and Fisher-Yates shuffled within a layer.
 * Writes a dense CSR batch whose arrays the caller allocated for n*2 layers, n*2*epl edges. */
int pvac_hip_gen_fresh_batch(pvac_hip_ctx* ctx, uint64_t seed, uint32_t edges_per_layer, pvac_ct_batch* X);
/* Same generator keyed by GLOBAL cipher index first_index + i, so a shard reproduces the
 * corresponding slice of a single-GPU batch (multi-GPU acceptance: N-GPU output == 1-GPU). */
int pvac_hip_gen_fresh_batch_at(pvac_hip_ctx* ctx, uint64_t seed, uint64_t first_index, uint32_t edges_per_layer,
                                pvac_ct_batch* X);
/* Product-layer nonces for a planned ct_mul (C->l_off from pvac_hip_ct_mul_plan), keyed by
 * (seed, GLOBAL pair index first_index + i, product layer): replaces make_nonce128's draws
 * (core/types.hpp:77-79) for synthetic, shard-invariant batches. out: 2 words per C layer slot. */
int pvac_hip_fill_nonces(pvac_hip_ctx* ctx, uint64_t seed, uint64_t first_index, const pvac_ct_batch* A,
                         const pvac_ct_batch* B, const pvac_ct_batch* C, uint64_t* out);
/* splitmix64 stream fill (device): out[i] = splitmix64(seed + (i+1)*golden). */
int pvac_hip_fill_random(pvac_hip_ctx* ctx, uint64_t seed, uint64_t* out, size_t n);
/* Host-only: the bucket count std::unordered_map::reserve(n) picks on this libstdc++ (the
 * emit-order pin of ct_mul, ops/arithmetic.hpp:75-76). No device access. */
uint64_t pvac_hip_bucket_count(uint64_t n);
/* per-cipher FNV-1a digest over (meta, w_lo, w_hi) of its edges in order (device out[n]). */
int pvac_hip_batch_digest(pvac_hip_ctx* ctx, const pvac_ct_batch* X, uint64_t* out);
/* per-cipher position-keyed digest (device out[n]): |E| + sum over edges e of
 * m(m(m(e * 0x9E3779B97F4A7C15 ^ meta) ^ w_lo) ^ w_hi) mod 2^64, m = the splitmix64 finaliser.
 * Order-sensitive, computed in parallel (one workgroup per cipher). */
int pvac_hip_batch_sumdigest(pvac_hip_ctx* ctx, const pvac_ct_batch* X, uint64_t* out);
/* The used rows of a capacity-padded batch (a plan's output, every pair at its capacity) packed
 * back to back into dst, e.g. before copying a result to the host. dst (DEVICE arrays): counts =
 * src's, offsets = their exclusive scans, rows and, when dst->sigma is set (src must carry sigma of
 * the same sigma_words), sigma rows; dst->n is set. dst's row arrays must hold the packed rows (src's
 * row capacity always does). totals (HOST [2]) = packed layer and edge counts. No reference
 * counterpart: the reference's Ciphers are std::vectors of exact size (core/types.hpp:95-98). */
int pvac_hip_batch_pack(pvac_hip_ctx* ctx, const pvac_ct_batch* src, pvac_ct_batch* dst, uint64_t* totals);

/* ---------------------------------------------------------------- LPN PRF
 * SecKey (core/types.hpp:134-137): prf_k and the LPN secret (ceil(lpn_n/64) words, host) with
 * pk.prm's lpn_t and noise rate tau_num/tau_den. The PRF also needs pk.H_digest: it is taken
 * from gen_H / set_H, or given with set_H_digest. */
int pvac_hip_ctx_set_secret(pvac_hip_ctx* ctx, const uint64_t prf_k[4], const uint64_t* lpn_s_host, uint32_t lpn_n,
                            uint32_t lpn_t, uint32_t tau_num, uint32_t tau_den);
int pvac_hip_ctx_set_H_digest(pvac_hip_ctx* ctx, const uint8_t digest[32]);
/* prf over n seeds (device, 3 words per seed: {ztag, nonce_lo, nonce_hi} = pvac::RSeed):
 * kind 0..5 = prf_R_core with domain pvac.prf.r.1..3 / pvac.prf.noise.1..3 (crypto/lpn.hpp:188-261),
 * 6 = prf_R (:263-268), 7 = prf_R_noise (:270-275). out: device, 2 words (lo, hi) per seed. */
int pvac_hip_prf(pvac_hip_ctx* ctx, int kind, size_t n, const uint64_t* seeds, uint64_t* out);

/* ---------------------------------------------------------------- encryption
 * enc_value (ops/encrypt.hpp:281-287) over n plaintexts (device u64). The reference draws every
 * random choice from getrandom (csprng_u64); here value i's draws are rnd[i * rnd_stride ...], in
 * the reference's order (mask, then enc_fp_depth(-mask), then enc_fp_depth(v + mask)): with the
 * draws the reference consumed, the output is byte-identical. C: 2 layers and edges_per_value
 * edge slots per value (pvac_hip_enc_caps), l_off/l_cnt/e_off/e_cnt written by the call
 * (capacity-padded CSR). status: device u32 per value: 0 ok; 1 rnd_stride draws were not enough;
 * 2 a merged edge group cancelled exactly (probability ~1/p; not reproduced). Needs set_secret,
 * the H digest, set_powg, and H for PVAC_ENC_WITH_SIGMA. */
#define PVAC_ENC_WITH_SIGMA 0x1u
int pvac_hip_enc_caps(pvac_hip_ctx* ctx, uint32_t* layers_per_value, uint32_t* edges_per_value, uint32_t* draws_hint);
int pvac_hip_enc_value(pvac_hip_ctx* ctx, size_t n, const uint64_t* values, const uint64_t* rnd, uint32_t rnd_stride,
                       pvac_ct_batch* C, uint32_t flags, uint32_t* status);
/* enc_value_depth(pk, sk, v, depth_hint) (ops/encrypt.hpp:281-287): as pvac_hip_enc_value with the
 * noise plan of depth_hint (plan_noise, encrypt.hpp:16-27: more Z2 / Z3 groups as the hint grows;
 * supported while 8 + 2 Z2 + 3 Z3 <= 256, i.e. depth_hint <= 124 with the default Params, else
 * PVAC_ENOSYS; the Params noise fields from pvac_hip_ctx_set_noise). values[i] = 0 gives
 * enc_zero_depth(pk, sk, depth_hint) (encrypt.hpp:293-298) byte for byte: fp_add(0, mask) is mask and
 * the draws are the same. Size outputs and rnd_stride with
 * pvac_hip_enc_caps_depth. */
int pvac_hip_enc_caps_depth(pvac_hip_ctx* ctx, int depth_hint, uint32_t* layers_per_value, uint32_t* edges_per_value,
                            uint32_t* draws_hint);
int pvac_hip_enc_value_depth(pvac_hip_ctx* ctx, size_t n, const uint64_t* values, const uint64_t* rnd, uint32_t rnd_stride,
                             int depth_hint, pvac_ct_batch* C, uint32_t flags, uint32_t* status);
/* prf_R of every BASE layer of X (ops/decrypt.hpp:44-46): R_out device, 2 words per layer SLOT
 * (slots addressed by l_off/l_cnt; PROD slots get 0) — the R_base input of pvac_hip_dec_value. */
int pvac_hip_base_R(pvac_hip_ctx* ctx, const pvac_ct_batch* X, uint64_t* R_out);

/* ---------------------------------------------------------------- decryption
 * dec_value (ops/decrypt.hpp:12-89) over a batch, given the BASE-layer R values (prf_R of each
 * BASE layer's seed under the secret key, crypto/lpn.hpp): R of every other layer is the product
 * of its parents' (layer_R_cached), inverses are fp_inv (field.hpp:229-273), and
 * dec = sum(+/- w * powg_B[idx] * R[layer]^-1), + for SGN_P. Bit-identical to the reference.
 * set_powg: pk.powg_B as `count` >= B (lo, hi) pairs in HOST memory.
 * R_base: device, 2 words per layer SLOT of X (parallel to X->layers; read for BASE layers only).
 * out: device, 2 words (lo, hi) per cipher. status: device u32 per cipher: 0 ok; 1 the layer
 * graph has a cycle or an out-of-range parent (the reference aborts); 2 an edge references a
 * layer or idx out of range (out-of-bounds reads in the reference). out is undefined unless 0. */
int pvac_hip_ctx_set_powg(pvac_hip_ctx* ctx, const uint64_t* powg_host, uint32_t count);
int pvac_hip_dec_value(pvac_hip_ctx* ctx, const pvac_ct_batch* X, const uint64_t* R_base, uint64_t* out,
                       uint32_t* status);

/* ---------------------------------------------------------------- .ct codec (host memory)
 * The reference's ciphertext file format (tests/add.cpp:22-155: saveCts / loadCts, putLayer,
 * putEdge) <-> SoA batches in HOST memory; no context or device needed (copy to the device with
 * hipMemcpy, or parse straight into pinned buffers). PROD layers carry no seed on disk, so parsed
 * PROD layers have ztag = nonce = 0. Every edge of a file must carry the same sigma nbits. */
#define PVAC_CT_MIXED_SIGMA 0x1u   /* pvac_ct_file_info.flags: edges disagree on sigma nbits */
typedef struct pvac_ct_file_info {
    uint64_t n_ciphers, total_layers, total_edges;
    uint32_t sigma_bits;    /* nbits of every edge's sigma (0: the file carries no sigmas) */
    uint32_t sigma_words;   /* ceil(sigma_bits / 64) */
    uint32_t flags;
    uint32_t pad;
} pvac_ct_file_info;
/* Validate a file image and size it (PVAC_EINVAL on a malformed or truncated image). */
int pvac_ct_scan(const uint8_t* buf, size_t len, pvac_ct_file_info* info);
/* Decode into X (host arrays sized from pvac_ct_scan; X->n = n_ciphers; X->sigma nullable, else
 * X->sigma_words >= info.sigma_words). Writes dense CSR l_off/l_cnt/e_off/e_cnt. threads <= 0:
 * one per hardware thread. PVAC_ENOSYS if edges disagree on sigma nbits. */
int pvac_ct_parse(const uint8_t* buf, size_t len, pvac_ct_batch* X, int threads);
/* Bytes pvac_ct_write produces for X; sigma_bits is written per edge when X->sigma != NULL
 * (the reference writes m_bits = 8192), 0 otherwise. */
int pvac_ct_serialized_size(const pvac_ct_batch* X, uint32_t sigma_bits, uint64_t* bytes);
int pvac_ct_write(const pvac_ct_batch* X, uint32_t sigma_bits, uint8_t* out, size_t capacity, uint64_t* written,
                  int threads);

#ifdef __cplusplus
}
#endif
#endif /* PVAC_HIP_H */
