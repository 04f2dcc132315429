// common.hpp — shared device helpers and launch declarations for libpvac_hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pvac_hip.h"
#include "fp127.hpp"

namespace pvhip {

constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ULL;   // ct_mul key hash (ops/arithmetic.hpp:73)

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t& s) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t meta_layer(uint64_t m) { return (uint32_t)m; }
__device__ __forceinline__ uint32_t meta_idx(uint64_t m) { return (uint32_t)(m >> 32) & 0xFFFFu; }
__device__ __forceinline__ uint32_t meta_ch(uint64_t m) { return (uint32_t)(m >> 48) & 0xFFu; }
__device__ __forceinline__ uint64_t make_meta(uint32_t layer, uint32_t idx, uint32_t ch) {
    return (uint64_t)layer | ((uint64_t)(idx & 0xFFFFu) << 32) | ((uint64_t)(ch & 0xFFu) << 48);
}

// Wave64 inclusive prefix sum with DPP (row_shr 1/2/4/8 inside 16-lane rows, then row_bcast
// 15/31 across rows): six VALU ops, no LDS round trips (unlike __shfl_up's ds_bpermute).
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t x) {
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
    return x;
}

// OR over the 64 lanes of a wave (same DPP network; lane 63 ends with the total), uniform result
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t x) {
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);
    return __builtin_amdgcn_readlane(x, 63);
}

__device__ __forceinline__ uint64_t wave_or_u64(uint64_t v) {
    return (uint64_t)wave_or_u32((uint32_t)v) | ((uint64_t)wave_or_u32((uint32_t)(v >> 32)) << 32);
}

// Workgroup-wide exclusive scan of one u32 per thread. `part` is LDS scratch of BS/64 words.
template <int BS>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* part, uint32_t& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t x = wave_incl_scan_u32(v);
    if (lane == 63) part[wave] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < BS / 64; ++w) {
        const uint32_t pw = part[w];
        base += (w < wave) ? pw : 0u;
        tot += pw;
    }
    total = tot;
    __syncthreads();
    return base + x - v;
}

// ---------------------------------------------------------------- launch wrappers
// (defined in the .hip translation units; all enqueue on `st` and return hipError_t)
hipError_t launch_fp_binop(int op, const uint64_t* alo, const uint64_t* ahi, const uint64_t* blo,
                           const uint64_t* bhi, uint64_t* clo, uint64_t* chi, size_t n, hipStream_t st);
hipError_t launch_fill_random(uint64_t seed, uint64_t* out, size_t n, hipStream_t st);
hipError_t launch_gen_fresh(uint64_t seed, uint64_t first, uint32_t epl, uint32_t B, const pvac_ct_batch& X,
                            hipStream_t st);
hipError_t launch_fill_nonces(uint64_t seed, uint64_t first, const pvac_ct_batch& A, const pvac_ct_batch& B,
                              const uint64_t* c_l_off, uint64_t* out, hipStream_t st);
hipError_t launch_batch_digest(const pvac_ct_batch& X, uint64_t* out, hipStream_t st);
hipError_t launch_batch_sumdigest(const pvac_ct_batch& X, uint64_t* out, hipStream_t st);
hipError_t launch_ct_scale(const pvac_ct_batch& X, uint64_t slo, uint64_t shi, hipStream_t st);

// x mod d for a runtime divisor d < 2^32 without a 64-bit division: m = floor((2^64-1)/d),
// q = mulhi(x, m) undershoots floor(x/d) by at most 2, so two conditional subtracts finish.
struct fastmod64 {
    uint64_t d, m;
};
__host__ __device__ inline fastmod64 make_fastmod64(uint64_t d) { return fastmod64{d, d ? ~0ull / d : 0}; }
__device__ __forceinline__ uint64_t fmod64(uint64_t x, const fastmod64& f) {
    const uint64_t q = __umul64hi(x, f.m);
    uint64_t r = x - q * f.d;
    r = r >= f.d ? r - f.d : r;
    r = r >= f.d ? r - f.d : r;
    return r;
}

// plan statistics written by the plan kernels (device, zeroed before launch)
struct plan_stats {
    unsigned long long total_layers, total_edges;   // the plan scans' totals (pvac_hip_ctx::totals)
    unsigned long long n_small, n_large, n_invalid;
    unsigned int max_keys, max_prod, max_na, max_nb, max_buckets, max_layers;
};

// pair classes written by the mul plan
enum : uint8_t { PAIR_EMPTY = 0, PAIR_SMALL = 1, PAIR_LARGE = 2 };

hipError_t launch_plan_mul(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, uint8_t* pair_class,
                           uint64_t* large_ids, plan_stats* stats, const uint32_t* nb_table, uint32_t nb_table_len,
                           uint32_t Bm, hipStream_t st);
hipError_t launch_gather_large(const pvac_ct_batch& A, const pvac_ct_batch& B, const uint64_t* ids, uint64_t n,
                               uint64_t* out, hipStream_t st);
hipError_t launch_plan_add(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, plan_stats* stats,
                           uint8_t* pair_class, uint64_t* merge_ids, uint64_t edge_budget, hipStream_t st);
hipError_t launch_gather_merge(const pvac_ct_batch& A, const pvac_ct_batch& B, const pvac_ct_batch& C,
                               const uint64_t* ids, uint64_t n, uint64_t* out, hipStream_t st);
// in-place exclusive scan of n u64 values (or of two arrays of n values at once: one launch per
// scan kernel); scratch >= scan_scratch_words(n) u64
size_t scan_scratch_words(size_t n);
hipError_t launch_exclusive_scan2_u64(uint64_t* d0, uint64_t* d1, size_t n, uint64_t* scratch,
                                      unsigned long long* total0, unsigned long long* total1, hipStream_t st);
hipError_t launch_exclusive_scan_u64(uint64_t* data, size_t n, uint64_t* scratch, unsigned long long* total_out,
                                     hipStream_t st);

// ---- ct_mul, fresh-shape path (k_mul_fresh.hip): LDS-resident, one workgroup per pair
constexpr uint32_t kFreshKeysMax = 1536;    // |A.L||B.L|B key slots
constexpr uint32_t kFreshProdMax = 4096;    // |A.E||B.E| products
constexpr uint32_t kFreshEdgesMax = 256;    // |A.E|, |B.E|
constexpr uint32_t kFreshLayersMax = 64;    // |C.L| before compaction

// One 64-byte header record per pair (written by k_mul_layers_fresh, read by k_ct_mul_fresh with
// a single scalar load): every per-pair field the aggregation kernel needs, in one cache line.
struct __attribute__((aligned(64))) fresh_rec {
    uint64_t aeo, beo, ceo;      // edge offsets of A, B, C
    uint64_t alo, blo, clo;      // layer offsets
    uint64_t nb_magic;           // fastmod64 multiplier of nbk
    uint32_t shape;              // nA | nB << 16   (each <= kFreshEdgesMax)
    uint16_t nbk;                // libstdc++ bucket count after reserve(nA nB); 0 = not a fresh pair
    uint8_t LA, LB;
};
static_assert(sizeof(fresh_rec) == 64, "fresh_rec is one cache line");

struct mul_fresh_args {
    pvac_ct_batch A, B, C;
    fresh_rec* recs;             // per pair, filled by k_mul_layers_fresh
    const uint64_t* nonces;
    const uint8_t* pair_class;
    uint32_t* pair_status;       // 0 = reference order, 1 = canonical order, 2 = rejected (bad refs)
    const uint32_t* nb_table;    // libstdc++ bucket count after reserve(n), n <= kFreshProdMax
    const uint64_t* nb_magic;    // fastmod64 multipliers for nb_table
    uint32_t* salt_pos;          // nullable: per output edge slot, its hash-order index
    uint64_t* redo_ids;          // pairs whose key sums cancelled to 0 mod p (re-run on the general path)
    unsigned int* redo_cnt;      // their count (device, zeroed before the launch)
    uint64_t canon_tag;
    uint64_t edge_budget;
    uint32_t Bm;
    uint32_t flags;
    // launch sizing (maxima over the small pairs of the batch)
    uint32_t ks_max, prod_max, na_max, nb_max, buckets_max, layers_max;
};
// pair_status values of ct_mul (device array): 0 reference order, 1 canonical order, 2 rejected,
// 3 = the fresh kernel found a key sum of 0 mod p and left the pair to the general path
constexpr uint32_t kPairRedo = 3;
hipError_t launch_mul_layers_fresh(const mul_fresh_args& a, hipStream_t st);
// args_dev: device copy of `a` (the kernel reads its arguments from memory, see k_mul_fresh.hip)
hipError_t launch_ct_mul_fresh(const mul_fresh_args& a, const mul_fresh_args* args_dev, int num_cus, hipStream_t st);

// ---- LPN PRF (k_prf.hip): prf_R_core / prf_R / prf_R_noise (crypto/lpn.hpp:159-275)
struct prf_consts {
    uint32_t mid[8];          // SHA-256 state after block 0 of the key derivation (prf_k, canon, H_digest[0..24))
    uint64_t hd_tail;         // H_digest[24..32) as a little-endian u64
    uint64_t dom_hash[6];     // fnv1a of pvac.prf.r.1..3, pvac.prf.noise.1..3 (lpn.hpp:150-157)
    uint64_t toep_hash;       // fnv1a("pvac.dom.toeplitz")
    const uint64_t* s_bits;   // LPN secret (device), s_words u64
    uint32_t s_words, tau_num, tau_den, pad;
};
// one prf_R_core evaluation: an RSeed and a domain index into prf_consts.dom_hash (0..5)
struct prf_request {
    uint64_t ztag, nonce_lo, nonce_hi;
    uint32_t dom;
    uint32_t pad;
};
hipError_t prf_upload_tables(hipStream_t st);
size_t prf_request_bytes();
// n core requests (see k_prf.hip prf_request) -> out[2 n]
hipError_t launch_prf_cores(const prf_consts& k, const void* req, uint64_t n, uint64_t* out, hipStream_t st);
// seeds: 3 u64 per seed {ztag, nonce_lo, nonce_hi}; kind 0..5 one core, 6 prf_R, 7 prf_R_noise.
// req_scratch: 3 n requests; core_scratch: 6 n u64 (kinds 6/7)
hipError_t launch_prf(const prf_consts& k, int kind, const uint64_t* seeds, uint64_t n, void* req_scratch,
                      uint64_t* core_scratch, uint64_t* out, hipStream_t st);
// prf_R of every BASE layer slot of X (slots < n_slots), 0 for others: R_out[2 s], [2 s + 1]
hipError_t launch_base_R(const prf_consts& k, const pvac_ct_batch& X, uint64_t n_slots, void* req_scratch,
                         uint64_t* core_scratch, uint64_t* R_out, hipStream_t st);

// ---- enc_value (k_enc.hip, ops/encrypt.hpp:114-291)
// pre-merge edges per half, 8 signal + 2 Z2 + 3 Z3: two capacity classes of the per-half plan record
// (the default plans and depth hints <= 15 fit the small one; depth hints up to 124 the large one)
constexpr uint32_t kEncPreSmall = 48;
constexpr uint32_t kEncPreMax = 256;
struct enc_plan_args {
    const uint64_t* values;   // n plaintexts
    const uint64_t* rnd;      // csprng_u64 draws: stride words per value
    uint32_t stride;
    uint32_t B, Z2, Z3;
    uint64_t n;
    uint64_t canon;
    const uint64_t* powg;     // B x (lo, hi)
};
size_t enc_half_bytes(uint32_t npre);   // per-half plan record of the capacity class npre needs
// per value: 2 output layers, <= 2 * (8 + 2 Z2 + 3 Z3) edges; cores per value = 2 * 3 * max(Z2 + Z3, 1)
uint32_t enc_cores_per_value(uint32_t Z2, uint32_t Z3);
// 1. draws (exact csprng order), merge groups, shuffle, PRF requests, and the pre-merge edge batch
//    `pre` (2 layers and 2 * npre edge slots per value; salts in pre_salt) for sigma
hipError_t launch_enc_plan(const enc_plan_args& a, void* halves, prf_request* req, pvac_ct_batch& pre,
                           uint64_t* pre_salt, uint32_t* status, hipStream_t st);
// 2. R, noise deltas and the solved coefficients -> pre-merge weights (pre.w_lo / w_hi)
hipError_t launch_enc_weights(const enc_plan_args& a, void* halves, const uint64_t* cores, pvac_ct_batch& pre,
                              hipStream_t st);
// 3. merged groups (fp_add chains, sigma XOR) in shuffled order -> C (2 layers, CSR stride 2 * npre)
hipError_t launch_enc_finish(const enc_plan_args& a, const void* halves, const pvac_ct_batch& pre, pvac_ct_batch& C,
                             uint32_t* status, hipStream_t st);

// ---- dec_value (k_dec.hip): BASE-layer R supplied, PROD R tree, inversions, signed edge sum
size_t dec_scratch_bytes(uint64_t total_layers);
hipError_t launch_dec_value(const pvac_ct_batch& X, const uint64_t* Rbase, const uint64_t* powg, uint32_t Bm,
                            const uint64_t* roff, uint64_t total_layers, void* scratch, uint64_t* out,
                            uint32_t* status, hipStream_t st);

// ---- ct_add / ct_sub over edge_budget (k_add_merge.hip): compact_edges + compact_layers per pair
struct merge_pair_info {
    uint64_t pair, aeo, beo, ceo, nA, nB;
    uint32_t LA, L;
};
size_t merge_scratch_bytes(uint64_t n_edges, uint32_t n_layers);
// counters: 2 device u64 (groups, kept edges) owned by the caller
hipError_t launch_add_merge(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, uint64_t pr,
                            const merge_pair_info& info, uint32_t Bm, int negate_b, void* scratch, size_t scratch_bytes,
                            unsigned long long* counters, hipStream_t st);

// ---- ct_mul, general path (k_mul_large.hip): multi-kernel, global scratch, one workgroup
// per (A-layer, B-layer) product task. The host prepares one descriptor per large pair with
// ABSOLUTE u32-word offsets into one scratch arena (64-bit arrays on even offsets).
constexpr uint32_t kLargeLayersMax = 16384;   // |A.L| + |B.L| + |A.L||B.L| handled in LDS
constexpr uint32_t kLargeDenseMin = 48;       // dense-owner product mode from this many edges

struct large_desc {
    uint64_t pair;               // index of the pair in the batch
    uint64_t n;                  // |A.E| * |B.E|  (< 2^32)
    uint64_t S;                  // |A.L| |B.L| B dense key slots
    uint64_t Lc;                 // |A.L| + |B.L| + |A.L||B.L|  (layers before compaction)
    uint64_t nblk;               // ceil(n / 16) first-insert-time blocks
    uint64_t capE;               // 2 min(n, S) output edge capacity
    fastmod64 nbm;               // libstdc++ bucket count after reserve(n)
    uint32_t LA, LB, nA, nB;
    uint32_t hbits;              // bucket hash table capacity = 2^hbits >= 2 S (dynamic chains only)
    // 1: emit order from per-A-edge counts (o_icnt) instead of the n/16 block marks (o_bmask): static
    // bucket groups, A-layer-major products, 1 <= |B.E| <= 63. The pair falls back to the block marks
    // (cnt[kCntIFail]) when a B layer is too big for the matrix-core mode or an A layer cannot be
    // staged as a dense table
    uint32_t iblk;
    // 1: direct mode (an iblk pair whose scratch holds no per-key sums): k_large_count_la counts the
    // emit positions from key PRESENCE before any multiply, k_large_scan_direct turns the counts into
    // offsets, and k_large_products_direct writes C's edge records at their positions from the
    // matrix-core sums staged in LDS. A pair that turns out to need more (shared buckets, the
    // canonical order, a fallback, a key whose products cancel) is left to the host's redo on the
    // full layout. Its A ids carry the dense cell (k_large_lists)
    uint32_t direct;
    uint32_t pad_d;
    uint64_t nb_m;               // floor(2^32 / |B.E|): t / |B.E| by div_small (k_mul_large.hip)
    // static bucket groups (bucket_count >= 2 S): per-slot chain head / next of the slots sharing
    // a libstdc++ bucket, word offsets into mul_large_args::grp (kNoGrp: dynamic chains via link)
    uint64_t g_head, g_next;
    // zero-initialised block [o_zero, o_zero + zero_words): cnt | hkey | hhead | bmask | bcnt | used
    uint64_t o_zero, zero_words;
    uint64_t o_cnt;              // [16] neA, neB, invalid, total edges, canonical, A / B id allocation, deferred tasks,
                                 // [kCntIFail] per-A-edge order abandoned (iblk pairs)
    uint64_t o_hkey;             // [2^hbits] u64 bucket ids + 1
    uint64_t o_hhead;            // [2^hbits] chain heads (slot + 1)
    uint64_t o_bmask;            // [nblk] u64 per 16 first-insert times: bucket-leader edge codes (2 bits
                                 // per time: 0 none, 1/2 edges, 3 more) | block edges << 32, then the
                                 // block's exclusive suffix offset << 32 (k_large_rank / scan / order)
    uint64_t o_bcnt;             // (unused, empty)
    uint64_t o_used;             // [Lc] product-layer used flags -> compact_layers remap
    // 0xFF-initialised: [S] first-insert time per key slot (INF = key absent)
    uint64_t o_tkey;
    // written before read
    uint64_t o_lstA, o_lstB;     // [2 LA] start,count per layer ++ [nA] edge ids; same for B
    uint64_t o_neA, o_neB;       // [LA] / [LB] non-empty layer lists
    uint64_t o_defer;            // [LA LB] tasks k_large_products_la leaves to k_large_products_defer
                                 // (la << 16 | lb index), counted in cnt[7]
    uint64_t o_info;             // [S] ebits (2 bits) | hash slot << 2
    uint64_t o_sums;             // [S] x 4 u64: P lo, P hi, M lo, M hi
    uint64_t o_nxt;              // [S] bucket chain links
    uint64_t o_tb;               // [S] bucket first-insert time
    uint64_t o_within;           // [S] edges of the same bucket emitted before this key
    uint64_t o_etot;             // [S] edges of the bucket (leaders only)
    uint64_t o_cpos;             // [S] canonical positions (guard_budget order)
    uint64_t o_order;            // [capE] emit order: slot << 1 | ch
    uint64_t o_hpos;             // [capE] hash-order index of each canonical-order edge
    uint64_t o_icnt;             // [nA] iblk: edges whose emit time lies in A edge i's product range
                                 // [i |B.E|, (i + 1) |B.E|), then their exclusive suffix offset
    uint64_t o_imask;            // [nA] x 2 u64 iblk: the range's keys with a P edge / an M edge (bit j
                                 // = B edge j), read by k_large_write_ranges; direct pairs: per A layer
                                 // (slice o_lstA's ids offset) the masks of its writer list
    uint64_t o_wle;              // direct pairs: [nA] writer lists, A edge | idx << 21 (k_large_count_la)
    uint64_t o_wln;              // direct pairs: [LA] writer list length per A layer
    // direct pairs: o_icnt holds one count byte per A edge (32-edge groups, 32 B each, zero padded)
    // and o_iwo [ceil(nA / 32)] each group's exclusive suffix offset (k_large_scan_direct)
    uint64_t o_iwo;
    uint64_t words;             // end of this pair's scratch (absolute)
};

struct mul_large_args {
    pvac_ct_batch A, B, C;
    const uint64_t* nonces;
    uint32_t* pair_status;
    const large_desc* desc;      // [nl]
    uint32_t* scratch;           // arena (u32 words)
    uint32_t nl;
    uint32_t Bm;
    uint64_t canon_tag;
    uint64_t edge_budget;
    uint32_t flags;
    uint32_t n_la;               // products: descriptors sel[0, n_la) take k_large_products_la, the rest
                                 // k_large_products (one workgroup per task)
    uint32_t* salt_pos;          // nullable: per output edge slot, its hash-order index
    const uint32_t* grp;         // static bucket-group tables (large_desc::g_head / g_next)
    const uint32_t* sel;         // [nl] descriptor indices, A-layer-major class first
    uint32_t lds_task;           // k_large_products_la: bytes of LDS below its staged B layers (set at launch)
    uint32_t la_per_wg;          // k_large_products_la: A layers per workgroup (max_la_wg = ceil(|A.L| / it))
    uint32_t la_xcd;             // k_large_products_la: 1 = all workgroups of a pair on one XCD (grid y padded to 8)
    uint32_t any_dyn;            // some pair has dynamic bucket chains (k_large_link runs)
    uint32_t all_iblk;           // every pair is iblk (rank / order / write on reduced grids)
    uint32_t any_direct;         // some pair is direct (large_desc::direct): the direct kernels run
    uint32_t layers_direct;      // k_large_layers: 1 = the direct pairs' pass (before their products),
                                 // 0 = every other pair (after the products)
    uint32_t all_direct;         // every pair is direct: the per-key kernels are not launched
    uint32_t dir_lb;             // k_large_products_direct: B layers its LDS holds (max |B.L| of the direct pairs)
    uint32_t pad4;
    uint64_t* redo_ids;          // pairs the host re-runs on the full layout (shared with the fresh kernel)
    unsigned int* redo_cnt;
    // chain steps (pvac_hip_ct_mul_chain): a pair whose A_img flag is set holds A as a dense image
    // (k_large_products_direct's image writer) instead of hash-order records; a direct pair of a
    // step with C_img writes C that way when it is dense, and k_large_direct_redo sets its flag
    uint32_t* A_img;             // nullable, [n pairs]
    uint32_t* C_img;             // nullable, [n pairs]
    unsigned long long* img_count;   // nullable: += 1 per pair written as an image
    // launch sizing (maxima over the nl descriptors; max_tasks over the per-task class, max_tasks_all
    // over all, max_la_wg = ceil(|A.L| / kLaPerWG) over the A-layer-major class)
    uint64_t max_S, max_zero, max_tasks, max_capE, max_lay, max_tasks_all, max_la_wg, max_nA;
};
// k_large_products_la: A layers per workgroup (default; PVAC_LA_PER_WG); pairs with at most
// kLaMaxLB B layers take it
constexpr uint32_t kLaPerWG = 8;
constexpr uint32_t kLaMaxLB = 4;
hipError_t launch_ct_mul_large(const mul_large_args& a, hipStream_t st);
// dense chain images back to hash-order records for the listed pairs whose flag is set (the flag is
// cleared): pairs = [n_pairs ids, then n_pairs offsets into tmp], tmp holds 3 words per edge of every
// listed pair (sum of their |A.E|); launches of at most y_cap pairs each (65535: the grid-y limit)
hipError_t launch_image_to_records(const pvac_ct_batch& A, uint32_t* img, const uint64_t* pairs, uint32_t n_pairs,
                                   uint64_t* tmp, uint32_t Bm, uint32_t y_cap, hipStream_t st);
// LDS of k_large_products_direct for B and nbl staged B layers (the direct mode needs it <= 160 KB)
uint32_t large_direct_lds_bytes(uint32_t Bm, uint32_t nbl);
// measured integer-ALU ceilings (k_ubench.hip)
hipError_t run_alu_probe(int kind, int num_cus, hipStream_t st, double* per_s);
hipError_t run_issue_probe(int op, int wps, int num_cus, hipStream_t st, double* per_s, double* clock_hz);
// ct_mul gsum invariant (k_check.hip, utils/metrics.hpp:70-113)
hipError_t launch_check_sizes(const pvac_ct_batch& A, const pvac_ct_batch& B, const pvac_ct_batch& C, unsigned int* mx,
                              hipStream_t st);
hipError_t launch_check_gsum(const pvac_ct_batch& A, const pvac_ct_batch& B, const pvac_ct_batch& C, const uint64_t* nonces,
                             const uint64_t* powg, uint32_t Bm, const unsigned int* mx_host, uint32_t* status,
                             unsigned long long* n_bad, int num_cus, uint8_t* gscratch, hipStream_t st);
// global scratch bytes launch_check_gsum needs when a pair's layer tables exceed LDS (0 if they fit)
uint64_t check_gsum_scratch_bytes(uint32_t Bm, const unsigned int* mx_host, uint64_t n, int num_cus);
// pvac_hip_ct_mul_chain statistics: out[0] += sum |C.E|, out[1] += sum |A.E| |X.E| (k_check.hip)
hipError_t launch_stage_rows(const pvac_ct_batch& src, const pvac_ct_batch& dst, hipStream_t st);
hipError_t launch_chain_stats(const pvac_ct_batch& A, const pvac_ct_batch& X, const pvac_ct_batch& C,
                              unsigned long long* out, hipStream_t st);
constexpr uint64_t kNoGrp = ~0ull;
constexpr uint32_t kCntWords = 16;    // large_desc::o_cnt words
constexpr uint32_t kCntIFail = 8;     // cnt word: an iblk pair uses the block marks after all
constexpr uint32_t kCntIShared = 9;   // cnt word: an iblk pair has keys sharing a bucket (order probes)
constexpr uint32_t kCntDirect = 10;   // cnt word: a direct pair's positions are final (k_large_scan_direct)
constexpr uint32_t kCntRedo = 11;     // cnt word: a direct pair was handed to the host's redo
constexpr uint32_t kCntImg = 12;      // cnt word: a direct pair writes C as a dense image (k_large_scan_direct)
constexpr uint32_t kIblkMaxNB = 63;   // iblk: |B.E| <= 63 (a 64-bit mask per A edge, bit 63 a flag)
// static bucket groups of key slots [0, S) for one bucket count: head[s] = 0 when s is alone in
// its bucket, else the first slot + 1 of the bucket's chain; next[s] = the following slot + 1
// (0 ends). tmp_key / tmp_head: 2^hbits entries, zeroed by the caller.
hipError_t launch_grp_build(fastmod64 nbm, uint32_t Bm, uint64_t S, uint32_t hbits, uint32_t* head, uint32_t* next,
                            unsigned long long* tmp_key, uint32_t* tmp_head, hipStream_t st);

hipError_t launch_ct_add(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, int negate_b,
                         uint32_t max_layers, const uint8_t* pair_class, hipStream_t st);

}  // namespace pvhip
