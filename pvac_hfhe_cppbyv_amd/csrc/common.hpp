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

// Workgroup-wide exclusive scan of one u32 per thread. `part` is LDS scratch of BS/64 words.
template <int BS>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* part, uint32_t& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
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
hipError_t launch_gen_fresh(uint64_t seed, uint32_t epl, uint32_t B, const pvac_ct_batch& X, hipStream_t st);
hipError_t launch_batch_digest(const pvac_ct_batch& X, uint64_t* out, hipStream_t st);
hipError_t launch_ct_scale(const pvac_ct_batch& X, uint64_t slo, uint64_t shi, hipStream_t st);

// plan statistics written by the plan kernels (device, zeroed before launch)
struct plan_stats {
    unsigned long long total_layers, total_edges;
    unsigned long long n_small, n_large, n_invalid;
    unsigned int max_keys, max_prod, max_na, max_nb, max_buckets, max_layers;
};

hipError_t launch_plan_mul(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, uint8_t* pair_class,
                           plan_stats* stats, const uint32_t* nb_table, uint32_t nb_table_len, uint32_t Bm,
                           uint32_t ks_small_max, uint32_t prod_small_max, hipStream_t st);
hipError_t launch_plan_add(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, plan_stats* stats,
                           hipStream_t st);
// in-place exclusive scan of n u64 values; scratch >= scan_scratch_words(n) u64
size_t scan_scratch_words(size_t n);
hipError_t launch_exclusive_scan_u64(uint64_t* data, size_t n, uint64_t* scratch, unsigned long long* total_out,
                                     hipStream_t st);

struct mul_small_args {
    pvac_ct_batch A, B, C;
    const uint64_t* nonces;
    uint32_t* salt_pos;          // nullable: hash-order index of each output edge (salt stream position)
    const uint8_t* pair_class;
    uint32_t* pair_status;
    const uint32_t* nb_table;
    uint64_t canon_tag;
    uint64_t edge_budget;
    uint32_t Bm;
    uint32_t flags;
    // launch sizing (maxima over the small pairs of the batch)
    uint32_t ks_max, prod_max, na_max, nb_max, buckets_max, layers_max;
};
hipError_t launch_ct_mul_small(const mul_small_args& a, int num_cus, hipStream_t st, int* blocks_used);

hipError_t launch_ct_add(const pvac_ct_batch& A, const pvac_ct_batch& B, pvac_ct_batch& C, int negate_b,
                         uint32_t max_layers, hipStream_t st);

}  // namespace pvhip
