// k_dec.hip — batched dec_value (reference ops/decrypt.hpp:12-89) given the BASE-layer R values.
//
// dec(C) = sum over edges of  +/- w * powg_B[idx] * R[layer]^-1   (+ for SGN_P, - otherwise)
// with R[BASE] = prf_R(pk, sk, seed) supplied by the caller (one per BASE layer slot) and
// R[other] = R[pa] * R[pb] (layer_R_cached: any non-BASE rule multiplies its parents). The
// reference aborts on a cycle or an out-of-range parent; here the cipher's status says so.
// Every term is canonical (fp_mul output), so the sum mod p is exact in any order: the edge
// sum is a parallel fp_add reduction and is bit-identical to the reference's sequential loop.
//
//   k_dec_layers : one block per cipher, dependency sweeps until every layer is resolved
//                  (depth of the layer DAG; parents-before-children orders need one sweep)
//   k_dec_inv    : one lane per layer slot, fp_inv (addition chain, 137 fp_mul)
//   k_dec_edges  : one block per cipher, fp_add tree of the signed terms
#include "common.hpp"

namespace pvhip {
namespace {

constexpr int kDB = 256;
constexpr uint8_t kUnres = 0, kRes = 1;

// R of every layer slot into dense scratch R[roff[c] + l] (roff = exclusive scan of l_cnt)
__global__ __launch_bounds__(kDB) void k_dec_layers(pvac_ct_batch X, const uint64_t* Rbase, const uint64_t* roff,
                                                    ulonglong2* R, uint8_t* state, uint32_t* status) {
    __shared__ uint32_t changed, bad;
    const uint64_t c = blockIdx.x;
    const uint32_t L = (uint32_t)X.l_cnt[c];
    const uint64_t lo = X.l_off[c], ro = roff[c];
    const pvac_layer* lay = X.layers + lo;
    if (threadIdx.x == 0) bad = 0;
    for (uint32_t l = threadIdx.x; l < L; l += kDB) {
        const bool base = lay[l].rule == 0;
        if (base) R[ro + l] = make_ulonglong2(Rbase[2 * (lo + l)], Rbase[2 * (lo + l) + 1]);
        state[ro + l] = base ? kRes : kUnres;
    }
    __syncthreads();
    for (uint32_t sweep = 0; sweep <= L; ++sweep) {   // every sweep resolves >= 1 layer or stops
        if (threadIdx.x == 0) changed = 0;
        __syncthreads();
        for (uint32_t l = threadIdx.x; l < L; l += kDB) {
            if (state[ro + l] != kUnres) continue;
            const uint32_t pa = lay[l].pa, pb = lay[l].pb;
            if (pa >= L || pb >= L) { bad = 1; continue; }   // decrypt.hpp:21-24 aborts
            if (state[ro + pa] == kRes && state[ro + pb] == kRes) {
                const ulonglong2 a = R[ro + pa], b = R[ro + pb];
                const fp r = fp_mul(fp{a.x, a.y}, fp{b.x, b.y});
                R[ro + l] = make_ulonglong2(r.lo, r.hi);
                __threadfence_block();
                state[ro + l] = kRes;
                changed = 1;
            }
        }
        __syncthreads();
        if (!changed || bad) break;
        __syncthreads();
    }
    __syncthreads();
    uint32_t unresolved = 0;
    for (uint32_t l = threadIdx.x; l < L; l += kDB) unresolved |= state[ro + l] == kUnres;
    if (unresolved) bad = 1;   // a cycle (decrypt.hpp:31-37 aborts) or a parent out of range
    __syncthreads();
    if (threadIdx.x == 0) status[c] = bad ? 1u : 0u;
}

__global__ __launch_bounds__(kDB) void k_dec_inv(ulonglong2* R, uint64_t total) {
    for (uint64_t s = (uint64_t)blockIdx.x * kDB + threadIdx.x; s < total; s += (uint64_t)gridDim.x * kDB) {
        const ulonglong2 v = R[s];
        const fp r = fp_inv(fp{v.x, v.y});
        R[s] = make_ulonglong2(r.lo, r.hi);
    }
}

__global__ __launch_bounds__(kDB) void k_dec_edges(pvac_ct_batch X, const ulonglong2* Rinv, const uint64_t* roff,
                                                   const ulonglong2* powg, uint32_t Bm, uint64_t* out,
                                                   uint32_t* status) {
    __shared__ ulonglong2 part[kDB / 64];
    __shared__ uint32_t bad;
    const uint64_t c = blockIdx.x;
    const uint32_t L = (uint32_t)X.l_cnt[c];
    const uint64_t eo = X.e_off[c], ne = X.e_cnt[c], ro = roff[c];
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    fp acc{0, 0};
    for (uint64_t e = threadIdx.x; e < ne; e += kDB) {
        const uint64_t m = X.meta[eo + e];
        const uint32_t lid = meta_layer(m), idx = meta_idx(m);
        if (lid >= L || idx >= Bm) { bad = 1; continue; }   // out-of-range reads in the reference
        const ulonglong2 g = powg[idx], ri = Rinv[ro + lid];
        const fp t = fp_mul(fp_mul(fp{X.w_lo[eo + e], X.w_hi[eo + e]}, fp{g.x, g.y}), fp{ri.x, ri.y});
        acc = meta_ch(m) == 0 ? fp_add(acc, t) : fp_sub(acc, t);
    }
    // wave tree, then the block's waves (fp_add of canonical values is exact)
    for (int d = 32; d >= 1; d >>= 1) {
        const fp o{(uint64_t)__shfl_xor((long long)acc.lo, d, 64), (uint64_t)__shfl_xor((long long)acc.hi, d, 64)};
        acc = fp_add(acc, o);
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x / 64] = make_ulonglong2(acc.lo, acc.hi);
    __syncthreads();
    if (threadIdx.x == 0) {
        fp s{0, 0};
        for (int w = 0; w < kDB / 64; ++w) s = fp_add(s, fp{part[w].x, part[w].y});
        out[2 * c] = s.lo;
        out[2 * c + 1] = s.hi;
        if (bad || status[c]) status[c] = bad ? 2u : status[c];
    }
}

}  // namespace

hipError_t launch_dec_value(const pvac_ct_batch& X, const uint64_t* Rbase, const uint64_t* powg, uint32_t Bm,
                            const uint64_t* roff, uint64_t total_layers, void* scratch, uint64_t* out,
                            uint32_t* status, hipStream_t st) {
    if (!X.n) return hipSuccess;
    if (X.n > 0x7FFFFFFFull) return hipErrorInvalidValue;
    ulonglong2* R = (ulonglong2*)scratch;
    uint8_t* state = (uint8_t*)(R + (total_layers ? total_layers : 1));
    hipLaunchKernelGGL(k_dec_layers, dim3((unsigned)X.n), dim3(kDB), 0, st, X, Rbase, roff, R, state, status);
    if (total_layers) {
        uint64_t blocks = (total_layers + kDB - 1) / kDB;
        if (blocks > 65536) blocks = 65536;
        hipLaunchKernelGGL(k_dec_inv, dim3((unsigned)blocks), dim3(kDB), 0, st, R, total_layers);
    }
    hipLaunchKernelGGL(k_dec_edges, dim3((unsigned)X.n), dim3(kDB), 0, st, X, (const ulonglong2*)R, roff,
                       (const ulonglong2*)powg, Bm, out, status);
    return hipGetLastError();
}

size_t dec_scratch_bytes(uint64_t total_layers) {
    const uint64_t t = total_layers ? total_layers : 1;
    return t * 16 + ((t + 15) & ~15ull);
}

}  // namespace pvhip
