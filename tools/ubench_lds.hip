// ubench_lds.hip — standalone microbenchmarks of the primitives the fresh ct_mul kernel is built
// from (tooling only; not part of the library). Each kernel runs a fixed number of rounds per
// wave over an LDS array and reports cycles per wave-instruction from s_memtime.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_lds tools/ubench_lds.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int ROUNDS = 256;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

// mode: 0 ds_add_u64 random, 1 ds_min_u32 random, 2 ds_wrxchg_rtn_b32 random, 3 ds_add_rtn_u32 random,
//       4 ds_add_u64 x3 contiguous-slot (48B stride) random, 5 ds_write_b128 contiguous, 6 ds_read_b128 random
template <int MODE>
__global__ __launch_bounds__(512) void k_lds(uint64_t* out, uint32_t slots, uint32_t seed) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint64_t* a64 = (uint64_t*)lds;
    uint32_t* a32 = (uint32_t*)lds;
    for (uint32_t i = threadIdx.x; i < slots * 6; i += blockDim.x) a64[i] = 0;
    __syncthreads();
    uint32_t addr[8];
    for (int k = 0; k < 8; ++k) addr[k] = mix(seed ^ (threadIdx.x * 8 + k) ^ (blockIdx.x << 20)) % slots;
    uint32_t sink = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < ROUNDS; ++r) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t s = addr[k] ^ (uint32_t)(r & 1);
            if (MODE == 0) atomicAdd((unsigned long long*)&a64[s], 1ull);
            if (MODE == 1) atomicMin(&a32[s], (uint32_t)(r * 8 + k));
            if (MODE == 2) sink += atomicExch(&a32[s], (uint32_t)r);
            if (MODE == 3) sink += atomicAdd(&a32[s], 1u);
            if (MODE == 4) {
                unsigned long long* q = (unsigned long long*)&a64[(s % (slots / 6 * 2)) * 3];
                atomicAdd(q + 0, 1ull); atomicAdd(q + 1, 2ull); atomicAdd(q + 2, 3ull);
            }
            if (MODE == 5) ((uint4*)lds)[(threadIdx.x + k * 512) % (slots * 3)] = make_uint4(r, k, r, k);
            if (MODE == 6) { uint4 v = ((uint4*)lds)[s % (slots * 3)]; sink += v.x + v.w; }
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (threadIdx.x % 64 == 0) out[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
    if (sink == 0x12345678u) out[0] = 0;
}

// 64x64 -> 128 multiply chains (4 independent chains per lane)
__global__ __launch_bounds__(512) void k_mad(uint64_t* out, uint64_t seed) {
    uint64_t x[4], y[4];
    for (int k = 0; k < 4; ++k) { x[k] = seed * (threadIdx.x + 1) + k; y[k] = seed ^ (k * 0x9E3779B97F4A7C15ull); }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < ROUNDS; ++r) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t lo = x[k] * y[k];
            const uint64_t hi = __umul64hi(x[k], y[k]);
            x[k] = lo ^ hi;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x % 64 == 0) out[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
    if ((x[0] ^ x[1] ^ x[2] ^ x[3]) == 0x1234) out[0] = 1;
}

template <class F>
static double run(const char* name, F launch, int blocks, uint64_t* d, double ops_per_wave) {
    launch();
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> h(blocks * 8);
    hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    double s = 0; for (auto v : h) s += (double)v;
    s /= h.size();
    printf("%-34s blocks=%4d  cyc/wave-instr=%7.2f  (wall %.3f ms)\n", name, blocks, s / ops_per_wave, ms);
    return s;
}

int main() {
    uint64_t* d; CK(hipMalloc(&d, 4096 * 8 * 8));
    const uint32_t slots = 1344;   // ~ the cfg3 key-slot count
    const size_t lds = slots * 48;
    for (int blocks : {256, 512}) {
        run("ds_add_u64 random", [&] { k_lds<0><<<blocks, 512, lds>>>(d, slots, 7); }, blocks, d, ROUNDS * 8);
        run("ds_min_u32 random", [&] { k_lds<1><<<blocks, 512, lds>>>(d, slots, 7); }, blocks, d, ROUNDS * 8);
        run("ds_wrxchg_rtn_b32 random", [&] { k_lds<2><<<blocks, 512, lds>>>(d, slots, 7); }, blocks, d, ROUNDS * 8);
        run("ds_add_rtn_u32 random", [&] { k_lds<3><<<blocks, 512, lds>>>(d, slots, 7); }, blocks, d, ROUNDS * 8);
        run("3x ds_add_u64 48B slot (per triple)", [&] { k_lds<4><<<blocks, 512, lds>>>(d, slots, 7); }, blocks, d, ROUNDS * 8);
        run("ds_write_b128 contiguous", [&] { k_lds<5><<<blocks, 512, lds>>>(d, slots, 7); }, blocks, d, ROUNDS * 8);
        run("ds_read_b128 random", [&] { k_lds<6><<<blocks, 512, lds>>>(d, slots, 7); }, blocks, d, ROUNDS * 8);
        run("u64 mul lo+hi (per mul)", [&] { k_mad<<<blocks, 512>>>(d, 0x1234567ull); }, blocks, d, ROUNDS * 4);
    }
    return 0;
}
