// Empirical residency: 3 x 256 workgroups of 512 threads, each spinning ~2 ms; count late starters.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
__device__ unsigned long long g_t[4096];
template <int SCR>
__global__ __launch_bounds__(512, 6) void k_probe(int* out, int spin) {
    extern __shared__ int s[];
    volatile int priv[SCR > 0 ? SCR : 1];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) g_t[blockIdx.x] = t0;
    s[threadIdx.x] = threadIdx.x;
    if (SCR > 0) for (int i = 0; i < SCR; ++i) priv[i] = i * threadIdx.x;
    __syncthreads();
    int acc = 0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) acc += s[(threadIdx.x + acc) & 511];
    if (SCR > 0) acc += priv[acc & (SCR - 1)];
    if (acc == 12345) out[threadIdx.x] = acc;
}
template <int SCR>
void run(int lds, int nwg) {
    int* out;
    hipMalloc(&out, 4096);
    hipLaunchKernelGGL(k_probe<SCR>, dim3(nwg), dim3(512), lds, 0, out, 200000);   // 2 ms at 100 MHz
    hipDeviceSynchronize();
    unsigned long long t[4096];
    hipMemcpyFromSymbol(t, HIP_SYMBOL(g_t), nwg * 8);
    unsigned long long mn = ~0ull;
    for (int i = 0; i < nwg; ++i) mn = t[i] < mn ? t[i] : mn;
    int late = 0;
    for (int i = 0; i < nwg; ++i) late += (t[i] - mn) > 100000;
    int nb = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_probe<SCR>, 512, lds);
    printf("scratch %3d ints, lds %6d B: API %d/CU, %d of %d workgroups started late\n", SCR, lds, nb, late, nwg);
    hipFree(out);
}
int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int lds : {40000, 50000, 52224, 53248, 53888, 54528}) run<0>(lds, 3 * cus);
    for (int lds : {40000, 53888}) run<22>(lds, 3 * cus);
    return 0;
}
