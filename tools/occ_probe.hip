#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(512) void k_dummy(int* p) {
    extern __shared__ int s[];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (p) p[threadIdx.x] = s[(threadIdx.x + 1) & 511];
}
int main() {
    int prev = -1;
    for (int b = 40 * 1024; b <= 82 * 1024; b += 128) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_dummy, 512, b) != hipSuccess) { printf("err\n"); return 1; }
        if (nb != prev) { printf("lds %d B -> %d blocks/CU\n", b, nb); prev = nb; }
    }
    return 0;
}
