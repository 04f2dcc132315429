// mfma_i8_probe.hip — checks the operand / result lane maps of v_mfma_i32_32x32x32_i8 that
// k_mul_large.hip's matrix-core products rely on, with random signed bytes on both operands:
//   A (M x K): lane l holds A[m = l & 31][k = (h = l >> 5, byte j)]
//   B (K x N): lane l holds B[k = (h, j)][n = l & 31]
//   D (M x N): lane l, register i holds D[m = (i & 3) + 8 (i >> 2) + 4 (l >> 5)][n = l & 31]
// i.e. byte j of lane half h on one operand meets byte j of the same half on the other.
// Build: hipcc --offload-arch=gfx950 -O2 tools/mfma_i8_probe.hip -o tools/mfma_i8_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <random>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k_probe(const v4i* a, const v4i* b, const v16i* c, v16i* d) {
    const int l = threadIdx.x;
    d[l] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[l], b[l], c[l], 0, 0, 0);
}

int main() {
    std::mt19937 rng(7);
    int8_t A[64][16], B[64][16];
    int32_t C[64][16], D[64][16];
    for (int trial = 0; trial < 4; ++trial) {
        for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 16; ++j) {
                A[l][j] = (int8_t)(rng() & 0xFF);
                B[l][j] = (int8_t)(rng() & 0xFF);
                C[l][j] = trial == 3 ? (int32_t)(rng() % 100000) - 50000 : 0;
            }
        if (trial == 1)   // extremes: every product at its magnitude bound
            for (int l = 0; l < 64; ++l)
                for (int j = 0; j < 16; ++j) A[l][j] = B[l][j] = (int8_t)-128;
        void *da, *db, *dc, *dd;
        if (hipMalloc(&da, sizeof A) || hipMalloc(&db, sizeof B) || hipMalloc(&dc, sizeof C) || hipMalloc(&dd, sizeof D)) {
            std::printf("alloc failed\n");
            return 1;
        }
        hipMemcpy(da, A, sizeof A, hipMemcpyHostToDevice);
        hipMemcpy(db, B, sizeof B, hipMemcpyHostToDevice);
        hipMemcpy(dc, C, sizeof C, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, (const v4i*)da, (const v4i*)db, (const v16i*)dc, (v16i*)dd);
        if (hipMemcpy(D, dd, sizeof D, hipMemcpyDeviceToHost) != hipSuccess) {
            std::printf("kernel failed\n");
            return 1;
        }
        int bad = 0;
        for (int l = 0; l < 64; ++l)
            for (int i = 0; i < 16; ++i) {
                const int m = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5), n = l & 31;
                int64_t want = C[l][i];
                for (int h = 0; h < 2; ++h)
                    for (int j = 0; j < 16; ++j) want += (int64_t)A[m + 32 * h][j] * B[n + 32 * h][j];
                if (want != D[l][i]) ++bad;
            }
        std::printf("mfma_i32_32x32x32_i8 trial %d: %d of 1024 results differ from the assumed lane maps\n", trial, bad);
        hipFree(da); hipFree(db); hipFree(dc); hipFree(dd);
        if (bad) return 2;
    }
    std::printf("mfma_i8_probe: ok\n");
    return 0;
}
