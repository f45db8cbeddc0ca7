// Write M x 256 fp32 (M = 393216, 402 MB) from registers in two patterns, 512-thread workgroups of 128
// rows: (a) the 32x32 MFMA C/D layout the GEMM epilogue uses (dword stores, 2 x 128 B rows per wave-
// instruction), (b) row-contiguous float4 stores (each wave-instruction 1 KB of one row).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(512) void store_mfma_layout(float* out, int N, float seed) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave >> 2, wn = wave & 3, h = lane >> 5, l32 = lane & 31;
    const long row0 = (long)blockIdx.x * 128;
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) {
            const int col = wn * 64 + j * 32 + l32;
            const long rbase = row0 + wm * 64 + i * 32 + 4 * h;
            float* cp = out + rbase * N + col;
#pragma unroll
            for (int r = 0; r < 16; ++r) cp[(long)((r & 3) + 8 * (r >> 2)) * N] = seed + r;
        }
}

__global__ __launch_bounds__(512) void store_rows_f4(float* out, int N, float seed) {
    const long base = (long)blockIdx.x * 128 * N;  // 128 rows x 256 floats = 8192 float4
    float4* o = reinterpret_cast<float4*>(out + base);
#pragma unroll
    for (int i = 0; i < 16; ++i) o[threadIdx.x + 512 * i] = make_float4(seed, seed + i, seed, seed);
}

int main() {
    const int M = 393216, N = 256;
    float* out;
    hipMalloc(&out, (size_t)M * N * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int k = 0; k < 2; ++k) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            for (int it = 0; it < 20; ++it) {
                if (k == 0) hipLaunchKernelGGL(store_mfma_layout, dim3(M / 128), dim3(512), 0, 0, out, N, 1.f);
                else hipLaunchKernelGGL(store_rows_f4, dim3(M / 128), dim3(512), 0, 0, out, N, 1.f);
            }
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("%s: %.1f us  %.2f TB/s\n", k == 0 ? "mfma-layout dword" : "row float4       ", ms / 20 * 1e3,
                   (double)M * N * 4 / (ms / 20 * 1e-3) / 1e12);
        }
    }
    return 0;
}
