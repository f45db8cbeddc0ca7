// FETCH_SIZE / WRITE_SIZE calibration in the MLP kernels' own access patterns (MI355X_MICROARCH.md, HBM: only the
// 16-B-per-lane streaming read and store are calibrated in the guide; other widths must be calibrated on a known byte
// count).  Each kernel touches every byte of a 512 MiB buffer once (> the 256 MiB Infinity Cache, so the bytes come
// from HBM) in one access pattern:
//   read_v4        16 B per lane, fully coalesced stream (the guide's calibrated case: FETCH_SIZE = 1/2 the bytes)
//   read_gemm_a    the x6 GEMMs' A-operand staging (mlp_gemm.hip load_a, 256-thread w4 workgroup): a 128-row x 1 KiB
//                  tile read as 16 chunks of 64 B per row, chunk-major (16 rows x 64 B per wave instruction)
//   read_c_b32     the input-gradient epilogue's H loads (epilogue_tiles_impl, full tiles): 4 B per lane, lanes 0-31
//                  one 128-B row piece, lanes 32-63 the piece four rows down
//   write_c_b32_nt the same pattern as nontemporal 4-B stores (the forward / input-gradient outputs)
//   write_v4       16 B per lane, fully coalesced stores (the guide's calibrated WRITE_SIZE case)
// Build and run (rocprofv3 passes: scripts/mlp_pmc.sh):
//   hipcc -O3 --offload-arch=gfx950 scripts/pmc_pattern_probe.hip -o scripts/pmc_pattern_probe.bin
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int64_t kBytes = 512ll << 20;
constexpr int64_t kFloats = kBytes / 4;
constexpr int kCols = 256;  // floats per row (1 KiB rows, the hidden width)
constexpr int64_t kRows = kFloats / kCols;

__global__ __launch_bounds__(256) void read_v4(const float4* __restrict__ src, float* __restrict__ sink, int64_t n4) {
    float acc = 0.f;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n4; i += static_cast<int64_t>(gridDim.x) * 256) {
        const float4 v = src[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) sink[threadIdx.x] = acc;  // keeps the loads live
}

// one workgroup per 128-row tile: chunk c, unit u = t + 256 i (i = 0, 1): row u >> 2, k = 16 c + 4 (u & 3)
__global__ __launch_bounds__(256) void read_gemm_a(const float* __restrict__ a, float* __restrict__ sink) {
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * 128;
    float acc = 0.f;
#pragma unroll 1
    for (int c = 0; c < 16; ++c) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int u = threadIdx.x + 256 * i;
            const float4 v = *reinterpret_cast<const float4*>(a + (row0 + (u >> 2)) * kCols + 16 * c + 4 * (u & 3));
            acc += v.x + v.y + v.z + v.w;
        }
    }
    if (acc == 12345.f) sink[threadIdx.x] = acc;
}

// one workgroup of 4 waves per 128-row tile, wave w owns columns 64 w .. +63: blocks (i, j) of 32 x 32, element r of a
// block at row 32 i + 4 h + (r & 3) + 8 (r >> 2), column 32 j + l32 (the 32x32x16 MFMA C map)
__global__ __launch_bounds__(256) void read_c_b32(const float* __restrict__ hsrc, float* __restrict__ sink) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
    const float* base = hsrc + static_cast<int64_t>(blockIdx.x) * 128 * kCols + 64 * w;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc += base[(32 * i + 4 * h + (r & 3) + 8 * (r >> 2)) * kCols + 32 * j + l32];
    if (acc == 12345.f) sink[threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void write_c_b32_nt(float* __restrict__ dst) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
    float* base = dst + static_cast<int64_t>(blockIdx.x) * 128 * kCols + 64 * w;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                __builtin_nontemporal_store(static_cast<float>(r + j),
                                            base + (32 * i + 4 * h + (r & 3) + 8 * (r >> 2)) * kCols + 32 * j + l32);
}

__global__ __launch_bounds__(256) void write_v4(float4* __restrict__ dst, int64_t n4) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n4; i += static_cast<int64_t>(gridDim.x) * 256)
        dst[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

int main() {
    float *buf, *sink;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, kBytes);
    const unsigned tiles = static_cast<unsigned>(kRows / 128);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(read_v4, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const float4*>(buf), sink, kFloats / 4);
        hipLaunchKernelGGL(read_gemm_a, dim3(tiles), dim3(256), 0, 0, buf, sink);
        hipLaunchKernelGGL(read_c_b32, dim3(tiles), dim3(256), 0, 0, buf, sink);
        hipLaunchKernelGGL(write_c_b32_nt, dim3(tiles), dim3(256), 0, 0, buf);
        hipLaunchKernelGGL(write_v4, dim3(4096), dim3(256), 0, 0, reinterpret_cast<float4*>(buf), kFloats / 4);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"bytes_per_launch\": %lld, \"kernels\": [\"read_v4\", \"read_gemm_a\", \"read_c_b32\", \"write_c_b32_nt\", "
           "\"write_v4\"]}\n", static_cast<long long>(kBytes));
    return 0;
}
