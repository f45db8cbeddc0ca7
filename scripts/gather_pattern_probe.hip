// FETCH_SIZE calibration in the mini-batch gather's access patterns (csrc/gather.hip gather_records_kernel): what a
// randomly drawn row costs at the HBM, measured on known accesses instead of assumed.
//   read_rec336_perm  the first 336 bytes (21 units: the used part) of every 384-byte record of a 512 MiB buffer,
//                     records in a scattered order (i * P mod n) -- the gather's record reads
//   read_side16_perm  one 16-byte unit of every 128-byte line of a 512 MiB buffer, lines in a scattered order -- the
//                     gather's slot-array read (one unit of a line nothing else touches)
//   read_v4           the guide's calibrated stream (16 B per lane, coalesced): FETCH_SIZE KiB x 2 = bytes
// Each kernel's bytes per launch are printed; implied HBM bytes = FETCH_SIZE x 1024 x (read_v4's factor).
// Build: hipcc -O3 --offload-arch=gfx950 scripts/gather_pattern_probe.hip -o scripts/gather_pattern_probe.bin
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int64_t kBytes = 512ll << 20;
constexpr int64_t kRec = kBytes / 384;        // records of 384 B
constexpr int64_t kLines = kBytes / 128;      // 128-byte lines
constexpr int64_t kP = 1000003;               // odd prime: i -> i * kP mod n is a permutation for n not a multiple

__global__ __launch_bounds__(256) void read_v4(const float4* __restrict__ src, float* __restrict__ sink, int64_t n4) {
    float acc = 0.f;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n4; i += static_cast<int64_t>(gridDim.x) * 256) {
        const float4 v = src[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) sink[threadIdx.x] = acc;
}

// 21 units of a record per row, rows of a block consecutive in the scattered order (the gather's 4 loads in flight)
__global__ __launch_bounds__(256) void read_rec336_perm(const float4* __restrict__ rec, float* __restrict__ sink) {
    float acc = 0.f;
    const int64_t total = kRec * 21;
    for (int64_t k = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; k < total; k += static_cast<int64_t>(gridDim.x) * 256) {
        const int64_t r = k / 21, u = k - r * 21;
        const int64_t src = (r * kP) % kRec;
        const float4 v = rec[src * 24 + u];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) sink[threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void read_side16_perm(const float4* __restrict__ side, float* __restrict__ sink) {
    float acc = 0.f;
    for (int64_t k = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; k < kLines; k += static_cast<int64_t>(gridDim.x) * 256) {
        const int64_t line = (k * kP) % kLines;
        const float4 v = side[line * 8 + (k & 7)];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) sink[threadIdx.x] = acc;
}

int main() {
    float *buf, *sink;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, kBytes);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(read_v4, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const float4*>(buf), sink, kBytes / 16);
        hipLaunchKernelGGL(read_rec336_perm, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const float4*>(buf), sink);
        hipLaunchKernelGGL(read_side16_perm, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const float4*>(buf), sink);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"read_v4_bytes\": %lld, \"records\": %lld, \"record_bytes_used\": 336, \"record_stride\": 384, "
           "\"side_lines\": %lld, \"side_bytes_used\": 16}\n",
           static_cast<long long>(kBytes), static_cast<long long>(kRec), static_cast<long long>(kLines));
    return 0;
}
