// Shared device helpers for librslrl_amd.so (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rslrl_amd.h"

namespace rslrl {

constexpr int kWave = 64;     // CDNA wavefront width (never 32)
constexpr int kBlock = 256;   // 4 waves: one per SIMD of a CU

inline int launch_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? RSLRL_OK : static_cast<int>(e);
}

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Wave-level sum (64 lanes) with a fixed butterfly order -> identical result in every lane.
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

// Block-level sum of kBlock threads; fixed order (wave butterfly, then waves 0..3 in order).
// `scratch` needs kBlock / kWave elements.  Result valid in thread 0 (returned to all threads).
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
    v = wave_sum(v);
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    __syncthreads();
    if (lane == 0) scratch[wid] = v;
    __syncthreads();
    T r = scratch[0];
#pragma unroll
    for (int w = 1; w < kBlock / kWave; ++w) r += scratch[w];
    return r;
}

}  // namespace rslrl
