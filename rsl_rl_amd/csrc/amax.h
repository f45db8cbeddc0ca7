// Max |x| of a launch's output, published for an h3 consumer (mlp_gemm.hip, mlp_bwd.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace rslrl {

// max |C| of a launch, without same-address contention: the workgroup's max (waves through LDS) goes to
// one of kAmaxGroups group words (atomic max; non-negative floats order as their bits); the last workgroup
// of each group (group ticket) forwards the group max to the global word, and the last group (global ticket)
// publishes it to *out.  Every word is re-armed to zero by its last reader.  ws layout (u32):
// [0, 64) group max, [64, 128) group tickets, 128 global max, 129 global ticket.
// Ordering without fences: all of these are device-scope atomics (performed at the coherence point, not in
// the per-XCD L2s) and each is waited for (vmcnt(0)) before the next one issues, so a ticket increment is
// never visible before the max it follows.  An agent-scope release fence here would write back the L2 of
// every XCD per workgroup (+150-200 us per launch measured).  Every thread of the workgroup (THREADS, a
// 1-D grid) calls this; out == nullptr (uniform) does nothing.
constexpr int kAmaxGroups = 64;

template <int THREADS>
__device__ __forceinline__ void amax_publish(float* out, unsigned* ws, float amx) {
    if (!out) return;  // uniform
    __shared__ float wave_max[THREADS / 64];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) amx = fmaxf(amx, __shfl_xor(amx, off, 64));
    if ((threadIdx.x & 63) == 0) wave_max[threadIdx.x >> 6] = amx;
    __syncthreads();
    if (threadIdx.x != 0) return;
    float m = wave_max[0];
#pragma unroll
    for (int w = 1; w < THREADS / 64; ++w) m = fmaxf(m, wave_max[w]);
    const unsigned nb = gridDim.x;
    const unsigned g = blockIdx.x % kAmaxGroups;
    const unsigned ng = nb < kAmaxGroups ? nb : kAmaxGroups;
    const unsigned in_group = (nb - g + kAmaxGroups - 1) / kAmaxGroups;
    auto amax_ = [](unsigned* a, unsigned v) {
        __hip_atomic_fetch_max(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    auto ticket_ = [](unsigned* a) {
        return __hip_atomic_fetch_add(a, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // returns: waited
    };
    auto load_ = [](unsigned* a) { return __hip_atomic_fetch_add(a, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    auto clear_ = [](unsigned* a) { __hip_atomic_exchange(a, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    amax_(ws + g, __float_as_uint(m));
    if (ticket_(ws + kAmaxGroups + g) != in_group - 1) return;
    const unsigned mg = load_(ws + g);
    clear_(ws + g);
    clear_(ws + kAmaxGroups + g);
    amax_(ws + 2 * kAmaxGroups, mg);
    if (ticket_(ws + 2 * kAmaxGroups + 1) != ng - 1) return;
    const unsigned mall = load_(ws + 2 * kAmaxGroups);
    *out = __uint_as_float(mall);
    clear_(ws + 2 * kAmaxGroups);
    clear_(ws + 2 * kAmaxGroups + 1);
}

}  // namespace rslrl
