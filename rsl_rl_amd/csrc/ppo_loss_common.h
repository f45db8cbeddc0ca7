// Per-sample pieces of the fused PPO loss shared by ppo_loss.hip (the loss kernels) and mlp_gemm.hip (the actor head
// that runs the loss inside its GEMM epilogue, rslrl_actor_head_fwd_bwd): constants of torch.distributions.Normal,
// torch.max's backward, the quad-lane sum and the fixed-order fold of per-block fp64 partials.
#pragma once

#include <hip/hip_runtime.h>

#include "common.h"

namespace rslrl {
namespace {

constexpr float kLogSqrt2Pi = 0.91893853320467274178f;  // log(sqrt(2*pi)), normal.py log_prob
constexpr float kEntC = 1.41893853320467274178f;         // 0.5 + 0.5*log(2*pi), normal.py entropy

// torch.max(a, b) backward (derivatives.yaml, maximum): ties give each side grad / 2.
__device__ __forceinline__ void max_grads(float a, float b, float g, float& ga, float& gb) {
    const float half = __fmul_rn(g, 0.5f);
    ga = (a > b) ? g : ((a == b) ? half : 0.0f);
    gb = (b > a) ? g : ((a == b) ? half : 0.0f);
}

constexpr int kFoldGroup = 64;

// Sum over the 4 lanes of a quad (DPP quad_perm [1,0,3,2] then [2,3,0,1]); every lane of the quad
// gets the same bits ((v0 + v1) + (v2 + v3), fp addition being commutative).
__device__ __forceinline__ float quad_sum(float v) {
    const float a = __fadd_rn(v, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1,
                                                                                      0xF, 0xF, false)));
    return __fadd_rn(a, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, a), 0x4E, 0xF,
                                                                             0xF, false)));
}

// Fixed-order fold of `n` (<= 64) partials per column (column c at src[c * ld + r]) into out[c]:
// 16 lanes per column, each adding rows l16, l16+16, l16+32, l16+48 in that order, then a 16-lane
// butterfly.  Every load is issued before the first add, so the fold costs one memory round trip.
// Loads use sc1 (bypass the non-coherent per-CU cache); the caller has acquired.
// kRows = 8 (rows l16 + 16 i, i < 8: n <= 128) for the groups of 128 blocks of a grid over 4096 blocks.
template <int kMaxC, int kRows = 4>
__device__ __forceinline__ void fold_columns(const double* __restrict__ src, int ld, int n, int ncols,
                                             double* __restrict__ out) {
    constexpr int kPasses = (kMaxC + 15) / 16;
    const int l16 = threadIdx.x & 15;
    const int cc = threadIdx.x >> 4;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<double*>(src), 0, static_cast<int>(sizeof(double) * ncols * ld), 0x00020000);
    double v[kPasses][kRows];
#pragma unroll
    for (int ps = 0; ps < kPasses; ++ps) {
        const int c = ps * 16 + cc;
#pragma unroll
        for (int i = 0; i < kRows; ++i) {
            const int r = l16 + 16 * i;
            // out-of-range offsets read 0 through the buffer resource
            const int off = (c < ncols && r < n) ? (c * ld + r) * 8 : 0x7ffffff0;
            v[ps][i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off, 0, 16 /* sc1 */));
        }
    }
#pragma unroll
    for (int ps = 0; ps < kPasses; ++ps) {
        double t = ((v[ps][0] + v[ps][1]) + v[ps][2]) + v[ps][3];
#pragma unroll
        for (int i = 4; i < kRows; ++i) t += v[ps][i];
#pragma unroll
        for (int off = 8; off >= 1; off >>= 1) t += __shfl_xor(t, off, kWave);
        const int c = ps * 16 + cc;
        if (l16 == 0 && c < ncols) out[c] = t;
    }
}

// Two-level fixed-order reduction of one fp64 value per column and block over the grid (at most kFoldGroup^2
// blocks): every block publishes `v` of column threadIdx.x (< ncols) to partials[c * nb + block]; the last
// arriving block of each group of kFoldGroup folds the group (fold_columns: the same order whatever the arrival
// order) into partials[ncols * nb + c * ng + g], and the last group to finish folds the groups into `folded` (LDS,
// ncols doubles).  Returns true only in that final block, with `folded` complete.  tickets: 1 + ng words, zero
// before the launch and re-armed to zero by it (the global word by the caller of the final block: it returns with
// tickets[0] still counting).  `flag`: an LDS int.  Called by every thread of the block.
// G: blocks per group -- kFoldGroup, or 2 kFoldGroup for grids over kFoldGroup^2 blocks (up to 8192; the groups then
// fold 8 rows per lane, fold_columns<kMaxC, 8>)
template <int kMaxC, int G = kFoldGroup>
__device__ __forceinline__ bool fold_grid_partials(double* __restrict__ partials, unsigned* __restrict__ tickets,
                                                   int nb, int ncols, double v, double* folded, int* flag) {
    constexpr int kFoldGroup = G;
    const int ng = (nb + kFoldGroup - 1) / kFoldGroup;
    if (static_cast<int>(threadIdx.x) < ncols)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(partials + static_cast<int64_t>(threadIdx.x) * nb +
                                                                 blockIdx.x),
                           __double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int g = blockIdx.x / kFoldGroup;
    const int g0 = g * kFoldGroup;
    const int gsz = min(kFoldGroup, nb - g0);
    if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(tickets + 1 + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = (t == static_cast<unsigned>(gsz) - 1);
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
    }
    __syncthreads();
    if (!*flag) return false;
    if (threadIdx.x == 0) __hip_atomic_store(tickets + 1 + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    fold_columns<kMaxC, (G > 64 ? 8 : 4)>(partials + g0, nb, gsz, ncols, folded);
    __syncthreads();
    if (ng == 1) return true;
    double* gpart = partials + static_cast<int64_t>(ncols) * nb;
    if (static_cast<int>(threadIdx.x) < ncols)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(gpart + static_cast<int64_t>(threadIdx.x) * ng + g),
                           __double_as_longlong(folded[threadIdx.x]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(tickets, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = (t == static_cast<unsigned>(ng) - 1);
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
    }
    __syncthreads();
    if (!*flag) return false;
    fold_columns<kMaxC>(gpart, ng, ng, ncols, folded);
    __syncthreads();
    return true;
}

// d(loss)/dV of one sample (ppo.py:305-313, :367 backward): the loss kernel's expression and operation order
// (ppo_loss.hip, ppo_loss_quad_kernel; both compiled with -ffp-contract=off), so both produce the same bits.
__device__ __forceinline__ float value_loss_grad(float V, float tv, float R, int clipped, float clip, float g_value) {
    if (clipped) {
        const float dv = V - tv;
        const float vc = tv + fminf(fmaxf(dv, -clip), clip);
        const float e1 = V - R;
        const float e2 = vc - R;
        const float vl = e1 * e1;
        const float vlc = e2 * e2;
        const float half = __fmul_rn(g_value, 0.5f);  // max(): ties split the gradient 1/2 : 1/2
        const float g1 = (vl > vlc) ? g_value : ((vl == vlc) ? half : 0.0f);
        const float g2 = (vlc > vl) ? g_value : ((vl == vlc) ? half : 0.0f);
        float dV = 2.0f * g1 * e1;
        if (dv >= -clip && dv <= clip) dV += 2.0f * g2 * e2;
        return dV;
    }
    const float e = R - V;
    return -2.0f * g_value * e;
}

}  // namespace
}  // namespace rslrl
