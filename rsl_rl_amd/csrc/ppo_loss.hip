// Fused PPO loss forward + backward on gfx950.
//
// Replaces, for one mini-batch, rsl_rl/algorithms/ppo.py:221-223 (optional per-mini-batch advantage
// normalisation), :259-269 (KL for the adaptive learning rate), :297-302 (clipped surrogate), :305-313
// (clipped value loss), :315 (total loss) and the autograd backward of :368 down to the policy outputs
// (mu, sigma, V), including the torch.distributions.Normal log_prob/entropy of actor_critic.py:106-171.
// The reference evaluates this as ~40 forward + ~40 backward ATen kernels over [B, A] / [B] tensors.
//
// One lane per sample: it reads the sample's mu/sigma/action/old_mu/old_sigma rows (16-byte loads when
// A % 4 == 0) and its five scalars once, computes log-prob, entropy, KL, ratio, both clipped terms and
// their exact autograd gradients (torch.max ties split 1/2 : 1/2; clamp passes the gradient on the
// closed interval), writes d/dmu, d/dV (and d/dsigma per row when sigma is per-row), and folds its
// loss terms -- plus d/dsigma for a shared [A] sigma -- into fp64 per-block partials.  A one-block
// finalize kernel folds the partials in fixed order into the scalars and the shared-sigma gradient.
// Bytes per sample (sigma shared): read 4A (mu) + 4A (actions) + 8A (old mu, sigma) + 20 (old_logp,
// adv, target V, returns, V), write 4A (d mu) + 4 (d V) = 20A + 24.

#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "common.h"
#include "ppo_loss_common.h"
#include "launch_timing.h"

namespace rslrl {
namespace {

constexpr int kMaxBlocks = 512;  // a lane handles ~3 samples at C3; the last block folds <= 512 partials

struct LossParams {
    int64_t B;
    int32_t A;
    int32_t sigma_mode;
    const float* mu;
    int64_t mu_stride;
    const float* sigma;
    int64_t sigma_stride;
    const float* values;
    const float* actions;
    const float* old_logp;
    const float* adv;
    const float* target_values;
    const float* returns;
    const float* old_mu;
    const float* old_sigma;
    float clip;
    float ratio_lo;  // (float)(1 - clip_param)
    float ratio_hi;  // (float)(1 + clip_param)
    float g_surr;    // 1 / B                 (MeanBackward of surrogate_loss)
    float g_value;   // value_loss_coef / B   (MulBackward then MeanBackward)
    float g_ent;     // -entropy_coef / B
    int32_t clipped_value;
    int32_t compute_kl;
    int32_t normalize_adv;
    float* grad_mu;
    int64_t grad_mu_stride;
    float* grad_sigma;
    int64_t grad_sigma_stride;
    float* grad_values;
    int64_t gv_stride;  // grad_values row stride (elements)
    const float* adv_stats;  // [2] = (mean, std) when normalize_adv
    float* stats;
    int32_t kl_fast;  // shared-sigma KL on per-action constants (quad kernel); 0: full expression everywhere
};

template <int MAXA, bool VEC>
__device__ __forceinline__ void load_row(const float* __restrict__ p, int A, float (&r)[MAXA]) {
    if constexpr (VEC) {
#pragma unroll
        for (int a = 0; a < MAXA; a += 4) {
            if (a < A) {
                const float4 v = *reinterpret_cast<const float4*>(p + a);
                r[a] = v.x;
                r[a + 1] = v.y;
                r[a + 2] = v.z;
                r[a + 3] = v.w;
            }
        }
    } else {
#pragma unroll
        for (int a = 0; a < MAXA; ++a)
            if (a < A) r[a] = p[a];
    }
}

template <int MAXA, bool VEC>
__device__ __forceinline__ void store_row(float* __restrict__ p, int A, const float (&r)[MAXA]) {
    if constexpr (VEC) {
#pragma unroll
        for (int a = 0; a < MAXA; a += 4)
            if (a < A) *reinterpret_cast<float4*>(p + a) = make_float4(r[a], r[a + 1], r[a + 2], r[a + 3]);
    } else {
#pragma unroll
        for (int a = 0; a < MAXA; ++a)
            if (a < A) p[a] = r[a];
    }
}


// Loss-term columns of the per-block partials; shared-sigma gradient columns follow.
enum { kColSurr = 0, kColValue, kColEnt, kColKl, kNumScalarCols };

// One lane per sample.  SHARED: sigma is the policy's [A] vector -> its log, reciprocals and the
// entropy are per-action constants computed once per lane; otherwise sigma is read per row.
// log-prob and the gradients use those reciprocals (<= 2 ulp from the reference's divisions, inside the
// 1e-5 tolerance); the KL keeps the reference's exact fp32 operation sequence (true divisions, logf)
// because near a zero KL its terms cancel to ~1e-5 and any reordering would show up relative to it.
// EXACT: A == MAXA, so every `a < A` guard folds away at compile time (runtime-A guards split the
// row loads into branchy basic blocks that serialise on their waits).
template <int MAXA, bool VEC, bool SHARED, bool EXACT>
__global__ __launch_bounds__(kBlock) void ppo_loss_kernel(LossParams p, double* __restrict__ partials,
                                                          unsigned* __restrict__ ticket, float value_loss_coef,
                                                          float entropy_coef) {
    constexpr int kMaxCols = kNumScalarCols + MAXA;
    __shared__ double wave_part[kBlock / kWave][kMaxCols];
    __shared__ int last_block;
    const int A = EXACT ? MAXA : p.A;
    const int ncols = kNumScalarCols + (SHARED ? A : 0);

    // per-action constants of a shared sigma: computed once per block by the first A lanes, then
    // broadcast from LDS into every lane's registers
    float c_s[MAXA], c_ls[MAXA], c_inv_den[MAXA], c_inv_s[MAXA], c_inv_s3[MAXA];
    float ent_shared = 0.0f;
    if constexpr (SHARED) {
        __shared__ float k_const[5][MAXA];
        if (threadIdx.x < A) {
            const float s = p.sigma[threadIdx.x];
            const float inv_s = 1.0f / s;
            k_const[0][threadIdx.x] = s;
            k_const[1][threadIdx.x] = logf(s);
            k_const[2][threadIdx.x] = 1.0f / __fmul_rn(2.0f, __fmul_rn(s, s));
            k_const[3][threadIdx.x] = inv_s;
            k_const[4][threadIdx.x] = inv_s * inv_s * inv_s;
        }
        __syncthreads();
#pragma unroll
        for (int a = 0; a < MAXA; ++a) {
            if (a < A) {
                c_s[a] = k_const[0][a];
                c_ls[a] = k_const[1][a];
                c_inv_den[a] = k_const[2][a];
                c_inv_s[a] = k_const[3][a];
                c_inv_s3[a] = k_const[4][a];
                ent_shared = __fadd_rn(ent_shared, __fadd_rn(kEntC, c_ls[a]));
            }
        }
    }
    float adv_mean = 0.0f, adv_den = 1.0f;
    if (p.normalize_adv) {
        adv_mean = p.adv_stats[0];
        adv_den = __fadd_rn(p.adv_stats[1], 1e-8f);  // ppo.py:223  (std + 1e-8)
    }

    // per-lane sums stay fp32 (a lane sees a few samples); cross-lane / cross-block folds are fp64
    float acc[kMaxCols];
#pragma unroll
    for (int c = 0; c < kMaxCols; ++c) acc[c] = 0.0f;

    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < p.B; i += stride) {
        float mu[MAXA], sg[MAXA], x[MAXA], omu[MAXA], osg[MAXA];
        load_row<MAXA, VEC>(p.mu + i * p.mu_stride, A, mu);
        if constexpr (!SHARED) load_row<MAXA, VEC>(p.sigma + i * p.sigma_stride, A, sg);
        load_row<MAXA, VEC>(p.actions + i * A, A, x);
        if (p.compute_kl) {
            load_row<MAXA, VEC>(p.old_mu + i * A, A, omu);
            load_row<MAXA, VEC>(p.old_sigma + i * A, A, osg);
        }
        const float old_logp = p.old_logp[i];
        float adv = p.adv[i];
        const float V = p.values[i];
        const float tv = p.target_values[i];
        const float R = p.returns[i];
        if (p.normalize_adv) adv = __fdiv_rn(__fsub_rn(adv, adv_mean), adv_den);

        // Normal(mu, sigma).log_prob(x).sum(-1), entropy().sum(-1), KL (normal.py; ppo.py:262-268)
        float logp = 0.0f, ent = SHARED ? ent_shared : 0.0f, kl = 0.0f;
#pragma unroll
        for (int a = 0; a < MAXA; ++a) {
            if (a < A) {
                float s, ls, inv_den;
                if constexpr (SHARED) {
                    s = c_s[a];
                    ls = c_ls[a];
                    inv_den = c_inv_den[a];
                } else {
                    s = sg[a];
                    ls = logf(s);
                    inv_den = 1.0f / (2.0f * s * s);
                    ent += kEntC + ls;
                }
                const float d = x[a] - mu[a];
                logp += (-(d * d) * inv_den - ls) - kLogSqrt2Pi;
                if (p.compute_kl) {
                    const float os = osg[a];
                    const float dm = __fsub_rn(omu[a], mu[a]);
                    const float t1 = logf(__fadd_rn(__fdiv_rn(s, os), 1.0e-5f));
                    const float t2 = __fdiv_rn(__fadd_rn(__fmul_rn(os, os), __fmul_rn(dm, dm)),
                                               __fmul_rn(2.0f, __fmul_rn(s, s)));
                    kl = __fadd_rn(kl, __fsub_rn(__fadd_rn(t1, t2), 0.5f));
                }
            }
        }

        // surrogate (ppo.py:297-302)
        const float ratio = expf(logp - old_logp);
        const float nadv = -adv;
        const float surr = nadv * ratio;
        const float rc = fminf(fmaxf(ratio, p.ratio_lo), p.ratio_hi);
        const float surr_c = nadv * rc;
        float g_s, g_sc;
        max_grads(surr, surr_c, p.g_surr, g_s, g_sc);
        const bool in_clip = (ratio >= p.ratio_lo) && (ratio <= p.ratio_hi);
        const float g_ratio = g_s * nadv + (in_clip ? g_sc * nadv : 0.0f);
        const float g_logp = g_ratio * ratio;

        // value loss (ppo.py:305-313)
        float vterm, dV;
        if (p.clipped_value) {
            const float dv = V - tv;
            const float vc = tv + fminf(fmaxf(dv, -p.clip), p.clip);
            const float e1 = V - R;
            const float e2 = vc - R;
            const float vl = e1 * e1;
            const float vlc = e2 * e2;
            vterm = fmaxf(vl, vlc);
            float g1, g2;
            max_grads(vl, vlc, p.g_value, g1, g2);
            dV = 2.0f * g1 * e1;
            if (dv >= -p.clip && dv <= p.clip) dV += 2.0f * g2 * e2;
        } else {
            const float e = R - V;
            vterm = e * e;
            dV = -2.0f * p.g_value * e;
        }
        p.grad_values[i * p.gv_stride] = dV;

        // d/dmu = g_logp (x - mu) / sigma^2;  d/dsigma = g_logp ((x - mu)^2 / sigma^3 - 1 / sigma) + g_ent / sigma
        float gmu[MAXA], gsg[MAXA];
        const float g2 = 2.0f * g_logp;
#pragma unroll
        for (int a = 0; a < MAXA; ++a) {
            if (a < A) {
                float inv_den, inv_s, inv_s3;
                if constexpr (SHARED) {
                    inv_den = c_inv_den[a];
                    inv_s = c_inv_s[a];
                    inv_s3 = c_inv_s3[a];
                } else {
                    const float s = sg[a];
                    inv_s = 1.0f / s;
                    inv_den = 0.5f * inv_s * inv_s;
                    inv_s3 = inv_s * inv_s * inv_s;
                }
                const float d = x[a] - mu[a];
                gmu[a] = g2 * d * inv_den;
                gsg[a] = g_logp * (d * d * inv_s3 - inv_s) + p.g_ent * inv_s;
            }
        }
        store_row<MAXA, VEC>(p.grad_mu + i * p.grad_mu_stride, A, gmu);
        if constexpr (SHARED) {
#pragma unroll
            for (int a = 0; a < MAXA; ++a)
                if (a < A) acc[kNumScalarCols + a] += gsg[a];
        } else {
            store_row<MAXA, VEC>(p.grad_sigma + i * p.grad_sigma_stride, A, gsg);
        }
        acc[kColSurr] += fmaxf(surr, surr_c);
        acc[kColValue] += vterm;
        acc[kColEnt] += ent;
        acc[kColKl] += kl;
    }

    // ---- per-block partials (column-major [ncols][gridDim.x]): wave butterfly per column, then waves in order
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
#pragma unroll
    for (int c = 0; c < kMaxCols; ++c) {
        if (c < ncols) {
            const double v = wave_sum(static_cast<double>(acc[c]));
            if (lane == 0) wave_part[wid][c] = v;
        }
    }
    __syncthreads();
    const int nb = gridDim.x;
    // Partials are stored write-through (sc1: 8-byte agent-scope atomic stores), so no release fence is
    // needed: a release (buffer_wbl2) would write back every dirty line of the XCD's L2 -- including
    // all the gradient rows just stored -- once per block, which made the kernel slower the more
    // blocks it had.  (MI355X_MICROARCH.md, "Valid forms": sc1 payload + drained waves + counter.)
    if (threadIdx.x < ncols) {
        double v = wave_part[0][threadIdx.x];
#pragma unroll
        for (int w = 1; w < kBlock / kWave; ++w) v += wave_part[w][threadIdx.x];
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(partials + static_cast<int64_t>(threadIdx.x) * nb +
                                                                 blockIdx.x),
                           __double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // every storing wave drains, barrier, then one lane takes a ticket; the last arriver acquires once
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = (t == static_cast<unsigned>(nb) - 1);
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        last_block = last;
    }
    __syncthreads();
    if (!last_block) return;
    // fixed-order fold: column c is handled by wave c % 4, lanes stride over blocks.  The partials are
    // read with sc1 buffer loads (L1 bypass) that, unlike atomic loads, the compiler keeps in flight
    // together instead of serialising one round trip per load.
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        partials, 0, static_cast<int>(sizeof(double) * ncols * nb), 0x00020000);
    for (int c = wid; c < ncols; c += kBlock / kWave) {
        double s = 0.0;
#pragma unroll 8
        for (int r = lane; r < nb; r += kWave) {
            const auto bits = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (c * nb + r) * 8, 0, 16 /* sc1 */);
            s += __builtin_bit_cast(double, bits);
        }
        s = wave_sum(s);
        if (lane == 0) wave_part[0][c] = s;  // row 0 is free again: every wave passed the barrier above
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double Bd = static_cast<double>(p.B);
        float* stats = p.stats;
        stats[1] = static_cast<float>(wave_part[0][kColSurr] / Bd);
        stats[2] = static_cast<float>(wave_part[0][kColValue] / Bd);
        stats[3] = static_cast<float>(wave_part[0][kColEnt] / Bd);
        stats[4] = static_cast<float>(wave_part[0][kColKl] / Bd);
        // ppo.py:315 in fp32: surrogate_loss + c_v * value_loss - c_e * entropy.mean()
        stats[0] = __fsub_rn(__fadd_rn(stats[1], __fmul_rn(value_loss_coef, stats[2])),
                             __fmul_rn(entropy_coef, stats[3]));
        if (!p.normalize_adv) {
            stats[5] = 0.0f;
            stats[6] = 0.0f;
        }
        stats[7] = 0.0f;
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm (stream-ordered)
    }
    if constexpr (SHARED) {
        if (threadIdx.x < A) p.grad_sigma[threadIdx.x] = static_cast<float>(wave_part[0][kNumScalarCols + threadIdx.x]);
    }
}

// ---- quad layout (A % 4 == 0, A <= 16): four lanes per sample ------------------------------------
//
// The lane-per-sample kernel above holds whole [A] rows per lane (182 VGPRs at A = 12: two waves per
// SIMD) and each of its row loads covers 64 rows at a 48-byte stride.  Here a wave owns a tile of 64
// samples and works on it in two layouts:
//   row layout    (4 rounds of 16 samples): lane l holds actions [APL*(l&3), APL*(l&3)+APL) of sample
//                 16*round + (l>>2) -- every row load / gradient store of a round is one contiguous
//                 16*A*4-byte segment, and every per-action transcendental (KL log, division) is
//                 evaluated once;
//   sample layout (lane l = sample l): ratio, clipped surrogate, clipped value loss, their gradients,
//                 coalesced scalar loads and the d/dV store.
// log-prob partials are summed inside each quad (two DPP adds) and moved to the sample layout with
// four ds_bpermute; d(loss)/d(log-prob) moves back the same way.  Per-element arithmetic is the same
// expression sequence as the lane-per-sample kernel; only the summation order of the A log-prob terms
// (three sequential, then a quad tree) and of the KL terms differs.
//
// Partials fold in two levels so that the grid can cover one tile per wave: groups of kFoldGroup
// blocks (last arriver of a group folds the group, fixed order), then the last group folds the groups.

constexpr int kQuadMaxBlocks = 256;  // one workgroup per CU; 6 tiles per wave at C3 (measured: 256 < 512 < 768 us)

using rsrc_t = __amdgpu_buffer_rsrc_t;

// Buffer resource over `bytes` bytes: loads past the end return 0 and stores past it are dropped, so
// the tail tile needs no per-lane guards on its memory operations (only on what it accumulates).
__device__ __forceinline__ rsrc_t make_rsrc(const void* ptr, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(ptr), 0, static_cast<int>(bytes), 0x00020000);
}

// APL consecutive fp32 values at byte offset `off` (dword-aligned; 16-/8-byte aligned for APL 4 / 2).
// Elements are copied out as values first: hipcc 7.2 lowers __builtin_bit_cast of a vector-element
// lvalue (x[k]) to a read of element 0.
template <int APL>
__device__ __forceinline__ void load_piece(rsrc_t r, uint32_t off, float (&v)[APL]) {
    if constexpr (APL == 4) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = __builtin_bit_cast(float, static_cast<unsigned>(x[k]));
    } else if constexpr (APL == 3) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, 0);
#pragma unroll
        for (int k = 0; k < 3; ++k) v[k] = __builtin_bit_cast(float, static_cast<unsigned>(x[k]));
    } else if constexpr (APL == 2) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
#pragma unroll
        for (int k = 0; k < 2; ++k) v[k] = __builtin_bit_cast(float, static_cast<unsigned>(x[k]));
    } else {
        v[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
    }
}

template <int APL>
__device__ __forceinline__ void store_piece(rsrc_t r, uint32_t off, const float (&v)[APL]) {
    using u = unsigned int;
    if constexpr (APL == 4) {
        __attribute__((ext_vector_type(4))) u x;
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = __builtin_bit_cast(u, v[k]);
        __builtin_amdgcn_raw_buffer_store_b128(x, r, off, 0, 0);
    } else if constexpr (APL == 3) {
        __attribute__((ext_vector_type(3))) u x;
#pragma unroll
        for (int k = 0; k < 3; ++k) x[k] = __builtin_bit_cast(u, v[k]);
        __builtin_amdgcn_raw_buffer_store_b96(x, r, off, 0, 0);
    } else if constexpr (APL == 2) {
        __attribute__((ext_vector_type(2))) u x;
#pragma unroll
        for (int k = 0; k < 2; ++k) x[k] = __builtin_bit_cast(u, v[k]);
        __builtin_amdgcn_raw_buffer_store_b64(x, r, off, 0, 0);
    } else {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(u, v[0]), r, off, 0, 0);
    }
}

__device__ __forceinline__ float load_f32(rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

// fold_columns for up to 256 partials per column: 16 lanes per column, each adding rows l16, l16 + 16, ..., l16 + 240
// in that order (all 16 loads in flight first), then a 16-lane butterfly -- one memory round trip.
template <int kMaxC>
__device__ __forceinline__ void fold_columns_wide(const double* __restrict__ src, int ld, int n, int ncols,
                                                  double* __restrict__ out) {
    constexpr int kPasses = (kMaxC + 15) / 16;
    const int l16 = threadIdx.x & 15;
    const int cc = threadIdx.x >> 4;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<double*>(src), 0, static_cast<int>(sizeof(double) * ncols * ld), 0x00020000);
#pragma unroll
    for (int ps = 0; ps < kPasses; ++ps) {
        const int c = ps * 16 + cc;
        double v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int r = l16 + 16 * i;
            const int off = (c < ncols && r < n) ? (c * ld + r) * 8 : 0x7ffffff0;  // out of range: reads 0
            v[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off, 0, 16 /* sc1 */));
        }
        double t = v[0];
#pragma unroll
        for (int i = 1; i < 16; ++i) t += v[i];
#pragma unroll
        for (int off = 8; off >= 1; off >>= 1) t += __shfl_xor(t, off, kWave);
        if (l16 == 0 && c < ncols) out[c] = t;
    }
}

// Waves per SIMD the register budget is sized for (no spills at these bounds, hipcc 7.2): two tiles
// (current + prefetched) of row pieces live per lane.
constexpr int quad_waves(int apl, bool shared, bool kl) { return (apl == 1 && (shared || !kl)) ? 4 : 2; }

template <int APL, bool SHARED, bool KL, int DEPTH = 1>
__global__ __launch_bounds__(kBlock, DEPTH > 1 ? 1 : quad_waves(APL, SHARED, KL)) void ppo_loss_quad_kernel(LossParams p, double* __restrict__ partials,
                                                               unsigned* __restrict__ tickets, float value_loss_coef,
                                                               float entropy_coef) {
    constexpr int A = 4 * APL;
    constexpr int kCols = kNumScalarCols + (SHARED ? A : 0);
    __shared__ double wave_part[kBlock / kWave][kCols];
    __shared__ double folded[kCols];
    __shared__ int last_flag;
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    const int q = lane & 3;
    const int s16 = lane >> 2;
    const int a0 = q * APL;

    float c_s[APL], c_ls[APL], c_inv_den[APL], c_inv_s[APL], c_inv_s3[APL];
    // KL with a shared sigma (ppo.py:262-268): the rollout stored one sigma per action for every sample (the
    // same std parameter), so log(sigma / old_sigma + 1e-5) is a per-action constant -- evaluated once here
    // from sample 0's old sigma and used for every element whose old sigma has exactly those bits (any other
    // element takes the full expression) -- and the division by the per-action constant D = 2 sigma^2 is
    // done as q0 = n * RN(1/D), q = fma(fma(-q0, D, n), RN(1/D), q0): the correctly rounded quotient
    // (Markstein's theorem; tested against true division in oracle/kl_division_check.c) for n and D in the
    // normal range, which the per-element test below keeps it to.  Same bits as __fdiv_rn, ~30 fewer VALU.
    float c_os[APL], c_t1[APL], c_D[APL], c_rD[APL];
    float ent_shared = 0.0f;
    float adv_mean = 0.0f, adv_den = 1.0f;

    float acc_surr = 0.0f, acc_value = 0.0f, acc_ent = 0.0f, acc_kl = 0.0f;
    float acc_sig[APL];
#pragma unroll
    for (int k = 0; k < APL; ++k) acc_sig[k] = 0.0f;

    // Buffer resources (byte extents < 2^31, checked by the host): rows of [B, A] operands share one
    // 32-bit offset per round; mu / grad_mu / sigma rows use their own strides.
    const uint32_t B32 = static_cast<uint32_t>(p.B);
    const uint32_t rowA = static_cast<uint32_t>(A) * 4u;
    const auto ext = [&](int64_t stride) { return static_cast<uint32_t>(((p.B - 1) * stride + A) * 4); };
    const rsrc_t r_mu = make_rsrc(p.mu, ext(p.mu_stride));
    const rsrc_t r_x = make_rsrc(p.actions, B32 * rowA);
    const rsrc_t r_omu = make_rsrc(p.old_mu, B32 * rowA);
    const rsrc_t r_osg = make_rsrc(p.old_sigma, B32 * rowA);
    const rsrc_t r_sg = make_rsrc(p.sigma, SHARED ? rowA : ext(p.sigma_stride));
    const rsrc_t r_gmu = make_rsrc(p.grad_mu, ext(p.grad_mu_stride));
    const rsrc_t r_gsg = make_rsrc(p.grad_sigma, SHARED ? rowA : ext(p.grad_sigma_stride));
    const rsrc_t r_ologp = make_rsrc(p.old_logp, B32 * 4u);
    const rsrc_t r_adv = make_rsrc(p.adv, B32 * 4u);
    const rsrc_t r_v = make_rsrc(p.values, B32 * 4u);
    const rsrc_t r_tv = make_rsrc(p.target_values, B32 * 4u);
    const rsrc_t r_ret = make_rsrc(p.returns, B32 * 4u);
    const rsrc_t r_gv = make_rsrc(p.grad_values, static_cast<uint32_t>(((p.B - 1) * p.gv_stride + 1) * 4));
    const uint32_t gv_row = static_cast<uint32_t>(p.gv_stride) * 4u;
    const uint32_t mu_row = static_cast<uint32_t>(p.mu_stride) * 4u;
    const uint32_t gmu_row = static_cast<uint32_t>(p.grad_mu_stride) * 4u;
    const uint32_t sg_row = static_cast<uint32_t>(p.sigma_stride) * 4u;
    const uint32_t gsg_row = static_cast<uint32_t>(p.grad_sigma_stride) * 4u;
    const uint32_t piece = static_cast<uint32_t>(a0) * 4u;

    const uint32_t ntiles = static_cast<uint32_t>(ceil_div(p.B, kWave));
    const uint32_t tstride = gridDim.x * (kBlock / kWave);
    // Software pipeline over this wave's tiles: the next tile's loads are issued before the current
    // tile is computed, so each wave keeps one tile (~13.5 KB at A = 12) in flight while it computes.
    // A tile index past the end loads zeros through the buffer resources and is never computed.
    struct TileIn {
        float old_logp, adv, V, tv, R;
        float mu[4][APL], x[4][APL], omu[4][APL], osg[4][APL], sr[4][APL];
    };
    const auto load_tile = [&](uint32_t tile, TileIn& t) {
        const uint32_t base = tile * kWave;
        const uint32_t is = base + lane;
        t.old_logp = load_f32(r_ologp, is * 4u);
        t.adv = load_f32(r_adv, is * 4u);
        t.V = load_f32(r_v, is * 4u);
        t.tv = load_f32(r_tv, is * 4u);
        t.R = load_f32(r_ret, is * 4u);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t iq = base + 16 * j + s16;
            load_piece<APL>(r_mu, iq * mu_row + piece, t.mu[j]);
            load_piece<APL>(r_x, iq * rowA + piece, t.x[j]);
            if constexpr (KL) {
                load_piece<APL>(r_omu, iq * rowA + piece, t.omu[j]);
                load_piece<APL>(r_osg, iq * rowA + piece, t.osg[j]);
            }
            if constexpr (!SHARED) load_piece<APL>(r_sg, iq * sg_row + piece, t.sr[j]);
        }
    };
    uint32_t tile = blockIdx.x * (kBlock / kWave) + wid;
    TileIn cur, ahead;  // DEPTH 2: `ahead` = the tile after the next one is loaded while this one is computed
    if (tile < ntiles) load_tile(tile, cur);
    if constexpr (DEPTH > 1) load_tile(tile + tstride, ahead);
    // the per-action constants after the first tile's loads are in flight (their loads and logf chains would
    // otherwise delay them)
    if constexpr (SHARED) {
#pragma unroll
        for (int k = 0; k < APL; ++k) {
            const float s = p.sigma[a0 + k];
            const float inv_s = 1.0f / s;
            c_s[k] = s;
            c_ls[k] = logf(s);
            c_inv_den[k] = 1.0f / __fmul_rn(2.0f, __fmul_rn(s, s));
            c_inv_s[k] = inv_s;
            c_inv_s3[k] = inv_s * inv_s * inv_s;
            if constexpr (KL) {
                const float os0 = p.B > 0 ? p.old_sigma[a0 + k] : 1.0f;
                const float D = __fmul_rn(2.0f, __fmul_rn(s, s));
                const bool d_ok = D >= 0x1p-60f && D <= 0x1p60f;  // else: every element takes the full path
                c_os[k] = (d_ok && p.kl_fast) ? os0 : __builtin_nanf("");  // NaN never compares equal
                c_t1[k] = logf(__fadd_rn(__fdiv_rn(s, os0), 1.0e-5f));
                c_D[k] = D;
                c_rD[k] = __fdiv_rn(1.0f, D);
            }
        }
#pragma unroll
        for (int a = 0; a < A; ++a) ent_shared = __fadd_rn(ent_shared, __fadd_rn(kEntC, logf(p.sigma[a])));
    }
    if (p.normalize_adv) {
        adv_mean = p.adv_stats[0];
        adv_den = __fadd_rn(p.adv_stats[1], 1e-8f);  // ppo.py:223  (std + 1e-8)
    }
    for (; tile < ntiles; tile += tstride) {
        TileIn nxt;
        load_tile(tile + DEPTH * tstride, nxt);
        const uint32_t base = tile * kWave;
        const uint32_t is = base + lane;
        const bool vs = is < B32;
        const float old_logp = cur.old_logp, V = cur.V, tv = cur.tv, R = cur.R;
        float adv = cur.adv;
        const auto& mu = cur.mu;
        const auto& x = cur.x;
        const auto& omu = cur.omu;
        const auto& osg = cur.osg;
        const auto& sr = cur.sr;

        float d[4][APL], lp[4], klp[4];
        bool kl_slow = false;  // some element of this lane needs the full KL expression
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool vq = base + 16 * j + s16 < B32;
            float lpart = 0.0f, klpart = 0.0f, entpart = 0.0f;
#pragma unroll
            for (int k = 0; k < APL; ++k) {
                float s, ls, inv_den;
                if constexpr (SHARED) {
                    s = c_s[k];
                    ls = c_ls[k];
                    inv_den = c_inv_den[k];
                } else {
                    s = sr[j][k];
                    ls = logf(s);
                    inv_den = 1.0f / (2.0f * s * s);
                    entpart += kEntC + ls;
                }
                const float dd = x[j][k] - mu[j][k];
                d[j][k] = dd;
                lpart += (-(dd * dd) * inv_den - ls) - kLogSqrt2Pi;
                if constexpr (KL) {
                    const float os = osg[j][k];
                    const float dm = __fsub_rn(omu[j][k], mu[j][k]);
                    const float n = __fadd_rn(__fmul_rn(os, os), __fmul_rn(dm, dm));
                    float t1, t2;
                    if constexpr (SHARED) {
                        t1 = c_t1[k];
                        const float q0 = __fmul_rn(n, c_rD[k]);
                        t2 = __builtin_fmaf(__builtin_fmaf(-q0, c_D[k], n), c_rD[k], q0);
                        kl_slow |= !(os == c_os[k] && n >= 0x1p-60f && n <= 0x1p60f);
                    } else {
                        t1 = logf(__fadd_rn(__fdiv_rn(s, os), 1.0e-5f));
                        t2 = __fdiv_rn(n, __fmul_rn(2.0f, __fmul_rn(s, s)));
                    }
                    klpart = __fadd_rn(klpart, __fsub_rn(__fadd_rn(t1, t2), 0.5f));
                }
            }
            klp[j] = klpart;
            if (vq) {
                if constexpr (!SHARED) acc_ent += entpart;
            }
            lp[j] = quad_sum(lpart);
        }
        if constexpr (KL) {
            if constexpr (SHARED) {
                if (kl_slow) {  // the reference's exact expression for every element of this lane (rare)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        float klpart = 0.0f;
#pragma unroll
                        for (int k = 0; k < APL; ++k) {
                            const float s = c_s[k], os = osg[j][k];
                            const float dm = __fsub_rn(omu[j][k], mu[j][k]);
                            const float t1 = logf(__fadd_rn(__fdiv_rn(s, os), 1.0e-5f));
                            const float t2 = __fdiv_rn(__fadd_rn(__fmul_rn(os, os), __fmul_rn(dm, dm)),
                                                       __fmul_rn(2.0f, __fmul_rn(s, s)));
                            klpart = __fadd_rn(klpart, __fsub_rn(__fadd_rn(t1, t2), 0.5f));
                        }
                        klp[j] = klpart;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (base + 16 * j + s16 < B32) acc_kl += klp[j];
        }

        // ---- sample layout: lane l <- log-prob of sample base + l (quad l & 15 of round l >> 4)
        const int src = (lane & 15) << 2;
        const float l0 = __shfl(lp[0], src, kWave), l1 = __shfl(lp[1], src, kWave);
        const float l2 = __shfl(lp[2], src, kWave), l3 = __shfl(lp[3], src, kWave);
        const int rnd = lane >> 4;
        const float logp = rnd == 0 ? l0 : (rnd == 1 ? l1 : (rnd == 2 ? l2 : l3));
        // (lanes past B compute on zero-filled inputs; their results are masked here and their d/dV
        // store is dropped by the buffer resource -- no branch, so the scalar loads issue with the rows)
        if (p.normalize_adv) adv = __fdiv_rn(__fsub_rn(adv, adv_mean), adv_den);
        // surrogate (ppo.py:297-302)
        const float ratio = expf(logp - old_logp);
        const float nadv = -adv;
        const float surr = nadv * ratio;
        const float rc = fminf(fmaxf(ratio, p.ratio_lo), p.ratio_hi);
        const float surr_c = nadv * rc;
        float g_s, g_sc;
        max_grads(surr, surr_c, p.g_surr, g_s, g_sc);
        const bool in_clip = (ratio >= p.ratio_lo) && (ratio <= p.ratio_hi);
        const float g_ratio = g_s * nadv + (in_clip ? g_sc * nadv : 0.0f);
        const float g_logp = vs ? g_ratio * ratio : 0.0f;
        // value loss (ppo.py:305-313)
        float vterm, dV;
        if (p.clipped_value) {
            const float dv = V - tv;
            const float vc = tv + fminf(fmaxf(dv, -p.clip), p.clip);
            const float e1 = V - R;
            const float e2 = vc - R;
            const float vl = e1 * e1;
            const float vlc = e2 * e2;
            vterm = fmaxf(vl, vlc);
            float g1, g2;
            max_grads(vl, vlc, p.g_value, g1, g2);
            dV = 2.0f * g1 * e1;
            if (dv >= -p.clip && dv <= p.clip) dV += 2.0f * g2 * e2;
        } else {
            const float e = R - V;
            vterm = e * e;
            dV = -2.0f * p.g_value * e;
        }
        // (stride 4: whole {dV, 0, 0, 0} rows measured slower than the 4-byte writes: 34.4 vs 32.2 us at C3)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dV), r_gv, is * gv_row, 0, 0);
        if (vs) {
            acc_surr += fmaxf(surr, surr_c);
            acc_value += vterm;
            if constexpr (SHARED) acc_ent += ent_shared;
        }

        // ---- row layout again: d/dmu, d/dsigma from d(loss)/d(log-prob) of each round's sample
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float gj = __shfl(g_logp, 16 * j + s16, kWave);
            const uint32_t iq = base + 16 * j + s16;
            float gmu[APL], gsg[APL];
            const float g2 = 2.0f * gj;
#pragma unroll
            for (int k = 0; k < APL; ++k) {
                float inv_den, inv_s, inv_s3;
                if constexpr (SHARED) {
                    inv_den = c_inv_den[k];
                    inv_s = c_inv_s[k];
                    inv_s3 = c_inv_s3[k];
                } else {
                    const float s = sr[j][k];
                    inv_s = 1.0f / s;
                    inv_den = 0.5f * inv_s * inv_s;
                    inv_s3 = inv_s * inv_s * inv_s;
                }
                const float dd = d[j][k];
                gmu[k] = g2 * dd * inv_den;
                gsg[k] = gj * (dd * dd * inv_s3 - inv_s) + p.g_ent * inv_s;
            }
            store_piece<APL>(r_gmu, iq * gmu_row + piece, gmu);  // past B: dropped by the resource
            if constexpr (SHARED) {
                const bool vq = iq < B32;
#pragma unroll
                for (int k = 0; k < APL; ++k) acc_sig[k] += vq ? gsg[k] : 0.0f;
            } else {
                store_piece<APL>(r_gsg, iq * gsg_row + piece, gsg);
            }
        }
        if constexpr (DEPTH > 1) {
            cur = ahead;
            ahead = nxt;
        } else {
            cur = nxt;
        }
    }

    // ---- block partials: scalar columns by wave butterfly; sigma columns over lanes of equal q
    {
        const double vs_[kNumScalarCols] = {wave_sum(static_cast<double>(acc_surr)),
                                             wave_sum(static_cast<double>(acc_value)),
                                             wave_sum(static_cast<double>(acc_ent)),
                                             wave_sum(static_cast<double>(acc_kl))};
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < kNumScalarCols; ++c) wave_part[wid][c] = vs_[c];
        }
        if constexpr (SHARED) {
#pragma unroll
            for (int k = 0; k < APL; ++k) {
                double v = static_cast<double>(acc_sig[k]);
#pragma unroll
                for (int off = 4; off < kWave; off <<= 1) v += __shfl_xor(v, off, kWave);
                if (lane < 4) wave_part[wid][kNumScalarCols + a0 + k] = v;
            }
        }
    }
    __syncthreads();
    const int nb = gridDim.x;
    const int ng = static_cast<int>(ceil_div(nb, kFoldGroup));
    double* gpart = partials + static_cast<int64_t>(kCols) * nb;  // [kCols][ng] group partials
    if (threadIdx.x < kCols) {
        double v = wave_part[0][threadIdx.x];
#pragma unroll
        for (int w = 1; w < kBlock / kWave; ++w) v += wave_part[w][threadIdx.x];
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(partials + static_cast<int64_t>(threadIdx.x) * nb +
                                                                 blockIdx.x),
                           __double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (nb <= kBlock) {  // one level: the last of the <= 256 blocks folds every partial in one round trip
        if (threadIdx.x == 0) {
            const unsigned t = __hip_atomic_fetch_add(tickets, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = (t == static_cast<unsigned>(nb) - 1);
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            last_flag = last;
        }
        __syncthreads();
        if (!last_flag) return;
        fold_columns_wide<kCols>(partials, nb, nb, kCols, folded);
        __syncthreads();
    } else {
    // level 1: the last arriver of this block's group folds the group's partials (fixed order)
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
        last_flag = last;
    }
    __syncthreads();
    if (!last_flag) return;
    if (threadIdx.x == 0) __hip_atomic_store(tickets + 1 + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    fold_columns<kCols>(partials + g0, nb, gsz, kCols, folded);
    __syncthreads();
    if (ng > 1) {
        if (threadIdx.x < kCols)
            __hip_atomic_store(
                reinterpret_cast<unsigned long long*>(gpart + static_cast<int64_t>(threadIdx.x) * ng + g),
                __double_as_longlong(folded[threadIdx.x]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // level 2: the last group folds the group partials
        if (threadIdx.x == 0) {
            const unsigned t = __hip_atomic_fetch_add(tickets, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = (t == static_cast<unsigned>(ng) - 1);
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            last_flag = last;
        }
        __syncthreads();
        if (!last_flag) return;
        fold_columns<kCols>(gpart, ng, ng, kCols, folded);
        __syncthreads();
    }
    }
    if (threadIdx.x == 0) {
        const double Bd = static_cast<double>(p.B);
        float* stats = p.stats;
        stats[1] = static_cast<float>(folded[kColSurr] / Bd);
        stats[2] = static_cast<float>(folded[kColValue] / Bd);
        stats[3] = static_cast<float>(folded[kColEnt] / Bd);
        stats[4] = static_cast<float>(folded[kColKl] / Bd);
        stats[0] = __fsub_rn(__fadd_rn(stats[1], __fmul_rn(value_loss_coef, stats[2])),
                             __fmul_rn(entropy_coef, stats[3]));
        if (!p.normalize_adv) {
            stats[5] = 0.0f;
            stats[6] = 0.0f;
        }
        stats[7] = 0.0f;
        __hip_atomic_store(tickets, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm (stream-ordered)
    }
    if constexpr (SHARED) {
        if (threadIdx.x < A) p.grad_sigma[threadIdx.x] = static_cast<float>(folded[kNumScalarCols + threadIdx.x]);
    }
}

// Per-mini-batch advantage statistics (ppo.py:221-223): moments -> (mean, unbiased std) in stats[5..6].
__global__ __launch_bounds__(kBlock) void mb_moments_kernel(const float* __restrict__ x, int64_t n,
                                                            double2* __restrict__ partials) {
    __shared__ double scratch[2][kBlock / kWave];
    double s = 0.0, ss = 0.0;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
        const double a = x[i];
        s += a;
        ss += a * a;
    }
    s = block_sum(s, scratch[0]);
    ss = block_sum(ss, scratch[1]);
    if (threadIdx.x == 0) partials[blockIdx.x] = make_double2(s, ss);
}

__global__ __launch_bounds__(kBlock) void mb_moments_fold_kernel(const double2* __restrict__ partials, int np,
                                                                 int64_t n, float* __restrict__ stats) {
    __shared__ double scratch[2][kBlock / kWave];
    double s = 0.0, ss = 0.0;
    for (int i = threadIdx.x; i < np; i += kBlock) {
        s += partials[i].x;
        ss += partials[i].y;
    }
    s = block_sum(s, scratch[0]);
    ss = block_sum(ss, scratch[1]);
    if (threadIdx.x == 0) {
        const double mean = s / static_cast<double>(n);
        double var = (ss - s * mean) / static_cast<double>(n - 1);
        if (var < 0.0) var = 0.0;
        stats[5] = static_cast<float>(mean);
        stats[6] = static_cast<float>(sqrt(var));
    }
}

constexpr int kMomentBlocks = 256;

// Grid cap; RSLRL_LOSS_MAX_BLOCKS overrides it (tuning knob, read once).
int max_blocks() {
    static const int v = [] {
        const char* e = std::getenv("RSLRL_LOSS_MAX_BLOCKS");
        const int x = e ? std::atoi(e) : 0;
        return x > 0 ? std::min(x, 4096) : kMaxBlocks;
    }();
    return v;
}

int loss_blocks(int64_t B) {
    return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(ceil_div(B, kBlock), max_blocks())));
}

// Quad-layout grid: one 64-sample tile per wave up to kQuadMaxBlocks (RSLRL_LOSS_QUAD_MAX_BLOCKS overrides).
int quad_blocks(int64_t B) {
    static const int cap = [] {
        const char* e = std::getenv("RSLRL_LOSS_QUAD_MAX_BLOCKS");
        const int x = e ? std::atoi(e) : 0;
        return x > 0 ? std::min(x, kFoldGroup * kFoldGroup) : kQuadMaxBlocks;
    }();
    return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(ceil_div(B, kBlock), cap)));
}

// Kernel choice, read per call so tests can exercise both: RSLRL_LOSS_KERNEL=lane / quad forces one,
// unset picks the quad kernel for a shared sigma (29 vs 32 us at C3) and the lane kernel for per-row
// sigma (34 vs 36 us: the row layout's extra sigma stream costs more than it saves).
bool use_quad(int sigma_mode) {
    const char* e = std::getenv("RSLRL_LOSS_KERNEL");
    if (e && std::string(e) == "lane") return false;
    if (e && std::string(e) == "quad") return true;
    return sigma_mode == 0;
}

// software-pipeline depth of the quad kernel (tiles in flight per wave beyond the one computed); RSLRL_LOSS_DEPTH
// overrides it (read per call: A/B runs)
int loss_depth() {
    const char* e = std::getenv("RSLRL_LOSS_DEPTH");
    return (e && e[0] == '2') ? 2 : 1;
}

template <int APL>
void launch_quad(const LossParams& p, int nb, double* part, unsigned* tickets, float cv, float ce, hipStream_t st) {
    const dim3 g(nb), b(kBlock);
    if (p.sigma_mode == 0 && p.compute_kl && loss_depth() == 2)
        launch_timed(kTagPpoLoss, ppo_loss_quad_kernel<APL, true, true, 2>, g, b, 0, st, p, part, tickets, cv, ce);
    else if (p.sigma_mode == 0 && p.compute_kl)
        launch_timed(kTagPpoLoss, ppo_loss_quad_kernel<APL, true, true>, g, b, 0, st, p, part, tickets, cv, ce);
    else if (p.sigma_mode == 0)
        launch_timed(kTagPpoLoss, ppo_loss_quad_kernel<APL, true, false>, g, b, 0, st, p, part, tickets, cv, ce);
    else if (p.compute_kl)
        launch_timed(kTagPpoLoss, ppo_loss_quad_kernel<APL, false, true>, g, b, 0, st, p, part, tickets, cv, ce);
    else
        launch_timed(kTagPpoLoss, ppo_loss_quad_kernel<APL, false, false>, g, b, 0, st, p, part, tickets, cv, ce);
}

template <int MAXA, bool EXACT>
void launch_loss_exact(const LossParams& p, bool vec, int nb, double* part, unsigned* ticket, float cv, float ce,
                       hipStream_t st) {
    const bool shared = p.sigma_mode == 0;
    const dim3 g(nb), b(kBlock);
    if (vec && shared)
        hipLaunchKernelGGL((ppo_loss_kernel<MAXA, true, true, EXACT>), g, b, 0, st, p, part, ticket, cv, ce);
    else if (vec)
        hipLaunchKernelGGL((ppo_loss_kernel<MAXA, true, false, EXACT>), g, b, 0, st, p, part, ticket, cv, ce);
    else if (shared)
        hipLaunchKernelGGL((ppo_loss_kernel<MAXA, false, true, EXACT>), g, b, 0, st, p, part, ticket, cv, ce);
    else
        hipLaunchKernelGGL((ppo_loss_kernel<MAXA, false, false, EXACT>), g, b, 0, st, p, part, ticket, cv, ce);
}

template <int MAXA>
void launch_loss(const LossParams& p, bool vec, int nb, double* part, unsigned* ticket, float cv, float ce,
                 hipStream_t st) {
    if (p.A == MAXA)
        launch_loss_exact<MAXA, true>(p, vec, nb, part, ticket, cv, ce, st);
    else
        launch_loss_exact<MAXA, false>(p, vec, nb, part, ticket, cv, ce, st);
}

// workspace layout: [tickets: global word, then one per fold group | pad to 1 KiB]
//                   [fp64 partials [cols][blocks], then group partials [cols][groups] | pad][mini-batch moments]
constexpr size_t kTicketBytes = 1024;

bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

}  // namespace
}  // namespace rslrl

using namespace rslrl;

extern "C" size_t rslrl_ppo_loss_workspace_bytes(int64_t B, int32_t A) {
    const size_t cols = kNumScalarCols + static_cast<size_t>(A > 0 ? A : 0);
    const size_t qb = static_cast<size_t>(quad_blocks(B));
    const size_t slots = std::max(static_cast<size_t>(loss_blocks(B)), qb + static_cast<size_t>(ceil_div(qb, kFoldGroup)));
    return kTicketBytes + align_up(sizeof(double) * cols * slots, 256) + sizeof(double2) * kMomentBlocks;
}

extern "C" int rslrl_ppo_loss_fwd_bwd(const rslrl_ppo_loss_args_t* a, void* workspace, size_t workspace_bytes,
                                      rslrl_stream_t stream) {
    if (!a) return RSLRL_E_INVALID_ARGUMENT;
    if (a->B < 1 || a->A < 1 || a->A > RSLRL_PPO_LOSS_MAX_ACTIONS) return RSLRL_E_INVALID_ARGUMENT;
    if (a->sigma_mode != 0 && a->sigma_mode != 1) return RSLRL_E_INVALID_ARGUMENT;
    if (!a->mu || !a->sigma || !a->values || !a->actions || !a->old_logp || !a->advantages || !a->target_values ||
        !a->returns || !a->old_mu || !a->old_sigma || !a->grad_mu || !a->grad_sigma || !a->grad_values || !a->stats)
        return RSLRL_E_INVALID_ARGUMENT;
    if (a->mu_stride < a->A || a->grad_mu_stride < a->A) return RSLRL_E_INVALID_ARGUMENT;
    if (a->sigma_mode == 1 && (a->sigma_stride < a->A || a->grad_sigma_stride < a->A)) return RSLRL_E_INVALID_ARGUMENT;
    if (!workspace) return RSLRL_E_INVALID_ARGUMENT;
    if (workspace_bytes < rslrl_ppo_loss_workspace_bytes(a->B, a->A)) return RSLRL_E_WORKSPACE_TOO_SMALL;
    if (!aligned16(workspace)) return RSLRL_E_MISALIGNED;

    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int A = a->A;
    const int nb = loss_blocks(a->B);
    const int nbq = quad_blocks(a->B);
    const size_t slots = std::max<size_t>(nb, nbq + ceil_div(nbq, kFoldGroup));
    unsigned* ticket = static_cast<unsigned*>(workspace);
    double* part = reinterpret_cast<double*>(static_cast<char*>(workspace) + kTicketBytes);
    double2* mpart = reinterpret_cast<double2*>(static_cast<char*>(workspace) + kTicketBytes +
                                                align_up(sizeof(double) * (kNumScalarCols + A) * slots, 256));

    LossParams p{};
    p.B = a->B;
    p.A = A;
    p.sigma_mode = a->sigma_mode;
    p.mu = a->mu;
    p.mu_stride = a->mu_stride;
    p.sigma = a->sigma;
    p.sigma_stride = a->sigma_stride;
    p.values = a->values;
    p.actions = a->actions;
    p.old_logp = a->old_logp;
    p.adv = a->advantages;
    p.target_values = a->target_values;
    p.returns = a->returns;
    p.old_mu = a->old_mu;
    p.old_sigma = a->old_sigma;
    p.clip = a->clip_param;
    p.ratio_lo = static_cast<float>(1.0 - static_cast<double>(a->clip_param));
    p.ratio_hi = static_cast<float>(1.0 + static_cast<double>(a->clip_param));
    const float Bf = static_cast<float>(a->B);
    p.g_surr = 1.0f / Bf;
    p.g_value = a->value_loss_coef / Bf;
    p.g_ent = -a->entropy_coef / Bf;
    p.clipped_value = a->use_clipped_value_loss ? 1 : 0;
    p.compute_kl = a->compute_kl ? 1 : 0;
    p.normalize_adv = a->normalize_advantage ? 1 : 0;
    p.grad_mu = a->grad_mu;
    p.grad_mu_stride = a->grad_mu_stride;
    p.grad_sigma = a->grad_sigma;
    p.grad_sigma_stride = a->grad_sigma_stride;
    p.grad_values = a->grad_values;
    p.gv_stride = a->grad_values_stride > 1 ? a->grad_values_stride : 1;
    p.adv_stats = a->stats + 5;
    p.stats = a->stats;
    {  // RSLRL_KL_FAST=0 disables the per-action-constant KL (read per call: the tests compare both bitwise)
        const char* e = std::getenv("RSLRL_KL_FAST");
        p.kl_fast = (e && e[0] == '0') ? 0 : 1;
    }

    if (p.normalize_adv) {
        const int mb = static_cast<int>(std::min<int64_t>(ceil_div(a->B, kBlock), kMomentBlocks));
        hipLaunchKernelGGL(mb_moments_kernel, dim3(mb), dim3(kBlock), 0, st, a->advantages, a->B, mpart);
        hipLaunchKernelGGL(mb_moments_fold_kernel, dim3(1), dim3(kBlock), 0, st, mpart, mb, a->B, a->stats);
        int rc = launch_status();
        if (rc != RSLRL_OK) return rc;
    }

    // 16-byte row accesses when every [B, A] operand allows it
    bool vec = (A % 4 == 0) && (a->mu_stride % 4 == 0) && (a->grad_mu_stride % 4 == 0) && aligned16(a->mu) &&
               aligned16(a->actions) && aligned16(a->old_mu) && aligned16(a->old_sigma) && aligned16(a->grad_mu);
    if (a->sigma_mode == 1)
        vec = vec && (a->sigma_stride % 4 == 0) && (a->grad_sigma_stride % 4 == 0) && aligned16(a->sigma) &&
              aligned16(a->grad_sigma);
    const float cv = a->value_loss_coef, ce = a->entropy_coef;
    const int64_t max_row = std::max({a->mu_stride, a->grad_mu_stride, a->sigma_mode == 1 ? a->sigma_stride : 0,
                                      a->sigma_mode == 1 ? a->grad_sigma_stride : 0, static_cast<int64_t>(A)});
    const bool fits32 = a->B * std::max(max_row, p.gv_stride) * 4 < (int64_t{1} << 31);  // 32-bit buffer offsets
    if (vec && fits32 && A % 4 == 0 && A <= 16 && use_quad(a->sigma_mode)) {
        switch (A / 4) {
            case 1: launch_quad<1>(p, nbq, part, ticket, cv, ce, st); break;
            case 2: launch_quad<2>(p, nbq, part, ticket, cv, ce, st); break;
            case 3: launch_quad<3>(p, nbq, part, ticket, cv, ce, st); break;
            default: launch_quad<4>(p, nbq, part, ticket, cv, ce, st); break;
        }
        return launch_status();
    }
    if (A <= 4)
        launch_loss<4>(p, vec, nb, part, ticket, cv, ce, st);
    else if (A <= 8)
        launch_loss<8>(p, vec, nb, part, ticket, cv, ce, st);
    else if (A <= 12)
        launch_loss<12>(p, vec, nb, part, ticket, cv, ce, st);
    else if (A <= 16)
        launch_loss<16>(p, vec, nb, part, ticket, cv, ce, st);
    else if (A <= 32)
        launch_loss<32>(p, vec, nb, part, ticket, cv, ce, st);
    else
        launch_loss<64>(p, vec, nb, part, ticket, cv, ce, st);
    return launch_status();
}

// ---- per-mini-batch tail of PPO.update (ppo.py:259-294 adaptive lr, :387-395 loss statistics) ----------
// One thread: the reference's host logic on device scalars, so the update loop needs no host round trip and
// no chain of one-element torch launches.
namespace {
__global__ void ppo_tail_kernel(const float* __restrict__ stats, const float* __restrict__ kl_src, double* lr,
                                float* lr32, int round_fp32, float kl_hi, float kl_lo, double* sums) {
    if (threadIdx.x != 0) return;
    if (lr) {
        const float kl = *kl_src;
        double v = *lr;
        // ppo.py:280-284 with the reference's operand types: kl (fp32 tensor) against Python floats -> fp32
        // comparisons; lr stays a Python float (fp64)
        if (kl > kl_hi) {
            v = fmax(v / 1.5, 1e-5);
        } else if (kl < kl_lo && kl > 0.0f) {
            v = fmin(v * 1.5, 1e-2);
        }
        if (round_fp32) v = static_cast<double>(static_cast<float>(v));  // ppo.py:288-290 fp32 broadcast
        *lr = v;
        *lr32 = static_cast<float>(v);
    }
    if (sums) {  // [value_function, surrogate, entropy] += the mini-batch's means (fp64 host accumulation)
        sums[0] += static_cast<double>(stats[2]);
        sums[1] += static_cast<double>(stats[1]);
        sums[2] += static_cast<double>(stats[3]);
    }
}
}  // namespace

extern "C" int rslrl_ppo_update_tail(const float* stats, const float* kl, double* lr, float* lr32, int32_t round_fp32,
                                     float kl_hi, float kl_lo, double* sums, rslrl_stream_t stream) {
    if (!stats || (lr && (!lr32 || !kl))) return RSLRL_E_INVALID_ARGUMENT;
    hipLaunchKernelGGL(ppo_tail_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), stats, kl, lr,
                       lr32, round_fp32, kl_hi, kl_lo, sums);
    return launch_status();
}

namespace rslrl {
LaunchTiming& launch_timing() {
    static LaunchTiming t;
    return t;
}
}  // namespace rslrl

extern "C" int rslrl_launch_timing_enable(int32_t capacity) {
    if (capacity < 0) return RSLRL_E_INVALID_ARGUMENT;
    LaunchTiming& t = launch_timing();
    std::lock_guard<std::mutex> lk(t.mu);
    if (capacity == 0) {  // disarm; the recorded launches stay readable
        t.on.store(false);
        return RSLRL_OK;
    }
    t.on.store(false);
    while (t.pool.size() < static_cast<size_t>(capacity)) {
        hipEvent_t e0 = nullptr, e1 = nullptr;
        hipError_t err = hipEventCreate(&e0);
        if (err == hipSuccess) err = hipEventCreate(&e1);
        if (err != hipSuccess) {
            if (e0) (void)hipEventDestroy(e0);
            return static_cast<int>(err);
        }
        t.pool.push_back({e0, e1, 0});
    }
    t.used = 0;
    t.cap = static_cast<size_t>(capacity);
    t.on.store(true);
    return RSLRL_OK;
}

extern "C" int rslrl_launch_timing_read_tag(int32_t tag, double* total_ms, int64_t* launches) {
    if (!total_ms || !launches || tag < 0 || tag >= kNumLaunchTags) return RSLRL_E_INVALID_ARGUMENT;
    LaunchTiming& t = launch_timing();
    // the used event pairs are copied under the lock and synchronised after it is released: a timed launch on
    // another thread (launch_timed takes the same lock) never waits for this read's event synchronisations
    std::vector<LaunchTiming::Slot> slots;
    {
        std::lock_guard<std::mutex> lk(t.mu);
        slots.assign(t.pool.begin(), t.pool.begin() + static_cast<std::ptrdiff_t>(t.used));
    }
    double sum = 0.0;
    int64_t n = 0;
    for (const auto& sl : slots) {
        if (sl.tag != tag) continue;
        hipError_t err = hipEventSynchronize(sl.stop);
        float ms = 0.0f;
        if (err == hipSuccess) err = hipEventElapsedTime(&ms, sl.start, sl.stop);
        if (err != hipSuccess) return static_cast<int>(err);
        sum += static_cast<double>(ms);
        ++n;
    }
    *total_ms = sum;
    *launches = n;
    return RSLRL_OK;
}

extern "C" int rslrl_launch_timing_read(double* total_ms, int64_t* launches) {
    return rslrl_launch_timing_read_tag(kTagPpoLoss, total_ms, launches);
}
