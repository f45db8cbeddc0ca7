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

#include <cstdlib>

#include "common.h"

namespace rslrl {
namespace {

constexpr int kMaxBlocks = 512;  // a lane handles ~3 samples at C3; the last block folds <= 512 partials
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;  // log(sqrt(2*pi)), normal.py log_prob
constexpr float kEntC = 1.41893853320467274178f;         // 0.5 + 0.5*log(2*pi), normal.py entropy

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
    const float* adv_stats;  // [2] = (mean, std) when normalize_adv
    float* stats;
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

// torch.max(a, b) backward (derivatives.yaml, maximum): ties give each side grad / 2.
__device__ __forceinline__ void max_grads(float a, float b, float g, float& ga, float& gb) {
    const float half = __fmul_rn(g, 0.5f);
    ga = (a > b) ? g : ((a == b) ? half : 0.0f);
    gb = (b > a) ? g : ((a == b) ? half : 0.0f);
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
        p.grad_values[i] = dV;

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

// workspace layout: [ticket word | pad to 256 B][fp64 partials [cols][blocks] | pad][mini-batch moments]
constexpr size_t kTicketBytes = 256;

bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

}  // namespace
}  // namespace rslrl

using namespace rslrl;

extern "C" size_t rslrl_ppo_loss_workspace_bytes(int64_t B, int32_t A) {
    const size_t cols = kNumScalarCols + static_cast<size_t>(A > 0 ? A : 0);
    return kTicketBytes + align_up(sizeof(double) * cols * static_cast<size_t>(loss_blocks(B)), 256) +
           sizeof(double2) * kMomentBlocks;
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
    unsigned* ticket = static_cast<unsigned*>(workspace);
    double* part = reinterpret_cast<double*>(static_cast<char*>(workspace) + kTicketBytes);
    double2* mpart = reinterpret_cast<double2*>(static_cast<char*>(workspace) + kTicketBytes +
                                                align_up(sizeof(double) * (kNumScalarCols + A) * nb, 256));

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
    p.adv_stats = a->stats + 5;
    p.stats = a->stats;

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
