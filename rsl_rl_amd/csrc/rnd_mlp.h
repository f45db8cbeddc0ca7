// The RND networks (rsl_rl/modules/rnd.py:85-95: networks/mlp.py Linear(in -> H) + ELU + Linear(H -> Q)) evaluated
// one row per lane from LDS-resident weights -- shared by the rollout record (intrinsic reward, rnd.py:113-135) and
// the update's predictor step (ppo.py:352-372).
//
// LDS image of one net (rnd_stage_net), zero-padded to compile-time widths INP >= in and HP >= H (multiples of 4):
//   w1 [HP][INP]  b1 [HP]  w2 [Q][HP]  b2 [Q] (padded to 4)
// Per hidden unit the fp32 fma chain in input order z = fma(w1[h][i], x[i], z), then + b1 (the same order as the
// fused rollout's intrinsic reward had since round 1); padded inputs (x = 0, w = 0) leave z unchanged, padded units
// get z = 0, ELU 0 and zero output weights.
#pragma once

#include "common.h"

namespace rslrl {

typedef float f32x2_t __attribute__((ext_vector_type(2)));

__host__ __device__ constexpr int rnd_net_floats(int inp, int hp, int q) { return hp * inp + hp + q * hp + ((q + 3) & ~3); }

// expm1(v) for v <= 0 in ~12 VALU, branch-free (the same series as mlp_gemm.hip's ELU epilogue): degree-9 Taylor on
// [-0.5, 0] (truncation < 3e-10 relative), exp(v) - 1 below (<= 2 ulp of the result)
__device__ __forceinline__ float rnd_expm1_neg(float v) {
    float t = __fmaf_rn(v, 2.7557319e-6f, 2.4801587e-5f);
    t = __fmaf_rn(v, t, 1.9841270e-4f);
    t = __fmaf_rn(v, t, 1.3888889e-3f);
    t = __fmaf_rn(v, t, 8.3333333e-3f);
    t = __fmaf_rn(v, t, 4.1666667e-2f);
    t = __fmaf_rn(v, t, 1.6666667e-1f);
    t = __fmaf_rn(v, t, 0.5f);
    t = __fmaf_rn(v, t, 1.0f);
    const float poly = v * t;
    const float e = __expf(v) - 1.0f;
    return v > -0.5f ? poly : e;
}
// ELU (alpha 1) as a select: the negative branch is computed unconditionally (the empty asm pins it), otherwise the
// compiler turns it into exec-masked branches and hoists the next hidden units' LDS weight reads across them
__device__ __forceinline__ float rnd_elu(float z) {
    float n = rnd_expm1_neg(fminf(z, 0.f));
    asm volatile("" : "+v"(n));
    return z > 0.f ? z : n;
}
// ELU(z) and torch's elu_backward factor on the input (exp(z) for z <= 0, 1 above) sharing one exp
__device__ __forceinline__ void rnd_elu_and_grad(float z, float& a, float& g) {
    const float v = fminf(z, 0.f);
    float t = __fmaf_rn(v, 2.7557319e-6f, 2.4801587e-5f);
    t = __fmaf_rn(v, t, 1.9841270e-4f);
    t = __fmaf_rn(v, t, 1.3888889e-3f);
    t = __fmaf_rn(v, t, 8.3333333e-3f);
    t = __fmaf_rn(v, t, 4.1666667e-2f);
    t = __fmaf_rn(v, t, 1.6666667e-1f);
    t = __fmaf_rn(v, t, 0.5f);
    t = __fmaf_rn(v, t, 1.0f);
    float e = __expf(v);
    float n = v > -0.5f ? v * t : e - 1.0f;
    asm volatile("" : "+v"(n), "+v"(e));
    a = z > 0.f ? z : n;
    g = z > 0.f ? 1.f : e;
}
// torch's elu_backward factor on the input: exp(z) for z <= 0, 1 above
__device__ __forceinline__ float rnd_elu_grad(float z) {
    float e = __expf(fminf(z, 0.f));
    asm volatile("" : "+v"(e));
    return z > 0.f ? 1.f : e;
}

// Cooperative copy of a net's four tensors into its LDS image (every thread of the block takes part; no barrier).
__device__ __forceinline__ void rnd_stage_net(float* __restrict__ dst, const float* __restrict__ w1,
                                              const float* __restrict__ b1, const float* __restrict__ w2,
                                              const float* __restrict__ b2, int in, int H, int Q, int INP, int HP) {
    const int n = rnd_net_floats(INP, HP, Q);
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        float v = 0.f;
        if (k < HP * INP) {
            const int h = k / INP, i = k - h * INP;
            if (h < H && i < in) v = w1[h * in + i];
        } else if (k < HP * INP + HP) {
            const int h = k - HP * INP;
            if (h < H) v = b1[h];
        } else if (k < HP * INP + HP + Q * HP) {
            const int r = k - HP * INP - HP;
            const int q = r / HP, h = r - q * HP;
            if (h < H) v = w2[q * H + h];
        } else {
            const int q = k - HP * INP - HP - Q * HP;
            if (q < Q) v = b2[q];
        }
        dst[k] = v;
    }
}

// rnd_stage_net with W1 transposed: w1t [INP][HP] (the HP weights of input i contiguous), same b1 / w2 / b2 layout
__device__ __forceinline__ void rnd_stage_net_t(float* __restrict__ dst, const float* __restrict__ w1,
                                                const float* __restrict__ b1, const float* __restrict__ w2,
                                                const float* __restrict__ b2, int in, int H, int Q, int INP, int HP) {
    const int n = rnd_net_floats(INP, HP, Q);
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        float v = 0.f;
        if (k < HP * INP) {
            const int i = k / HP, h = k - i * HP;
            if (h < H && i < in) v = w1[h * in + i];
        } else if (k < HP * INP + HP) {
            const int h = k - HP * INP;
            if (h < H) v = b1[h];
        } else if (k < HP * INP + HP + Q * HP) {
            const int r = k - HP * INP - HP;
            const int q = r / HP, h = r - q * HP;
            if (h < H) v = w2[q * H + h];
        } else {
            const int q = k - HP * INP - HP - Q * HP;
            if (q < Q) v = b2[q];
        }
        dst[k] = v;
    }
}

// Hidden pre-activations z[0 .. HP) of one row x[0 .. INP) (x zero past `in`).  EXACT: in == INP (no guards).
// w: the net's LDS image (16-byte aligned).
template <int INP, int HP, bool EXACT>
__device__ __forceinline__ void rnd_hidden(const float* __restrict__ w, int in, const float (&x)[INP], float (&z)[HP]) {
    static_assert(INP % 4 == 0 && HP % 4 == 0, "padded widths");
    const float* b1 = w + HP * INP;
#pragma unroll
    for (int h = 0; h < HP; ++h) {
        const float4* wr = reinterpret_cast<const float4*>(w + h * INP);
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < INP / 4; ++k) {
            if (EXACT || 4 * k < in) {
                const float4 w4 = wr[k];
                acc = fmaf(w4.x, x[4 * k], acc);
                acc = fmaf(w4.y, x[4 * k + 1], acc);
                acc = fmaf(w4.z, x[4 * k + 2], acc);
                acc = fmaf(w4.w, x[4 * k + 3], acc);
            }
        }
        z[h] = __fadd_rn(acc, b1[h]);
        // one hidden unit at a time: unbounded, the scheduler reads the whole HP x INP image ahead into registers
        __builtin_amdgcn_sched_barrier(0);
    }
}

// The same pre-activations from the transposed image w1t [INP][HP] (rnd_stage_net_t): input-major, two hidden units
// per packed fma -- per unit the same fma chain in input order, so the same bits as rnd_hidden.
template <int INP, int HP, bool EXACT>
__device__ __forceinline__ void rnd_hidden_t(const float* __restrict__ w, int in, const float (&x)[INP], float (&z)[HP]) {
    static_assert(INP % 4 == 0 && HP % 4 == 0, "padded widths");
    f32x2_t acc[HP / 2];
#pragma unroll
    for (int k = 0; k < HP / 2; ++k) acc[k] = f32x2_t{0.f, 0.f};
#pragma unroll
    for (int i = 0; i < INP; ++i) {
        if (EXACT || i < in) {
            const float4* wr = reinterpret_cast<const float4*>(w + i * HP);
            const f32x2_t xi = f32x2_t{x[i], x[i]};
#pragma unroll
            for (int k = 0; k < HP / 4; ++k) {
                const float4 w4 = wr[k];
                acc[2 * k] = __builtin_elementwise_fma(f32x2_t{w4.x, w4.y}, xi, acc[2 * k]);
                acc[2 * k + 1] = __builtin_elementwise_fma(f32x2_t{w4.z, w4.w}, xi, acc[2 * k + 1]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);  // one input at a time (see rnd_hidden)
    }
    const float* b1 = w + HP * INP;
#pragma unroll
    for (int k = 0; k < HP / 2; ++k) {
        z[2 * k] = __fadd_rn(acc[k].x, b1[2 * k]);
        z[2 * k + 1] = __fadd_rn(acc[k].y, b1[2 * k + 1]);
    }
}

// y[q] = b2[q] + sum_h w2[q][h] a[h] (fma chain in hidden order), q < Q
template <int INP, int HP, int MAXQ>
__device__ __forceinline__ void rnd_output(const float* __restrict__ w, int Q, const float (&a)[HP], float (&y)[MAXQ]) {
    const float* w2 = w + HP * INP + HP;
    const float* b2 = w2 + Q * HP;
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) {
        float acc = 0.f;
        if (q < Q) {
#pragma unroll
            for (int h = 0; h < HP; ++h) acc = fmaf(w2[q * HP + h], a[h], acc);
            acc = __fadd_rn(acc, b2[q]);
        }
        y[q] = acc;
    }
}

}  // namespace rslrl
