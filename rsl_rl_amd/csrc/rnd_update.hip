// RND predictor training step of one mini-batch (update leg) on gfx950.
//
// Replaces rsl_rl/algorithms/ppo.py:352-363 + :369-372 for the RND networks of rsl_rl/modules/rnd.py:85-95
// (networks/mlp.py: Linear(in -> H) + ELU + Linear(H -> Q)):
//   s     = (state - mean) / (std + eps)                 (optional; normalization.py:40-42, under no_grad)
//   p     = predictor(s),  t = target(s).detach()
//   loss  = mse_loss(p, t) = sum (p - t)^2 / (B Q)
//   grad  = d loss / d (W1, b1, W2, b2) of the predictor    (rnd_loss.backward())
// which the reference runs as ~12 forward + ~12 backward ATen launches per mini-batch (plus a target forward
// whose value never changes within update()).
//
// One launch, 256 threads per workgroup, tiles of 256 rows (one row per thread):
//   forward   each thread evaluates its row (rnd_mlp.h: input-major hidden layer on packed fmas, weights in LDS):
//             t (target weights in LDS; or t read from the cached embedding), p, dp = fp32(2/(BQ)) (p - t)
//             (torch's mse_loss_backward), dz = (W2^T dp) * ELU'(z) with ELU'(z) = exp(z) for z <= 0 (torch's
//             elu_backward on the input);
//   reduction the weight gradient is a sum of per-row outer products over the B rows.  The 4 waves take turns
//             writing their 64 rows into an LDS chunk stored column-major ([column][64 rows], column stride 68:
//             conflict-free lane-per-row writes, 16-byte reads of 4 consecutive rows); every thread then adds the
//             chunk's rows into the gradient entries it owns: a (H/16) x (in/16) block of dW1 on a 16 x 16 thread
//             grid (3 x 3 at C5's 48 -> 48: 6 16-byte reads per 36 FMAs, as packed fmas over row pairs), the
//             db1 / dW2 / db2 entries spread over the first threads.
// Per-workgroup fp32 partials [G][P] are folded in fp64, in workgroup order, by rnd_fold_kernel (one thread
// per gradient entry per 1/16 of the workgroups, then the 16 slices in order), which also finishes the loss.
#include <algorithm>

#include "common.h"
#include "rnd_mlp.h"

namespace rslrl {
namespace {

constexpr int kRows = 256;       // rows per tile (one per thread)
constexpr int kChunk = 64;       // rows per LDS reduction chunk (one wave's rows)
constexpr int kColStride = 68;   // floats per chunk column (64 rows + 4: the 16 x-columns a wave reads hit 16
                                 // distinct 4-bank groups)
constexpr int kMaxGroups = 512;  // workgroups (partials rows); 2 per CU (<= the fold block's 1024 threads)
constexpr int kFoldSlices = 16;  // fold: workgroup slices per gradient entry

struct RndParams {
    int64_t B;
    int in, H, Q;
    float eps;
    const float* state;
    int64_t stride;
    const float* mean;
    const float* std;
    const float* pw[4];  // predictor w1, b1, w2, b2
    const float* tw[4];  // target w1, b1, w2, b2 (tw[0] == nullptr: read temb)
    float* temb;
    float norm;        // fp32(2 / (B Q))
    int P;             // gradient entries
    float* partials;   // [G][P]
    double* lpart;     // [G] loss partials (sum of squared differences)
};

// the (normalised) state row of `row` into registers; zeros past `in` and for rows past B.  VEC (in == MAXIN,
// 16-byte aligned rows): unconditional 16-byte loads of a clamped row, then the zero select -- a guarded 4-byte load
// per element issued 48 scattered-row loads per lane
template <int MAXIN, bool VEC>
__device__ __forceinline__ void load_state(const RndParams& p, int64_t row, bool valid, int in, float (&x)[MAXIN]) {
    const float* sr = p.state + (valid ? row : 0) * p.stride;
    if constexpr (VEC) {
        static_assert(MAXIN % 4 == 0, "whole 16-byte units");
#pragma unroll
        for (int k = 0; k < MAXIN / 4; ++k) {
            const float4 v = reinterpret_cast<const float4*>(sr)[k];
            x[4 * k] = valid ? v.x : 0.f;
            x[4 * k + 1] = valid ? v.y : 0.f;
            x[4 * k + 2] = valid ? v.z : 0.f;
            x[4 * k + 3] = valid ? v.w : 0.f;
        }
    } else {
#pragma unroll
        for (int i = 0; i < MAXIN; ++i) x[i] = (i < in && valid) ? sr[i] : 0.f;
    }
    if (p.mean) {  // (x - mean) / (std + eps)
#pragma unroll
        for (int i = 0; i < MAXIN; ++i)
            if (i < in) x[i] = __fdiv_rn(__fsub_rn(x[i], p.mean[i]), __fadd_rn(p.std[i], p.eps));
    }
}

template <int INP, int MAXHP, int MAXQ, bool EXACT>
__global__ __launch_bounds__(kBlock) void rnd_update_kernel(RndParams p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int BH = MAXHP / 16;         // dW1 block rows per thread (1..4)
    constexpr int BI = (INP + 15) / 16;    // dW1 block columns per thread
    constexpr int kExtra = (MAXHP + MAXQ * MAXHP + MAXQ + kBlock - 1) / kBlock;  // db1 / dW2 / db2 entries per thread
    const int in = EXACT ? INP : p.in;
    const int H = p.H;
    const int Q = EXACT ? MAXQ : p.Q;
    const int nw = rnd_net_floats(INP, MAXHP, Q);  // a multiple of 4
    const bool own_target = p.tw[0] != nullptr;
    // LDS: predictor image | target image (if any) | reduction chunk [columns][kColStride]
    float* wp = lds;
    float* wt = lds + nw;
    float* chunk = lds + (own_target ? 2 * nw : nw);
    // chunk columns: dz [MAXHP] | x [in] | a [MAXHP] | dp [Q]
    const int col_x = MAXHP, col_a = MAXHP + in, col_dp = 2 * MAXHP + in;
    rnd_stage_net_t(wp, p.pw[0], p.pw[1], p.pw[2], p.pw[3], in, H, Q, INP, MAXHP);
    if (own_target) rnd_stage_net_t(wt, p.tw[0], p.tw[1], p.tw[2], p.tw[3], in, H, Q, INP, MAXHP);

    // gradient entries owned by this thread
    const int tr = threadIdx.x >> 4, tc = threadIdx.x & 15;  // 16 x 16 grid over dW1 blocks
    // row sums as two fp32 partial sums per entry (even / odd rows: one packed fma per row pair), added at the end
    f32x2_t g1[BH][BI], gx[kExtra];
#pragma unroll
    for (int u = 0; u < BH; ++u)
#pragma unroll
        for (int v = 0; v < BI; ++v) g1[u][v] = f32x2_t{0.f, 0.f};
    // extra entries e = thread + 256 k of [db1 (H) | dW2 (Q x H) | db2 (Q)]: chunk columns of their two factors (dz[h];
    // dp[q] and a[h]; dp[q]) -- ca < 0: the factor 1; cq < 0: no entry
    int cq[kExtra], ca[kExtra];
#pragma unroll
    for (int k = 0; k < kExtra; ++k) {
        gx[k] = f32x2_t{0.f, 0.f};
        const int e = threadIdx.x + k * kBlock;
        const int f = e - H;  // index into [dW2 | db2]
        const int q = f < Q * H ? f / H : f - Q * H;
        cq[k] = e < H ? e : (f < Q * H + Q ? col_dp + q : -1);
        ca[k] = (e >= H && f < Q * H) ? col_a + (f - q * H) : -1;
    }
    double lsum = 0.0;
    __syncthreads();

    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    const int64_t ntiles = ceil_div(p.B, kRows);
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t row = tile * kRows + threadIdx.x;
        const bool valid = row < p.B;
        float a[MAXHP], dz[MAXHP], dp[MAXQ];
        // an opaque zero per tile keeps the weight reads inside the loop (hoisted, the 2 x 2401 LDS values of C5
        // would be held in registers across tiles and spill)
        int opaque;
        asm volatile("s_mov_b32 %0, 0" : "=s"(opaque));
        const float* wpt = wp + (opaque & ~3);  // (a multiple of 4 floats: 16-byte LDS reads stay possible)
        const float* wtt = wt + (opaque & ~3);
        // ---- forward + loss + backward to dz for this thread's row (the state row is dead afterwards: the
        // reduction reloads it, so that only a and dz stay in registers there)
        {
            float x[INP];
            load_state<INP, EXACT>(p, row, valid, in, x);
            float t[MAXQ];
            if (own_target) {  // target first: only x and t are live meanwhile
                float zt[MAXHP];
                rnd_hidden_t<INP, MAXHP, EXACT>(wtt, in, x, zt);
#pragma unroll
                for (int h = 0; h < MAXHP; ++h) zt[h] = rnd_elu(zt[h]);
                rnd_output<INP, MAXHP, MAXQ>(wtt, Q, zt, t);
                if (p.temb && valid) {
#pragma unroll
                    for (int q = 0; q < MAXQ; ++q)
                        if (q < Q) p.temb[row * Q + q] = t[q];
                }
            } else {
#pragma unroll
                for (int q = 0; q < MAXQ; ++q) t[q] = (q < Q && valid) ? p.temb[row * Q + q] : 0.f;
            }
            float z[MAXHP];
            rnd_hidden_t<INP, MAXHP, EXACT>(wpt, in, x, z);
#pragma unroll
            for (int h = 0; h < MAXHP; ++h) {
                rnd_elu_and_grad(z[h], a[h], dz[h]);
            }
            float y[MAXQ];
            rnd_output<INP, MAXHP, MAXQ>(wpt, Q, a, y);
            float l = 0.f;
#pragma unroll
            for (int q = 0; q < MAXQ; ++q) {
                const float d = __fsub_rn(y[q], t[q]);
                dp[q] = (q < Q && valid) ? __fmul_rn(p.norm, d) : 0.f;
                if (q < Q) l = __fadd_rn(l, __fmul_rn(d, d));
            }
            lsum += valid ? static_cast<double>(l) : 0.0;
            // da[h] = sum_q w2[q][h] dp[q]; dz = da * ELU'(z)  (dz[] holds ELU'(z) on entry; padded units have
            // zero output weights -> dz 0)
            const float* w2 = wpt + MAXHP * INP + MAXHP;
#pragma unroll
            for (int h = 0; h < MAXHP; ++h) {
                float da = 0.f;
#pragma unroll
                for (int q = 0; q < MAXQ; ++q)
                    if (q < Q) da = fmaf(w2[q * MAXHP + h], dp[q], da);
                dz[h] = valid ? __fmul_rn(da, dz[h]) : 0.f;
            }
        }
        // ---- reduction: wave w's rows through the LDS chunk, every thread adds them into its entries.  The state
        // row is reloaded (L2) here, before the first barrier, so that its latency is not waited out by the other
        // waves at the barrier of this wave's turn
        float x[INP];
        load_state<INP, EXACT>(p, row, valid, in, x);
        for (int w = 0; w < kBlock / kWave; ++w) {
            if (wid == w) {  // column-major: lane = row -> consecutive addresses per column
#pragma unroll
                for (int h = 0; h < MAXHP; ++h) {
                    chunk[h * kColStride + lane] = dz[h];
                    chunk[(col_a + h) * kColStride + lane] = a[h];
                }
#pragma unroll
                for (int i = 0; i < INP; ++i)
                    if (i < in) chunk[(col_x + i) * kColStride + lane] = x[i];
#pragma unroll
                for (int q = 0; q < MAXQ; ++q)
                    if (q < Q) chunk[(col_dp + q) * kColStride + lane] = dp[q];
            }
            __syncthreads();
#pragma unroll 2
            for (int r4 = 0; r4 < kChunk; r4 += 4) {  // 4 rows per step: one 16-byte read per column
                float4 zv[BH], xv[BI];
#pragma unroll
                for (int u = 0; u < BH; ++u)
                    zv[u] = *reinterpret_cast<const float4*>(chunk + (tr * BH + u) * kColStride + r4);
#pragma unroll
                for (int v = 0; v < BI; ++v)
                    xv[v] = (tc * BI + v < in) ? *reinterpret_cast<const float4*>(chunk + (col_x + tc * BI + v) * kColStride + r4)
                                               : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int u = 0; u < BH; ++u) {
#pragma unroll
                    for (int v = 0; v < BI; ++v) {  // rows (r, r+1) then (r+2, r+3) into the even / odd sums
                        g1[u][v] = __builtin_elementwise_fma(f32x2_t{zv[u].x, zv[u].y}, f32x2_t{xv[v].x, xv[v].y}, g1[u][v]);
                        g1[u][v] = __builtin_elementwise_fma(f32x2_t{zv[u].z, zv[u].w}, f32x2_t{xv[v].z, xv[v].w}, g1[u][v]);
                    }
                }
#pragma unroll
                for (int k = 0; k < kExtra; ++k) {
                    if (cq[k] >= 0) {
                        const float4 d4 = *reinterpret_cast<const float4*>(chunk + cq[k] * kColStride + r4);
                        const float4 a4 = ca[k] >= 0 ? *reinterpret_cast<const float4*>(chunk + ca[k] * kColStride + r4)
                                                     : make_float4(1.f, 1.f, 1.f, 1.f);
                        gx[k] = __builtin_elementwise_fma(f32x2_t{d4.x, d4.y}, f32x2_t{a4.x, a4.y}, gx[k]);
                        gx[k] = __builtin_elementwise_fma(f32x2_t{d4.z, d4.w}, f32x2_t{a4.z, a4.w}, gx[k]);
                    }
                }
            }
            __syncthreads();
        }
    }

    // ---- per-workgroup partials [dW1 | db1 | dW2 | db2]
    float* part = p.partials + static_cast<int64_t>(blockIdx.x) * p.P;
#pragma unroll
    for (int u = 0; u < BH; ++u) {
        const int h = tr * BH + u;
        if (h < H) {
#pragma unroll
            for (int v = 0; v < BI; ++v) {
                const int i = tc * BI + v;
                if (i < in) part[h * in + i] = __fadd_rn(g1[u][v].x, g1[u][v].y);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kExtra; ++k) {
        const int e = threadIdx.x + k * kBlock;
        if (e < H + Q * H + Q) part[H * in + e] = __fadd_rn(gx[k].x, gx[k].y);
    }
    __shared__ double scratch[kBlock / kWave];
    const double ls = block_sum(lsum, scratch);
    if (threadIdx.x == 0) p.lpart[blockIdx.x] = ls;
}

// grad[e] = fp32(sum over workgroups g, in order, of partials[g][e]) -- 16 slices of the workgroups per entry
// (one wave each, 64 entries per block), then the slices in order; block 0 also folds the loss.
__global__ __launch_bounds__(1024) void rnd_fold_kernel(const float* __restrict__ partials, const double* __restrict__ lpart,
                                                        int G, int P, float* __restrict__ grad, double inv_numel,
                                                        double* loss_sum, float* loss) {
    __shared__ double sl[kFoldSlices][kWave];
    const int lane = threadIdx.x & (kWave - 1);
    const int s = threadIdx.x / kWave;
    const int e = blockIdx.x * kWave + lane;
    constexpr int kPer = kMaxGroups / kFoldSlices;  // partials per thread (G <= kMaxGroups)
    const int g0 = s * kPer;
    double acc = 0.0;
    if (e < P) {
        // every load in flight at once, then the adds in workgroup order (one memory round trip)
        float v[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) v[k] = g0 + k < G ? partials[static_cast<int64_t>(g0 + k) * P + e] : 0.f;
#pragma unroll
        for (int k = 0; k < kPer; ++k) acc += static_cast<double>(v[k]);
    }
    sl[s][lane] = acc;
    __syncthreads();
    if (s == 0 && e < P) {
        double t = sl[0][lane];
#pragma unroll
        for (int k = 1; k < kFoldSlices; ++k) t += sl[k][lane];
        grad[e] = static_cast<float>(t);
    }
    if (blockIdx.x == 0) {  // the loss: G <= kMaxGroups partials over the first waves, then waves in order
        __shared__ double wl[kFoldSlices];
        double t = threadIdx.x < static_cast<unsigned>(G) ? lpart[threadIdx.x] : 0.0;
        t = wave_sum(t);
        if (lane == 0) wl[s] = t;
        __syncthreads();
        if (threadIdx.x == 0) {
            double tot = 0.0;
#pragma unroll
            for (int k = 0; k < kFoldSlices; ++k) tot += wl[k];
            const float mse = static_cast<float>(tot * inv_numel);
            if (loss) *loss = mse;
            if (loss_sum) *loss_sum += static_cast<double>(mse);
        }
    }
}

int groups_for(int64_t B) { return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(ceil_div(B, kRows), kMaxGroups))); }

template <int INP, int MAXHP, int MAXQ, bool EXACT>
int launch(const RndParams& p, int G, bool own_target, hipStream_t st) {
    const int nw = rnd_net_floats(INP, MAXHP, p.Q);
    const int cols = 2 * MAXHP + p.in + p.Q;
    const size_t lds = sizeof(float) * (static_cast<size_t>(own_target ? 2 * nw : nw) + static_cast<size_t>(cols) * kColStride);
    auto k = rnd_update_kernel<INP, MAXHP, MAXQ, EXACT>;
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
        if (e != hipSuccess) return static_cast<int>(e);
    }
    hipLaunchKernelGGL(k, dim3(G), dim3(kBlock), lds, st, p);
    return launch_status();
}

}  // namespace
}  // namespace rslrl

using namespace rslrl;

extern "C" size_t rslrl_rnd_update_workspace_bytes(int64_t B, int32_t in, int32_t hidden, int32_t out) {
    const size_t P = static_cast<size_t>(hidden) * in + hidden + static_cast<size_t>(out) * hidden + out;
    const size_t G = static_cast<size_t>(groups_for(B));
    return align_up(G * P * sizeof(float), 256) + G * sizeof(double);
}

extern "C" int rslrl_rnd_update(const rslrl_rnd_update_args_t* a, void* workspace, size_t workspace_bytes,
                                rslrl_stream_t stream) {
    if (!a) return RSLRL_E_INVALID_ARGUMENT;
    if (a->B < 1 || a->in < 1 || a->in > RSLRL_RND_MAX_IN || a->hidden < 1 || a->hidden > RSLRL_RND_MAX_HIDDEN ||
        a->out < 1 || a->out > RSLRL_RND_MAX_OUT)
        return RSLRL_E_INVALID_ARGUMENT;
    if (!a->state || a->state_stride < a->in || !a->pred_w1 || !a->pred_b1 || !a->pred_w2 || !a->pred_b2 || !a->grad)
        return RSLRL_E_INVALID_ARGUMENT;
    if ((a->state_mean == nullptr) != (a->state_std == nullptr)) return RSLRL_E_INVALID_ARGUMENT;
    if (a->target_w1 && (!a->target_b1 || !a->target_w2 || !a->target_b2)) return RSLRL_E_INVALID_ARGUMENT;
    if (!a->target_w1 && !a->target_embedding) return RSLRL_E_INVALID_ARGUMENT;
    if (!workspace) return RSLRL_E_INVALID_ARGUMENT;
    if (workspace_bytes < rslrl_rnd_update_workspace_bytes(a->B, a->in, a->hidden, a->out))
        return RSLRL_E_WORKSPACE_TOO_SMALL;
    if (reinterpret_cast<uintptr_t>(workspace) & 15) return RSLRL_E_MISALIGNED;
    const int G = groups_for(a->B);
    RndParams p{};
    p.B = a->B;
    p.in = a->in;
    p.H = a->hidden;
    p.Q = a->out;
    p.eps = a->state_eps;
    p.state = a->state;
    p.stride = a->state_stride;
    p.mean = a->state_mean;
    p.std = a->state_std;
    p.pw[0] = a->pred_w1, p.pw[1] = a->pred_b1, p.pw[2] = a->pred_w2, p.pw[3] = a->pred_b2;
    p.tw[0] = a->target_w1, p.tw[1] = a->target_b1, p.tw[2] = a->target_w2, p.tw[3] = a->target_b2;
    p.temb = a->target_embedding;
    // torch mse_loss_backward: norm = 2. / numel (double), applied as a scalar of the input's dtype
    p.norm = static_cast<float>(2.0 / static_cast<double>(a->B * a->out));
    p.P = a->hidden * a->in + a->hidden + a->out * a->hidden + a->out;
    p.partials = static_cast<float*>(workspace);
    p.lpart = reinterpret_cast<double*>(static_cast<char*>(workspace) +
                                        align_up(static_cast<size_t>(G) * p.P * sizeof(float), 256));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const bool own = a->target_w1 != nullptr;
    int rc;
    const bool aligned_rows = (reinterpret_cast<uintptr_t>(a->state) & 15) == 0 && (a->state_stride & 3) == 0;
    if (a->in == 48 && a->hidden == 48 && a->out == 1 && aligned_rows)  // config C5
        rc = launch<48, 48, 1, true>(p, G, own, st);
    else if (a->in <= 16 && a->hidden <= 32 && a->out <= 4)
        rc = launch<16, 32, 4, false>(p, G, own, st);
    else
        rc = launch<64, 64, 8, false>(p, G, own, st);
    if (rc != RSLRL_OK) return rc;
    hipLaunchKernelGGL(rnd_fold_kernel, dim3(static_cast<unsigned>(ceil_div(p.P, kWave))), dim3(kWave * kFoldSlices), 0,
                       st, p.partials, p.lpart, G, p.P, a->grad, 1.0 / static_cast<double>(a->B * a->out), a->loss_sum,
                       a->loss);
    return launch_status();
}
