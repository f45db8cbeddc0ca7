// Running observation / reward normalisers, rsl_rl/networks/normalization.py:
//   EmpiricalNormalization.update (:44-66): count += n; rate = n / count; (mean_x, var_x) = batch moments
//     (population variance); delta = mean_x - mean; mean += rate * delta;
//     var += rate * (var_x - var + delta * (mean_x - mean)); std = sqrt(var)     -- skipped once count >= until
//   EmpiricalNormalization.forward (:40-42): (x - mean) / (std + eps)
//   EmpiricalDiscountedVariationNormalization.forward (:84-99): avg = avg * gamma + r (the discounted sum,
//     _DiscountedAverage :108-130), update(avg), then r / std when std > 0
//
// Batch moments: per-workgroup fp64 (sum, sum of squares) per column over a slice of rows, folded in a fixed
// order by one workgroup which also applies the running update with the reference's fp32 operation order
// (torch's own reductions round differently; the moments agree to fp32 rounding).  The `until` test reads
// the device-side count, so no host synchronisation is needed (the reference's `if count >= until` syncs).
#include <algorithm>

#include "common.h"

namespace rslrl {
namespace {

constexpr int kMaxCols = 256;
constexpr int kRowsPerBlock = 1024;

// partial[blk][c] = (sum x, sum x^2) over rows [blk * kRowsPerBlock, ...) of column c.  Thread layout:
// 256 threads = (256 / D') row lanes x D' columns, D' = D rounded up to a power of two <= 256.
__global__ __launch_bounds__(kBlock) void col_moments_kernel(const float* __restrict__ x, int64_t N, int D,
                                                             int64_t row_stride, int dpow, double2* __restrict__ part) {
    __shared__ double2 red[kBlock];
    const int c = threadIdx.x % dpow;
    const int lane_rows = kBlock / dpow;
    const int rl = threadIdx.x / dpow;
    const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kRowsPerBlock;
    const int64_t r1 = std::min<int64_t>(N, r0 + kRowsPerBlock);
    double s = 0.0, ss = 0.0;
    if (c < D) {
        for (int64_t r = r0 + rl; r < r1; r += lane_rows) {
            const double v = x[r * row_stride + c];
            s += v;
            ss += v * v;
        }
    }
    red[threadIdx.x] = make_double2(s, ss);
    __syncthreads();
    if (threadIdx.x < dpow) {  // fixed-order fold over the row lanes of this column
        double2 acc = red[threadIdx.x];
        for (int k = 1; k < lane_rows; ++k) {
            const double2 t = red[k * dpow + threadIdx.x];
            acc.x += t.x;
            acc.y += t.y;
        }
        if (threadIdx.x < D) part[static_cast<int64_t>(blockIdx.x) * D + threadIdx.x] = acc;
    }
}

// one workgroup: fold the partials (block order), moments in fp64 -> fp32, then the running update
__global__ __launch_bounds__(kBlock) void normalizer_update_kernel(const double2* __restrict__ part, int nblk, int64_t N,
                                                                   int D, float* __restrict__ mean,
                                                                   float* __restrict__ var, float* __restrict__ stdv,
                                                                   int64_t* __restrict__ count, int64_t until) {
    const int64_t cnt0 = *count;
    if (until >= 0 && cnt0 >= until) return;
    __syncthreads();  // every thread has read the old count before thread 0 writes it
    const int64_t cnt = cnt0 + N;
    // rate = n / count: torch true-divides the int64 tensor in the default float type
    const float rate = __fdiv_rn(static_cast<float>(N), static_cast<float>(cnt));
    for (int c = threadIdx.x; c < D; c += kBlock) {
        double s = 0.0, ss = 0.0;
        for (int b = 0; b < nblk; ++b) {
            const double2 t = part[static_cast<int64_t>(b) * D + c];
            s += t.x;
            ss += t.y;
        }
        const double m = s / static_cast<double>(N);
        double v = ss / static_cast<double>(N) - m * m;
        if (v < 0.0) v = 0.0;
        const float mean_x = static_cast<float>(m);
        const float var_x = static_cast<float>(v);
        const float mu = mean[c];
        const float delta = __fsub_rn(mean_x, mu);
        const float mu_new = __fadd_rn(mu, __fmul_rn(rate, delta));
        const float vr = var[c];
        const float inner = __fadd_rn(__fsub_rn(var_x, vr), __fmul_rn(delta, __fsub_rn(mean_x, mu_new)));
        const float var_new = __fadd_rn(vr, __fmul_rn(rate, inner));
        mean[c] = mu_new;
        var[c] = var_new;
        stdv[c] = __fsqrt_rn(var_new);
    }
    if (threadIdx.x == 0) *count = cnt;
}

__global__ __launch_bounds__(kBlock) void normalizer_apply_kernel(const float* __restrict__ x, int64_t N, int D,
                                                                  int64_t row_stride, const float* __restrict__ mean,
                                                                  const float* __restrict__ stdv, float eps,
                                                                  float* __restrict__ y) {
    const int64_t total = N * D;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < total;
         i += static_cast<int64_t>(gridDim.x) * kBlock) {
        const int64_t r = i / D;
        const int c = static_cast<int>(i - r * D);
        y[i] = __fdiv_rn(__fsub_rn(x[r * row_stride + c], mean[c]), __fadd_rn(stdv[c], eps));
    }
}

// reward normaliser, stage 1: avg = first ? r : avg * gamma + r (in place), then moments of avg
__global__ __launch_bounds__(kBlock) void disc_avg_kernel(const float* __restrict__ r, int64_t N, float gamma,
                                                          int first, float* __restrict__ avg) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < N;
         i += static_cast<int64_t>(gridDim.x) * kBlock)
        avg[i] = first ? r[i] : __fadd_rn(__fmul_rn(avg[i], gamma), r[i]);
}

// reward normaliser, stage 3: out = r / std when std > 0 else r (normalization.py:96-99)
__global__ __launch_bounds__(kBlock) void reward_scale_kernel(const float* __restrict__ r, int64_t N,
                                                              const float* __restrict__ stdv, float* __restrict__ out) {
    const float s = stdv[0];
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < N;
         i += static_cast<int64_t>(gridDim.x) * kBlock)
        out[i] = s > 0.f ? __fdiv_rn(r[i], s) : r[i];
}

int pow2_at_least(int d) {
    int p = 1;
    while (p < d) p <<= 1;
    return p;
}

int launch_moments_update(const float* x, int64_t N, int D, int64_t row_stride, float* mean, float* var, float* stdv,
                          int64_t* count, int64_t until, void* ws, size_t ws_bytes, hipStream_t st) {
    const int64_t nblk = ceil_div(N, kRowsPerBlock);
    if (ws_bytes < static_cast<size_t>(nblk) * D * sizeof(double2)) return RSLRL_E_WORKSPACE_TOO_SMALL;
    double2* part = static_cast<double2*>(ws);
    hipLaunchKernelGGL(col_moments_kernel, dim3(static_cast<unsigned>(nblk)), dim3(kBlock), 0, st, x, N, D, row_stride,
                       pow2_at_least(D), part);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(normalizer_update_kernel, dim3(1), dim3(kBlock), 0, st, part, static_cast<int>(nblk), N, D, mean,
                       var, stdv, count, until);
    return launch_status();
}

unsigned grid_for(int64_t n) { return static_cast<unsigned>(std::min<int64_t>(4096, std::max<int64_t>(1, ceil_div(n, kBlock)))); }

}  // namespace
}  // namespace rslrl

using namespace rslrl;

extern "C" size_t rslrl_normalizer_workspace_bytes(int64_t N, int32_t D) {
    if (N < 1 || D < 1) return 0;
    return static_cast<size_t>(ceil_div(N, kRowsPerBlock)) * D * sizeof(double2);
}

extern "C" int rslrl_normalizer_update(const float* x, int64_t N, int32_t D, int64_t row_stride, float* mean,
                                       float* var, float* stdv, int64_t* count, int64_t until, void* workspace,
                                       size_t workspace_bytes, rslrl_stream_t stream) {
    if (N < 0 || D < 1 || D > kMaxCols || row_stride < D) return RSLRL_E_INVALID_ARGUMENT;
    if (N == 0) return RSLRL_OK;
    if (!x || !mean || !var || !stdv || !count || !workspace) return RSLRL_E_INVALID_ARGUMENT;
    return launch_moments_update(x, N, D, row_stride, mean, var, stdv, count, until, workspace, workspace_bytes,
                                 reinterpret_cast<hipStream_t>(stream));
}

extern "C" int rslrl_normalizer_apply(const float* x, int64_t N, int32_t D, int64_t row_stride, const float* mean,
                                      const float* stdv, float eps, float* y, rslrl_stream_t stream) {
    if (N < 0 || D < 1 || row_stride < D) return RSLRL_E_INVALID_ARGUMENT;
    if (N == 0) return RSLRL_OK;
    if (!x || !mean || !stdv || !y) return RSLRL_E_INVALID_ARGUMENT;
    hipLaunchKernelGGL(normalizer_apply_kernel, dim3(grid_for(N * D)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), x, N, D, row_stride, mean, stdv, eps, y);
    return launch_status();
}

extern "C" int rslrl_reward_normalize(const float* rewards, int64_t N, float gamma, float* disc_avg, int32_t first,
                                      float* mean, float* var, float* stdv, int64_t* count, int64_t until,
                                      int32_t training, float* out, void* workspace, size_t workspace_bytes,
                                      rslrl_stream_t stream) {
    if (N < 0) return RSLRL_E_INVALID_ARGUMENT;
    if (N == 0) return RSLRL_OK;
    if (!rewards || !stdv || !out || (training && (!disc_avg || !mean || !var || !count || !workspace)))
        return RSLRL_E_INVALID_ARGUMENT;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (training) {
        hipLaunchKernelGGL(disc_avg_kernel, dim3(grid_for(N)), dim3(kBlock), 0, st, rewards, N, gamma, first, disc_avg);
        int rc = launch_status();
        if (rc) return rc;
        // the discounted sums are a [N] batch of a scalar quantity (shape [] -> D = 1)
        rc = launch_moments_update(disc_avg, N, 1, 1, mean, var, stdv, count, until, workspace, workspace_bytes, st);
        if (rc) return rc;
    }
    hipLaunchKernelGGL(reward_scale_kernel, dim3(grid_for(N)), dim3(kBlock), 0, st, rewards, N, stdv, out);
    return launch_status();
}
