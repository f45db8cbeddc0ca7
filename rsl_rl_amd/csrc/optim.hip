// Gradient-norm clipping + Adam step of PPO.update (rsl_rl/algorithms/ppo.py:373-374:
// nn.utils.clip_grad_norm_(policy.parameters(), max_grad_norm); optimizer.step()) in two launches over the
// parameter list, replacing ~10 torch launches (per-tensor norms, norm of norms, clamp, reciprocal, foreach
// multiply) and torch's fused Adam.
//
// Adam follows torch's fused CUDA kernel (ATen/native/cuda/fused_adam_utils.cuh) operation for operation:
// step += 1 first; bias corrections 1 - beta^step in double, passed on as fp32; the moment updates evaluated
// as one double fma from fp32 operands and rounded to fp32; step_size = fp32(lr / bc1); denom = fp32(double(sqrtf(v) /
// bc2_sqrt) + eps) with the division in fp32; param -= step_size * m / denom in fp32.  Clipping: coef = max_norm / (||g||_2 + 1e-6),
// clamped to <= 1 (a NaN norm stays NaN), g = fp32(g * coef) as torch's foreach multiply, written back to
// .grad as clip_grad_norm_ leaves it; the norm is accumulated in fp64 in a fixed
// order (torch's per-tensor fp32 norms differ from it in the last bit at most).
#include "common.h"

namespace rslrl {
namespace {

constexpr int kBlocks = 512;  // fixed partition of the concatenated elements (deterministic order); 512 blocks
                              // keep ~2 elements per thread at C3's 290k parameters (128: ~9 dependent
                              // iterations per thread, 19-20 us per launch)
constexpr int kThreadsA = 256;

struct Span {
    int64_t begin, end;  // this block's elements of the concatenation
};

__device__ __forceinline__ Span block_span(int64_t total) {
    const int64_t per = (total + kBlocks - 1) / kBlocks;
    const int64_t b = static_cast<int64_t>(blockIdx.x) * per;
    return {b < total ? b : total, b + per < total ? b + per : total};
}

// workspace: [0, kTicketBytes) arrival tickets (u32, zero before and after: the grid's at 0, group g's at
// 128 (g + 1) -- each on a line of its own), fp64 partials [kBlocks], fp32 coef, then per tensor {bc1, bc2 sqrt,
// step size} (written by grad_sq_kernel's last block after it advanced the step counters, read by adam_kernel)
constexpr int kTicketGroup = 64;  // blocks per arrival group: at most 64 atomics queue on one word (512 on one word
                                  // was most of this launch's time, and of round 5's one-launch Adam)
constexpr int kTicketBytes = 128 * (kBlocks / kTicketGroup + 1);
constexpr size_t kPartOff = kTicketBytes;
constexpr size_t kCoefOff = kPartOff + kBlocks * sizeof(double);
constexpr size_t kConstOff = kCoefOff + 256;
constexpr size_t kAdamWsBytes = kConstOff + 3 * sizeof(float) * RSLRL_ADAM_MAX_TENSORS;

// the per-mini-batch tail of PPO.update (ppo_loss.hip ppo_tail_kernel's expressions; ppo.py:259-294, :387-395), run
// by one thread of the norm launch's block 0 when fused in (rslrl_clip_adam_step_tail)
__device__ __forceinline__ void ppo_tail_device(const rslrl_ppo_tail_t& t, float* lr32_out) {
    if (t.lr) {
        const float kl = *t.kl;
        double v = *t.lr;
        if (kl > t.kl_hi) {
            v = fmax(v / 1.5, 1e-5);
        } else if (kl < t.kl_lo && kl > 0.0f) {
            v = fmin(v * 1.5, 1e-2);
        }
        if (t.round_fp32) v = static_cast<double>(static_cast<float>(v));
        *t.lr = v;
        *t.lr32 = static_cast<float>(v);
        *lr32_out = static_cast<float>(v);
    }
    if (t.sums) {
        t.sums[0] += static_cast<double>(t.stats[2]);
        t.sums[1] += static_cast<double>(t.stats[1]);
        t.sums[2] += static_cast<double>(t.stats[3]);
    }
}

__global__ __launch_bounds__(kThreadsA) void grad_sq_kernel(rslrl_adam_args_t a, unsigned* ticket, double* part,
                                                            float* coef, float* consts, rslrl_ppo_tail_t tail,
                                                            int with_tail) {
    __shared__ double scratch[kThreadsA / kWave];
    __shared__ int last;
    __shared__ float tail_lr32;
    // torch: _foreach_add_(state_steps, 1) before the update -- block 0, one lane per tensor, all in flight at once,
    // off the grid's critical path (the last block only folds the norm); on the same lane that tensor's bias
    // corrections and step size for adam_kernel (fused_adam_utils.cuh's expressions, once per tensor instead of once
    // per block and tensor).  adam_kernel reads neither the counters nor these before this launch has ended.
    if (blockIdx.x == 0) {
        // the lr rule first: the step sizes below take the lr it wrote (handed over in LDS)
        const bool tail_lr = with_tail && tail.lr && a.lr_dev == tail.lr32;
        if (with_tail) {
            if (threadIdx.x == 0) ppo_tail_device(tail, &tail_lr32);
            __syncthreads();
        }
        float* sp = nullptr;
#pragma unroll
        for (int i = 0; i < RSLRL_ADAM_MAX_TENSORS; ++i)
            if (static_cast<int>(threadIdx.x) == i) sp = a.t[i].step;
        if (static_cast<int>(threadIdx.x) < a.n) {
            const float st1 = *sp + 1.0f;
            *sp = st1;
            const double step = static_cast<double>(st1);
            const double lr = tail_lr  ? static_cast<double>(tail_lr32)
                              : a.lr_dev ? static_cast<double>(*a.lr_dev)
                                         : a.lr;
            const float bc1 = static_cast<float>(1.0 - pow(static_cast<double>(a.beta1), step));
            const float bc2s = static_cast<float>(sqrt(1.0 - pow(static_cast<double>(a.beta2), step)));
            consts[3 * threadIdx.x] = bc1;
            consts[3 * threadIdx.x + 1] = bc2s;
            consts[3 * threadIdx.x + 2] = static_cast<float>(lr / static_cast<double>(bc1));
        }
    }
    const int64_t total = a.offsets[a.n];
    const Span sp = block_span(total);
    double s = 0.0;
    // tensors in order, each clipped to the block's span: the tensor index is wave-uniform, so its pointer and
    // offsets are scalar loads (a per-lane index into the argument block made every element wait on a load
    // chain)
    for (int ti = 0; ti < a.n; ++ti) {
        const int64_t o0 = a.offsets[ti], o1 = a.offsets[ti + 1];
        const int64_t lo = sp.begin > o0 ? sp.begin : o0, hi = sp.end < o1 ? sp.end : o1;
        const float* __restrict__ g = a.t[ti].grad - o0;
        for (int64_t e = lo + threadIdx.x; e < hi; e += kThreadsA) {
            const float v = g[e];
            s += static_cast<double>(v) * static_cast<double>(v);
        }
    }
    // block sum in a fixed order (wave butterflies, then waves in order)
    s = wave_sum(s);
    if ((threadIdx.x & (kWave - 1)) == 0) scratch[threadIdx.x / kWave] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double bsum = 0.0;
        for (int w = 0; w < kThreadsA / kWave; ++w) bsum += scratch[w];
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(part + blockIdx.x), __double_as_longlong(bsum),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // two-level arrival: the group's last block takes the grid's ticket
        const unsigned grp = blockIdx.x / kTicketGroup;
        const unsigned gsize = min(static_cast<unsigned>(kTicketGroup), gridDim.x - grp * kTicketGroup);
        unsigned* gt = ticket + 32 * (grp + 1);
        int l = 0;
        if (__hip_atomic_fetch_add(gt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
            __hip_atomic_store(gt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned ng = (gridDim.x + kTicketGroup - 1) / kTicketGroup;
            l = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
        }
        last = l;
    }
    __syncthreads();
    if (!last) return;
    // the last block folds the kBlocks partials in a fixed order: kBlocks / kThreadsA per thread (all loads in
    // flight at once, added in index order), wave butterflies, then the waves in order
    static_assert(kBlocks % kThreadsA == 0, "whole partials per thread");
    constexpr int kPer = kBlocks / kThreadsA;
    double pl[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k)
        pl[k] = __longlong_as_double(__hip_atomic_load(
            reinterpret_cast<unsigned long long*>(part + threadIdx.x + k * kThreadsA), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_AGENT));
    double pv = pl[0];
#pragma unroll
    for (int k = 1; k < kPer; ++k) pv += pl[k];
    pv = wave_sum(pv);
    __syncthreads();  // scratch is reused
    if ((threadIdx.x & (kWave - 1)) == 0) scratch[threadIdx.x / kWave] = pv;
    __syncthreads();
    if (threadIdx.x != 0) return;
    double tot = 0.0;
    for (int w = 0; w < kThreadsA / kWave; ++w) tot += scratch[w];
    float c = 1.0f;
    if (a.max_grad_norm > 0.0f) {
        const float norm = static_cast<float>(sqrt(tot));
        const float cf = a.max_grad_norm / (norm + 1e-6f);
        // torch.clamp(clip_coef, max=1.0) propagates a NaN norm (every gradient then becomes NaN, as in torch)
        c = isnan(cf) ? cf : fminf(cf, 1.0f);
    }
    *coef = c;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kThreadsA) void adam_kernel(rslrl_adam_args_t a, const float* __restrict__ coef,
                                                         const float* __restrict__ consts) {
    const int64_t total = a.offsets[a.n];
    const Span sp = block_span(total);
    const float c = *coef;
    const double b1 = a.beta1, b2 = a.beta2, eps = a.eps;
    // tensors in order, clipped to the block's span (wave-uniform tensor index: scalar pointer loads)
    for (int ti = 0; ti < a.n; ++ti) {
        const int64_t o0 = a.offsets[ti], o1 = a.offsets[ti + 1];
        const int64_t lo = sp.begin > o0 ? sp.begin : o0, hi = sp.end < o1 ? sp.end : o1;
        if (lo >= hi) continue;
        const rslrl_adam_tensor_t t = a.t[ti];
        const float bc2s = consts[3 * ti + 1];
        const float step_size = consts[3 * ti + 2];
        for (int64_t e = lo + threadIdx.x; e < hi; e += kThreadsA) {
            const int64_t i = e - o0;
            const float g = t.grad[i] * c;  // the clipped gradient (fp32 multiply, as torch's foreach mul)
            t.grad[i] = g;  // clip_grad_norm_ scales .grad in place: after the step .grad holds the clipped values
            // torch's build contracts b*m + (1-b)*g into one double fma; the unfused sum rounds differently in
            // ~0.3% of elements once narrowed to fp32 (measured), so the fma is spelled out here
            const double gd = static_cast<double>(g);
            const float m = static_cast<float>(fma(b1, static_cast<double>(t.exp_avg[i]), (1.0 - b1) * gd));
            const float v = static_cast<float>(fma(b2, static_cast<double>(t.exp_avg_sq[i]), (1.0 - b2) * gd * gd));
            const float q = sqrtf(v) / bc2s;  // fp32 division, then the double eps add (fused_adam_utils.cuh:77)
            const float denom = static_cast<float>(static_cast<double>(q) + eps);
            t.exp_avg[i] = m;
            t.exp_avg_sq[i] = v;
            t.param[i] = t.param[i] - step_size * m / denom;
        }
    }
}

}  // namespace
}  // namespace rslrl

using namespace rslrl;

extern "C" size_t rslrl_adam_workspace_bytes(void) { return kAdamWsBytes; }

namespace {
int clip_adam(const rslrl_adam_args_t* args, const rslrl_ppo_tail_t* tail, void* workspace, size_t workspace_bytes,
              rslrl_stream_t stream) {
    if (!args || !workspace || args->n < 1 || args->n > RSLRL_ADAM_MAX_TENSORS) return RSLRL_E_INVALID_ARGUMENT;
    if (tail && (!tail->stats || (tail->lr && (!tail->lr32 || !tail->kl)))) return RSLRL_E_INVALID_ARGUMENT;
    const rslrl_ppo_tail_t no_tail{};
    if (workspace_bytes < rslrl_adam_workspace_bytes()) return RSLRL_E_WORKSPACE_TOO_SMALL;
    rslrl_adam_args_t a = *args;
    int64_t off = 0;
    for (int i = 0; i < a.n; ++i) {
        const rslrl_adam_tensor_t& t = a.t[i];
        if (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq || !t.step || t.numel < 0) return RSLRL_E_INVALID_ARGUMENT;
        a.offsets[i] = off;
        off += t.numel;
    }
    a.offsets[a.n] = off;  // all-empty tensors still advance the step counters (torch increments them too)
    char* ws = static_cast<char*>(workspace);
    unsigned* ticket = reinterpret_cast<unsigned*>(ws);
    double* part = reinterpret_cast<double*>(ws + kPartOff);
    float* coef = reinterpret_cast<float*>(ws + kCoefOff);
    float* consts = reinterpret_cast<float*>(ws + kConstOff);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(grad_sq_kernel, dim3(kBlocks), dim3(kThreadsA), 0, st, a, ticket, part, coef, consts,
                       tail ? *tail : no_tail, tail ? 1 : 0);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(adam_kernel, dim3(kBlocks), dim3(kThreadsA), 0, st, a, coef, consts);
    return launch_status();
}
}  // namespace

extern "C" int rslrl_clip_adam_step(const rslrl_adam_args_t* args, void* workspace, size_t workspace_bytes,
                                    rslrl_stream_t stream) {
    return clip_adam(args, nullptr, workspace, workspace_bytes, stream);
}

extern "C" int rslrl_clip_adam_step_tail(const rslrl_adam_args_t* args, const rslrl_ppo_tail_t* tail,
                                         void* workspace, size_t workspace_bytes, rslrl_stream_t stream) {
    if (!tail) return RSLRL_E_INVALID_ARGUMENT;
    return clip_adam(args, tail, workspace, workspace_bytes, stream);
}
