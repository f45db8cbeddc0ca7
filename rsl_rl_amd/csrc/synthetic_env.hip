// The synthetic VecEnv of the benchmark (random observations, rewards and dones of the stated shape)
// as one launch per env step -- the environment a PPO iteration is timed against, not part of the PPO hot path.
//
// Per env n at step s (counter-based: philox4x32-10 keyed by the env's seed, counter (s, n, block, 0)):
//   obs[n, :]   ~ N(0, 1)   (Box-Muller on philox uniforms, 4 values per 16-byte store)
//   reward[n]   ~ N(0, 1),  u ~ U(0, 1)
//   ep[n] += 1;  over = ep[n] >= max_episode_length
//   done[n]      = over or u < done_prob                                   (int64)
//   time_out[n]  = over or u < done_prob * timeout_prob                    (fp32)
//   ep[n]        = done ? 0 : ep[n]
// (the semantics of env/synthetic.py's torch implementation, which CPU tensors keep using).
#include <algorithm>

#include "common.h"

namespace rslrl {
namespace {

struct U4 {
    uint32_t x, y, z, w;
};

// philox4x32-10 (Salmon et al., SC'11)
__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = static_cast<uint64_t>(0xD2511F53u) * c.x;
        const uint64_t p1 = static_cast<uint64_t>(0xCD9E8D57u) * c.z;
        const uint32_t hi0 = static_cast<uint32_t>(p0 >> 32), lo0 = static_cast<uint32_t>(p0);
        const uint32_t hi1 = static_cast<uint32_t>(p1 >> 32), lo1 = static_cast<uint32_t>(p1);
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// uniform in (0, 1] from 24 random bits
__device__ __forceinline__ float unit(uint32_t v) { return (static_cast<float>(v >> 8) + 1.0f) * (1.0f / 16777216.0f); }

__device__ __forceinline__ float4 normals4(U4 r) {
    const float r0 = sqrtf(-2.0f * logf(unit(r.x))), r1 = sqrtf(-2.0f * logf(unit(r.z)));
    float s0, c0, s1, c1;
    sincospif(2.0f * unit(r.y), &s0, &c0);
    sincospif(2.0f * unit(r.w), &s1, &c1);
    return make_float4(r0 * c0, r0 * s0, r1 * c1, r1 * s1);
}

struct EnvParams {
    float* obs;
    float* rewards;
    int64_t* dones;
    float* time_outs;
    int64_t* ep;
    int64_t N;
    int32_t O4;  // obs row in 16-byte units
    uint32_t k0, k1;
    uint32_t step;
    float done_prob, timeout_prob;
    int64_t max_len;
};

__global__ __launch_bounds__(kBlock) void synthetic_env_kernel(EnvParams p) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    const int64_t units = p.N * p.O4;
    if (t < units) {  // one 16-byte unit of the observations
        const int64_t n = t / p.O4;
        const uint32_t j = static_cast<uint32_t>(t - n * p.O4);
        const U4 r = philox(U4{p.step, static_cast<uint32_t>(n), j + 1u, static_cast<uint32_t>(n >> 32)}, p.k0, p.k1);
        reinterpret_cast<float4*>(p.obs)[t] = normals4(r);
    }
    if (t < p.N) {  // the env's scalars (counter block 0)
        const U4 r = philox(U4{p.step, static_cast<uint32_t>(t), 0u, static_cast<uint32_t>(t >> 32)}, p.k0, p.k1);
        const float4 z = normals4(r);
        const float u = unit(philox(U4{p.step, static_cast<uint32_t>(t), 0x80000000u, 1u}, p.k0, p.k1).x) -
                        (1.0f / 16777216.0f);  // [0, 1)
        p.rewards[t] = z.x;
        const int64_t len = p.ep[t] + 1;
        const bool over = len >= p.max_len;
        const bool done = over || u < p.done_prob;
        const bool tout = over || (p.timeout_prob > 0.f && u < p.done_prob * p.timeout_prob);
        p.dones[t] = done ? 1 : 0;
        p.time_outs[t] = tout ? 1.f : 0.f;
        p.ep[t] = done ? 0 : len;
    }
}

}  // namespace
}  // namespace rslrl

using namespace rslrl;

extern "C" int rslrl_synthetic_env_step(float* obs, int32_t num_obs, float* rewards, int64_t* dones, float* time_outs,
                                        int64_t* episode_length, int64_t N, uint64_t seed, uint32_t step,
                                        float done_prob, float timeout_prob, int64_t max_episode_length,
                                        rslrl_stream_t stream) {
    if (N < 0 || num_obs < 0 || (num_obs & 3)) return RSLRL_E_INVALID_ARGUMENT;
    if (N == 0) return RSLRL_OK;
    if (!rewards || !dones || !time_outs || !episode_length || (num_obs > 0 && !obs)) return RSLRL_E_INVALID_ARGUMENT;
    if (reinterpret_cast<uintptr_t>(obs) & 15) return RSLRL_E_MISALIGNED;
    EnvParams p{};
    p.obs = obs;
    p.rewards = rewards;
    p.dones = dones;
    p.time_outs = time_outs;
    p.ep = episode_length;
    p.N = N;
    p.O4 = num_obs / 4;
    p.k0 = static_cast<uint32_t>(seed);
    p.k1 = static_cast<uint32_t>(seed >> 32);
    p.step = step;
    p.done_prob = done_prob;
    p.timeout_prob = timeout_prob;
    p.max_len = max_episode_length;
    const int64_t work = std::max<int64_t>(N * p.O4, N);
    hipLaunchKernelGGL(synthetic_env_kernel, dim3(static_cast<unsigned>(ceil_div(work, kBlock))), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), p);
    return launch_status();
}
