// GAE reverse scan + advantage normalisation on gfx950.
//
// Replaces rsl_rl/storage/rollout_storage.py:127-149 (RolloutStorage.compute_returns): the reference
// runs a Python loop over T steps of ~13 ATen kernels each on [N, 1] slabs (~320 launches), then a
// global mean/std.  Here:
//   gae_scan_kernel   one lane per environment walks t = T-1 .. 0 (the recurrence is serial in t and
//                     independent across envs).  All T (value, reward, done) loads of a lane are issued
//                     before the recurrence (TMAX-unrolled register arrays), so the wave has 3*T
//                     coalesced loads in flight; writes returns and raw advantages and emits one fp64
//                     (count, mean, M2) partial per block for the normalisation: each lane keeps its T
//                     advantages in registers and takes their mean and centred sum of squares exactly as a
//                     two-pass variance would, lanes and waves merge by Chan's pairwise formula in a fixed tree
//                     (round 5: this replaced round 3's separate centring pass -- one launch and a re-read of
//                     the advantages fewer, and still no sum(a^2) - n mean^2 cancellation).
//   adv_normalize     every block folds the <= kMaxPartials partials in one fixed order (so all blocks
//                     agree bitwise), then rescales the advantages with 16-byte accesses.
// Bytes per element (T*N of them): read 4 (V) + 4 (R) + 1 (done), write 4 (returns) + 4 (adv) = 17 in
// the scan; read 4 + write 4 = 8 in the normaliser.
//   gae_fused_slots   (round 5, rslrl_compute_returns_slots) both in one launch with a grid barrier between them:
//                     read V, R, done, log-prob (13 B), write returns, advantages, slot (24 B) per element.
//
// Bit-exactness: every fp32 operation of the reference expression is issued separately with
// round-to-nearest intrinsics in the reference's evaluation order (Python left-to-right:
// (nnt*gamma)*next_v, ((nnt*gamma)*lam)*adv), and advantages = returns - values exactly as :145.

#include <atomic>
#include <cstdlib>
#include <mutex>

#include "common.h"

namespace rslrl {
namespace {

constexpr int kMaxPartials = 512;

struct GaeStep {
    // One reverse step of rollout_storage.py:136-142; returns the new advantage.
    static __device__ __forceinline__ float step(float v, float r, unsigned d, float next_v, float adv,
                                                 float gamma, float lam) {
        const float nnt = __fsub_rn(1.0f, static_cast<float>(d));          // :136
        const float a = __fmul_rn(nnt, gamma);
        const float delta = __fsub_rn(__fadd_rn(r, __fmul_rn(a, next_v)), v);  // :138
        const float g = __fmul_rn(__fmul_rn(nnt, gamma), lam);
        return __fadd_rn(delta, __fmul_rn(g, adv));                      // :140
    }
};

// Chan et al.'s pairwise update of (count, mean, M2 = sum of squared deviations): exact in real arithmetic, and in
// fp64 free of the sum(a^2) - n mean^2 cancellation.  Either side may be empty.
struct Moments {
    double n, mean, m2;
};

__device__ __forceinline__ Moments chan(const Moments& a, const Moments& b) {
    const double n = a.n + b.n;
    if (n == 0.0) return a;
    const double delta = b.mean - a.mean;
    const double fb = b.n / n;
    return {n, a.mean + delta * fb, a.m2 + b.m2 + delta * delta * a.n * fb};
}

// block-wide merge in a fixed tree (wave: lane i takes lane i + off for off = 32 .. 1; then the waves in order);
// the result is valid in thread 0
__device__ __forceinline__ Moments block_chan(Moments m, double (*scratch)[3]) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const Moments o{__shfl_down(m.n, off, kWave), __shfl_down(m.mean, off, kWave), __shfl_down(m.m2, off, kWave)};
        if ((threadIdx.x & (kWave - 1)) < off) m = chan(m, o);
    }
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    __syncthreads();
    if (lane == 0) {
        scratch[wid][0] = m.n;
        scratch[wid][1] = m.mean;
        scratch[wid][2] = m.m2;
    }
    __syncthreads();
    Moments r{scratch[0][0], scratch[0][1], scratch[0][2]};
#pragma unroll
    for (int w = 1; w < kBlock / kWave; ++w) r = chan(r, Moments{scratch[w][0], scratch[w][1], scratch[w][2]});
    return r;
}

// EXACT: T == TMAX, the `t < T` guards fold away and all 3*T loads issue back to back.
template <int TMAX, bool EXACT>
__global__ __launch_bounds__(kBlock) void gae_scan_kernel(
    const float* __restrict__ values, const float* __restrict__ rewards, const uint8_t* __restrict__ dones,
    const float* __restrict__ last_values, float gamma, float lam, int T_, int64_t N,
    float* __restrict__ returns, float* __restrict__ advantages, double4* __restrict__ partials) {
    const int T = EXACT ? TMAX : T_;
    __shared__ double scratch[kBlock / kWave][3];
    Moments m{0.0, 0.0, 0.0};
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
    for (int64_t n = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; n < N; n += stride) {
        if constexpr (TMAX > 0) {
            float v[TMAX], r[TMAX], av[TMAX];
            unsigned d[TMAX];
#pragma unroll
            for (int t = 0; t < TMAX; ++t) {
                if (t < T) {
                    const int64_t i = static_cast<int64_t>(t) * N + n;
                    v[t] = values[i];
                    r[t] = rewards[i];
                    d[t] = dones[i];
                }
            }
            float next_v = last_values[n];
            float adv = 0.0f;
            double s = 0.0;
#pragma unroll
            for (int t = TMAX - 1; t >= 0; --t) {
                if (t < T) {
                    const int64_t i = static_cast<int64_t>(t) * N + n;
                    adv = GaeStep::step(v[t], r[t], d[t], next_v, adv, gamma, lam);
                    const float ret = __fadd_rn(adv, v[t]);  // :142
                    const float a = __fsub_rn(ret, v[t]);    // :145
                    returns[i] = ret;
                    advantages[i] = a;
                    av[t] = a;
                    s += static_cast<double>(a);
                    next_v = v[t];
                }
            }
            if (partials != nullptr) {  // this environment's T advantages: mean, then the centred sum of squares
                const double mean = s / static_cast<double>(T);
                double m2 = 0.0;
#pragma unroll
                for (int t = 0; t < TMAX; ++t) {
                    if (t < T) {
                        const double dlt = static_cast<double>(av[t]) - mean;
                        m2 += dlt * dlt;
                    }
                }
                m = chan(m, Moments{static_cast<double>(T), mean, m2});
            }
        } else {  // long rollouts: streaming loop (Welford's update per element)
            float next_v = last_values[n];
            float adv = 0.0f;
            for (int t = T - 1; t >= 0; --t) {
                const int64_t i = static_cast<int64_t>(t) * N + n;
                const float v = values[i];
                adv = GaeStep::step(v, rewards[i], dones[i], next_v, adv, gamma, lam);
                const float ret = __fadd_rn(adv, v);
                const float a = __fsub_rn(ret, v);
                returns[i] = ret;
                advantages[i] = a;
                m.n += 1.0;
                const double dlt = static_cast<double>(a) - m.mean;
                m.mean += dlt / m.n;
                m.m2 += dlt * (static_cast<double>(a) - m.mean);
                next_v = v;
            }
        }
    }
    if (partials != nullptr) {
        m = block_chan(m, scratch);
        if (threadIdx.x == 0) partials[blockIdx.x] = make_double4(m.n, m.mean, m.m2, 0.0);
    }
}

// (count, mean, M2) partials of an arbitrary vector (standalone normaliser): Welford per lane over its grid-stride
// elements, then the block tree.
__global__ __launch_bounds__(kBlock) void moments_kernel(const float* __restrict__ x, int64_t n,
                                                         double4* __restrict__ partials) {
    __shared__ double scratch[kBlock / kWave][3];
    Moments m{0.0, 0.0, 0.0};
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
        const double a = x[i];
        m.n += 1.0;
        const double dlt = a - m.mean;
        m.mean += dlt / m.n;
        m.m2 += dlt * (a - m.mean);
    }
    m = block_chan(m, scratch);
    if (threadIdx.x == 0) partials[blockIdx.x] = make_double4(m.n, m.mean, m.m2, 0.0);
}

// Mean and unbiased std (torch.Tensor.std default, correction = 1) from the (count, mean, M2) partials, merged in a
// fixed order (thread t takes partials t, t + 256; then the block tree): every block gets the same bits.
__device__ __forceinline__ void fold_moments(const double4* __restrict__ partials, int np, int64_t n,
                                             float* mean_out, float* std_out) {
    __shared__ double scratch[kBlock / kWave][3];
    Moments m{0.0, 0.0, 0.0};
    for (int i = threadIdx.x; i < np; i += kBlock) {
        const double4 p = partials[i];
        m = chan(m, Moments{p.x, p.y, p.z});
    }
    m = block_chan(m, scratch);
    const double var = n > 1 ? m.m2 / static_cast<double>(n - 1) : __builtin_nan("");  // torch: NaN std for one element
    *mean_out = static_cast<float>(m.mean);
    *std_out = static_cast<float>(sqrt(var));
}

__global__ __launch_bounds__(kBlock) void adv_normalize_kernel(float* __restrict__ adv, int64_t n,
                                                               const double4* __restrict__ partials, int np,
                                                               float eps) {
    float mean, std;
    fold_moments(partials, np, n, &mean, &std);
    const float denom = __fadd_rn(std, eps);  // rollout_storage.py:149  (std + 1e-8)
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
    const int64_t tid = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    const bool vec = (reinterpret_cast<uintptr_t>(adv) & 15) == 0;
    const int64_t nvec = vec ? n / 4 : 0;
    float4* adv4 = reinterpret_cast<float4*>(adv);
    for (int64_t i = tid; i < nvec; i += stride) {
        float4 a = adv4[i];
        a.x = __fdiv_rn(__fsub_rn(a.x, mean), denom);
        a.y = __fdiv_rn(__fsub_rn(a.y, mean), denom);
        a.z = __fdiv_rn(__fsub_rn(a.z, mean), denom);
        a.w = __fdiv_rn(__fsub_rn(a.w, mean), denom);
        adv4[i] = a;
    }
    for (int64_t i = nvec * 4 + tid; i < n; i += stride) adv[i] = __fdiv_rn(__fsub_rn(adv[i], mean), denom);
}

// adv_normalize_kernel that also writes each env-step's transition-record slot {value, log-prob, return, advantage,
// 0, 0, 0, 0} (RolloutStorage's per-update slot, rollout_storage.py field semantics unchanged): the pass that
// produces the final advantages is the one that places them, so no separate slot copy runs per update.  Two
// consecutive lanes write one 32-byte slot (unit 0 the four scalars, unit 1 zeros): each slot leaves the store whole.
__global__ __launch_bounds__(kBlock) void adv_normalize_slot_kernel(float* __restrict__ adv, int64_t n,
                                                                    const double4* __restrict__ partials, int np,
                                                                    float eps, const float* __restrict__ values,
                                                                    const float* __restrict__ logp,
                                                                    const float* __restrict__ returns,
                                                                    float* __restrict__ rec, int64_t R, int64_t off) {
    float mean, std;
    fold_moments(partials, np, n, &mean, &std);
    const float denom = __fadd_rn(std, eps);  // rollout_storage.py:149  (std + 1e-8)
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
    for (int64_t k = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; k < 2 * n; k += stride) {
        const int64_t i = k >> 1;
        float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((k & 1) == 0) {
            const float a = __fdiv_rn(__fsub_rn(adv[i], mean), denom);
            adv[i] = a;
            u = make_float4(values[i], logp[i], returns[i], a);
        }
        *reinterpret_cast<float4*>(rec + i * R + off + 4 * (k & 1)) = u;
    }
}

// adv_normalize_kernel that also writes the update's scalar slot array {value, log-prob, return, advantage} (one
// float4 per env-step, contiguous [T*N, 4]): every store is a coalesced 16-byte unit, where the in-record slots above
// are 32-byte pieces at the record stride (~1.6 TB/s: 49 us of the 72 us compute_returns at C3, profiles/r3_*).  The
// mini-batch gather takes each row's slot from this array beside the record (rslrl_gather_records_side).
__global__ __launch_bounds__(kBlock) void adv_normalize_slots_kernel(float* __restrict__ adv, int64_t n,
                                                                     const double4* __restrict__ partials, int np,
                                                                     float eps, const float* __restrict__ values,
                                                                     const float* __restrict__ logp,
                                                                     const float* __restrict__ returns,
                                                                     float4* __restrict__ slots) {
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
    const int64_t tid = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    // four env-steps per thread and iteration (16-byte loads of the four sources, 64 contiguous bytes of slots), so a
    // grid of a few blocks per CU covers the rollout and the partial fold runs once per block, not per 256 elements;
    // the first iteration's loads are issued before the fold (they do not depend on it: the fold's latency hides
    // under them).  The scalar loop takes the tail (and every element when a source is not 16-byte aligned).
    const bool vec = ((reinterpret_cast<uintptr_t>(adv) | reinterpret_cast<uintptr_t>(values) |
                       reinterpret_cast<uintptr_t>(logp) | reinterpret_cast<uintptr_t>(returns)) & 15) == 0;
    const int64_t nvec = vec ? n / 4 : 0;
    float4 a4 = {}, v4 = {}, l4 = {}, r4 = {};
    if (tid < nvec) {
        a4 = reinterpret_cast<const float4*>(adv)[tid];
        v4 = reinterpret_cast<const float4*>(values)[tid];
        l4 = reinterpret_cast<const float4*>(logp)[tid];
        r4 = reinterpret_cast<const float4*>(returns)[tid];
    }
    float mean, std;
    fold_moments(partials, np, n, &mean, &std);
    const float denom = __fadd_rn(std, eps);  // rollout_storage.py:149  (std + 1e-8)
    for (int64_t i = tid; i < nvec; i += stride) {
        if (i != tid) {
            a4 = reinterpret_cast<const float4*>(adv)[i];
            v4 = reinterpret_cast<const float4*>(values)[i];
            l4 = reinterpret_cast<const float4*>(logp)[i];
            r4 = reinterpret_cast<const float4*>(returns)[i];
        }
        float4 o;
        o.x = __fdiv_rn(__fsub_rn(a4.x, mean), denom);
        o.y = __fdiv_rn(__fsub_rn(a4.y, mean), denom);
        o.z = __fdiv_rn(__fsub_rn(a4.z, mean), denom);
        o.w = __fdiv_rn(__fsub_rn(a4.w, mean), denom);
        reinterpret_cast<float4*>(adv)[i] = o;
        float4* s = slots + 4 * i;
        s[0] = make_float4(v4.x, l4.x, r4.x, o.x);
        s[1] = make_float4(v4.y, l4.y, r4.y, o.y);
        s[2] = make_float4(v4.z, l4.z, r4.z, o.z);
        s[3] = make_float4(v4.w, l4.w, r4.w, o.w);
    }
    for (int64_t i = nvec * 4 + tid; i < n; i += stride) {
        const float a = __fdiv_rn(__fsub_rn(adv[i], mean), denom);
        adv[i] = a;
        slots[i] = make_float4(values[i], logp[i], returns[i], a);
    }
}

int scan_blocks(int64_t N) { return static_cast<int>(std::min<int64_t>(ceil_div(N, kBlock), kMaxPartials)); }

int elementwise_blocks(int64_t n) {
    return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 4 * kBlock), 2048)));
}

// ---- compute_returns_slots in ONE launch (round 5): scan, grid barrier, normalisation from registers ----------------
// One env per lane (nb = N / 256 blocks, every block resident at once -- checked against the occupancy on the host):
// the lane keeps its T values and returns in registers through the whole kernel, so the normalisation reads neither
// the advantages nor the values back, and the raw advantages are never written.  The block partials are the scan's
// (same partition, same Chan tree) and every block folds them in fold_moments' order after the barrier: mean / std,
// returns, advantages and slots are bit-identical to gae_scan_kernel + adv_normalize_slots_kernel.
//
// Grid barrier: the partials go out as agent-scope atomic stores; thread 0 of each block reads the generation word,
// takes a ticket, and the last arrival re-arms the ticket (0) and bumps the generation; the others spin on
// the generation with s_sleep (bounded: after ~2^22 polls a block gives up and raises the error word instead of
// hanging -- it cannot happen with every block resident).  Workspace: [kMaxPartials double4][ticket][generation]
// [error]; the ticket must be zero before the first call (zero-filled allocation) and is left zero.
constexpr int kBarOffset = sizeof(double4) * kMaxPartials;

__device__ __forceinline__ void gae_grid_barrier(unsigned* bar, unsigned nb) {
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned* ticket = bar;
        unsigned* gen = bar + 1;
        // no release / acquire fences (on gfx950 they write back / invalidate the whole L2 of the XCD -- the
        // scan's returns are in it): the partials went out as agent-scope atomic stores, which complete at the
        // coherence point before the ticket is taken (vmcnt), and are read back by agent-scope atomic loads
        const unsigned g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == nb - 1) {
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(gen, g0 + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            unsigned polls = 0;
            while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g0) {
                __builtin_amdgcn_s_sleep(2);
                if (++polls == (1u << 22)) {
                    __hip_atomic_store(bar + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
    }
    __syncthreads();
}

template <int T>
__global__ __launch_bounds__(kBlock) void gae_fused_slots_kernel(
    const float* __restrict__ values, const float* __restrict__ rewards, const uint8_t* __restrict__ dones,
    const float* __restrict__ last_values, float gamma, float lam, int64_t N, float eps, float* __restrict__ returns,
    float* __restrict__ advantages, const float* __restrict__ logp, float4* __restrict__ slots,
    double4* __restrict__ partials, unsigned* __restrict__ bar) {
    __shared__ double scratch[kBlock / kWave][3];
    const int64_t n = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    const bool ok = n < N;
    float v[T], ret[T];
    Moments m{0.0, 0.0, 0.0};
    if (ok) {
        float r[T];
        unsigned d[T];
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int64_t i = static_cast<int64_t>(t) * N + n;
            v[t] = values[i];
            r[t] = rewards[i];
            d[t] = dones[i];
        }
        float next_v = last_values[n];
        float adv = 0.0f;
        double s = 0.0;
#pragma unroll
        for (int t = T - 1; t >= 0; --t) {
            adv = GaeStep::step(v[t], r[t], d[t], next_v, adv, gamma, lam);
            ret[t] = __fadd_rn(adv, v[t]);  // :142
            returns[static_cast<int64_t>(t) * N + n] = ret[t];
            s += static_cast<double>(__fsub_rn(ret[t], v[t]));  // :145
            next_v = v[t];
        }
        const double mean = s / static_cast<double>(T);
        double m2 = 0.0;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const double dlt = static_cast<double>(__fsub_rn(ret[t], v[t])) - mean;
            m2 += dlt * dlt;
        }
        m = chan(m, Moments{static_cast<double>(T), mean, m2});
    }
    m = block_chan(m, scratch);
    if (threadIdx.x == 0) {
        unsigned long long* p = reinterpret_cast<unsigned long long*>(partials + blockIdx.x);
        __hip_atomic_store(p, __double_as_longlong(m.n), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p + 1, __double_as_longlong(m.mean), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p + 2, __double_as_longlong(m.m2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    float lp[T];  // the log-probs load while the grid gathers
    if (ok) {
#pragma unroll
        for (int t = 0; t < T; ++t) lp[t] = logp[static_cast<int64_t>(t) * N + n];
    }
    gae_grid_barrier(bar, gridDim.x);
    // fold_moments' order over the partials (atomic loads: another XCD's L2 wrote them)
    Moments f{0.0, 0.0, 0.0};
    for (int i = threadIdx.x; i < static_cast<int>(gridDim.x); i += kBlock) {
        const unsigned long long* p = reinterpret_cast<const unsigned long long*>(partials + i);
        const Moments q{__longlong_as_double(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                        __longlong_as_double(__hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                        __longlong_as_double(__hip_atomic_load(p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))};
        f = chan(f, q);
    }
    f = block_chan(f, scratch);
    const int64_t total = static_cast<int64_t>(T) * N;
    const double var = total > 1 ? f.m2 / static_cast<double>(total - 1) : __builtin_nan("");
    const float mean = static_cast<float>(f.mean);
    const float denom = __fadd_rn(static_cast<float>(sqrt(var)), eps);  // rollout_storage.py:149
    if (ok) {
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int64_t i = static_cast<int64_t>(t) * N + n;
            const float a = __fdiv_rn(__fsub_rn(__fsub_rn(ret[t], v[t]), mean), denom);
            advantages[i] = a;
            slots[i] = make_float4(v[t], lp[t], ret[t], a);
        }
    }
}

// blocks of gae_fused_slots_kernel<T> the device holds at once (0: no fused instance for T)
int gae_fused_capacity(int T) {
    // per device (the current one) and T, computed once; concurrent first calls compute the same value
    constexpr int kMaxDev = 64;
    static std::atomic<int> cap[kMaxDev][4];
    static std::once_flag init;
    std::call_once(init, [] {
        for (auto& d : cap)
            for (auto& c : d) c.store(-1, std::memory_order_relaxed);
    });
    const int k = T == 8 ? 0 : T == 16 ? 1 : T == 24 ? 2 : T == 32 ? 3 : -1;
    int dev = 0;
    if (k < 0 || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 0;
    int c = cap[dev][k].load(std::memory_order_relaxed);
    if (c < 0) {
        int cus = 0, per = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 0;
        const void* f = k == 0 ? reinterpret_cast<const void*>(&gae_fused_slots_kernel<8>)
                        : k == 1 ? reinterpret_cast<const void*>(&gae_fused_slots_kernel<16>)
                        : k == 2 ? reinterpret_cast<const void*>(&gae_fused_slots_kernel<24>)
                                 : reinterpret_cast<const void*>(&gae_fused_slots_kernel<32>);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, kBlock, 0) != hipSuccess) per = 0;
        c = per * cus;
        cap[dev][k].store(c, std::memory_order_relaxed);
    }
    return c;
}

template <int TMAX>
void launch_scan(int nb, hipStream_t st, const float* v, const float* r, const uint8_t* d, const float* lv,
                 float g, float l, int T, int64_t N, float* ret, float* adv, double4* part) {
    if (T == TMAX)
        hipLaunchKernelGGL((gae_scan_kernel<TMAX, true>), dim3(nb), dim3(kBlock), 0, st, v, r, d, lv, g, l, T, N, ret,
                           adv, part);
    else
        hipLaunchKernelGGL((gae_scan_kernel<TMAX, false>), dim3(nb), dim3(kBlock), 0, st, v, r, d, lv, g, l, T, N, ret,
                           adv, part);
}

}  // namespace
}  // namespace rslrl

using namespace rslrl;

extern "C" size_t rslrl_compute_returns_workspace_bytes(int64_t T, int64_t N) {
    (void)T;
    (void)N;
    return kBarOffset + 64;  // the partials, then the one-launch form's barrier words
}

extern "C" size_t rslrl_normalize_workspace_bytes(int64_t n) {
    (void)n;
    return sizeof(double4) * kMaxPartials;
}

namespace {
// RecordSlot: optional destination of the normalisation pass (rslrl_compute_returns_records)
struct RecordSlot {
    const float* log_prob;
    float* records;         // records (record_floats > 0) or the contiguous float4 slot array (record_floats == 0)
    int64_t record_floats;
    int64_t offset;
};

int compute_returns_impl(const float* values, const float* rewards, const uint8_t* dones, const float* last_values,
                         float gamma, float lam, int64_t T, int64_t N, int32_t normalize_advantage, float* returns,
                         float* advantages, void* workspace, size_t workspace_bytes, rslrl_stream_t stream,
                         const RecordSlot* slot) {
    if (T < 0 || N < 0 || T > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
    if (T == 0 || N == 0) return RSLRL_OK;
    if (!values || !rewards || !dones || !last_values || !returns || !advantages) return RSLRL_E_INVALID_ARGUMENT;
    double4* part = nullptr;
    if (normalize_advantage) {
        if (!workspace) return RSLRL_E_INVALID_ARGUMENT;
        if (workspace_bytes < rslrl_compute_returns_workspace_bytes(T, N)) return RSLRL_E_WORKSPACE_TOO_SMALL;
        if (reinterpret_cast<uintptr_t>(workspace) & 15) return RSLRL_E_MISALIGNED;
        part = static_cast<double4*>(workspace);
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int nb = scan_blocks(N);
    const int t = static_cast<int>(T);
    static const bool fused_on = [] {
        const char* e = std::getenv("RSLRL_GAE_FUSED");
        return !(e && e[0] == '0');
    }();
    if (slot && slot->record_floats == 0 && fused_on && nb == ceil_div(N, kBlock) && nb <= gae_fused_capacity(t)) {
        // one launch: scan + grid barrier + normalisation + slots (bit-identical to the two-launch path below)
        unsigned* bar = reinterpret_cast<unsigned*>(static_cast<char*>(workspace) + kBarOffset);
        float4* sl = reinterpret_cast<float4*>(slot->records);
#define RSLRL_GAE_FUSED_LAUNCH(TT)                                                                                    \
    hipLaunchKernelGGL((gae_fused_slots_kernel<TT>), dim3(nb), dim3(kBlock), 0, st, values, rewards, dones,           \
                       last_values, gamma, lam, N, 1e-8f, returns, advantages, slot->log_prob, sl, part, bar)
        if (t == 8) RSLRL_GAE_FUSED_LAUNCH(8);
        else if (t == 16) RSLRL_GAE_FUSED_LAUNCH(16);
        else if (t == 24) RSLRL_GAE_FUSED_LAUNCH(24);
        else RSLRL_GAE_FUSED_LAUNCH(32);
#undef RSLRL_GAE_FUSED_LAUNCH
        return launch_status();
    }
    if (t <= 8)
        launch_scan<8>(nb, st, values, rewards, dones, last_values, gamma, lam, t, N, returns, advantages, part);
    else if (t <= 16)
        launch_scan<16>(nb, st, values, rewards, dones, last_values, gamma, lam, t, N, returns, advantages, part);
    else if (t <= 24)
        launch_scan<24>(nb, st, values, rewards, dones, last_values, gamma, lam, t, N, returns, advantages, part);
    else if (t <= 32)
        launch_scan<32>(nb, st, values, rewards, dones, last_values, gamma, lam, t, N, returns, advantages, part);
    else
        launch_scan<0>(nb, st, values, rewards, dones, last_values, gamma, lam, t, N, returns, advantages, part);
    int rc = launch_status();
    if (rc != RSLRL_OK || !normalize_advantage) return rc;
    const int64_t n = T * N;
    if (slot && slot->record_floats == 0) {
        const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 4 * kBlock), 1024));
        hipLaunchKernelGGL(adv_normalize_slots_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0, st,
                           advantages, n, part, nb, 1e-8f, values, slot->log_prob, returns,
                           reinterpret_cast<float4*>(slot->records));
    } else if (slot) {
        const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(ceil_div(2 * n, kBlock), 4096));
        hipLaunchKernelGGL(adv_normalize_slot_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0, st,
                           advantages, n, part, nb, 1e-8f, values, slot->log_prob, returns, slot->records,
                           slot->record_floats, slot->offset);
    } else {
        hipLaunchKernelGGL(adv_normalize_kernel, dim3(elementwise_blocks(n)), dim3(kBlock), 0, st, advantages, n, part,
                           nb, 1e-8f);
    }
    return launch_status();
}
}  // namespace

extern "C" int rslrl_compute_returns(const float* values, const float* rewards, const uint8_t* dones,
                                     const float* last_values, float gamma, float lam, int64_t T, int64_t N,
                                     int32_t normalize_advantage, float* returns, float* advantages,
                                     void* workspace, size_t workspace_bytes, rslrl_stream_t stream) {
    return compute_returns_impl(values, rewards, dones, last_values, gamma, lam, T, N, normalize_advantage, returns,
                                advantages, workspace, workspace_bytes, stream, nullptr);
}

extern "C" int rslrl_compute_returns_records(const float* values, const float* rewards, const uint8_t* dones,
                                             const float* last_values, float gamma, float lam, int64_t T, int64_t N,
                                             float* returns, float* advantages, const float* log_prob, float* records,
                                             int64_t record_floats, int64_t slot_offset, void* workspace,
                                             size_t workspace_bytes, rslrl_stream_t stream) {
    if (!log_prob || !records || record_floats <= 0 || (record_floats & 3) || slot_offset < 0 || (slot_offset & 3) ||
        slot_offset + 8 > record_floats)
        return RSLRL_E_INVALID_ARGUMENT;
    if (reinterpret_cast<uintptr_t>(records) & 15) return RSLRL_E_MISALIGNED;
    const RecordSlot slot{log_prob, records, record_floats, slot_offset};
    return compute_returns_impl(values, rewards, dones, last_values, gamma, lam, T, N, 1, returns, advantages,
                                workspace, workspace_bytes, stream, &slot);
}

extern "C" int rslrl_compute_returns_slots(const float* values, const float* rewards, const uint8_t* dones,
                                           const float* last_values, float gamma, float lam, int64_t T, int64_t N,
                                           float* returns, float* advantages, const float* log_prob, float* slots,
                                           void* workspace, size_t workspace_bytes, rslrl_stream_t stream) {
    if (!log_prob || !slots) return RSLRL_E_INVALID_ARGUMENT;
    if (reinterpret_cast<uintptr_t>(slots) & 15) return RSLRL_E_MISALIGNED;
    const RecordSlot slot{log_prob, slots, 0, 0};
    return compute_returns_impl(values, rewards, dones, last_values, gamma, lam, T, N, 1, returns, advantages,
                                workspace, workspace_bytes, stream, &slot);
}

extern "C" int rslrl_normalize_advantages(float* advantages, int64_t n, float eps, void* workspace,
                                          size_t workspace_bytes, rslrl_stream_t stream) {
    if (n < 0) return RSLRL_E_INVALID_ARGUMENT;
    if (n == 0) return RSLRL_OK;
    if (!advantages || !workspace) return RSLRL_E_INVALID_ARGUMENT;
    if (workspace_bytes < rslrl_normalize_workspace_bytes(n)) return RSLRL_E_WORKSPACE_TOO_SMALL;
    if (reinterpret_cast<uintptr_t>(workspace) & 15) return RSLRL_E_MISALIGNED;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    double4* part = static_cast<double4*>(workspace);
    const int nb = static_cast<int>(std::min<int64_t>(ceil_div(n, kBlock), kMaxPartials));
    hipLaunchKernelGGL(moments_kernel, dim3(nb), dim3(kBlock), 0, st, advantages, n, part);
    int rc = launch_status();
    if (rc != RSLRL_OK) return rc;
    hipLaunchKernelGGL(adv_normalize_kernel, dim3(elementwise_blocks(n)), dim3(kBlock), 0, st, advantages, n, part,
                       nb, eps);
    return launch_status();
}
