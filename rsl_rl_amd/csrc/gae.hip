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
#include <string>

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

#ifdef RSLRL_GAE_STAMPS
// diagnostic build only (never the shipped library; scripts/gae_stamps.py): per block, s_memrealtime (100 MHz, one clock
// for the whole chip) at 6 points of the one-launch kernel -> g_gae_stamps[block * 8 + k]; [7] = 1 for the last arrival
__device__ uint64_t* g_gae_stamps;
#define GAE_STAMP(k)                                                                                              \
    do {                                                                                                          \
        if (g_gae_stamps && threadIdx.x == 0) {                                                                   \
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                                      \
            g_gae_stamps[static_cast<int64_t>(blockIdx.x) * 8 + (k)] = __builtin_amdgcn_s_memrealtime();            \
        }                                                                                                         \
    } while (0)
#else
#define GAE_STAMP(k) \
    do {             \
    } while (0)
#endif

// ---- compute_returns_slots in ONE launch: scan, grid barrier, normalisation --------------------------------------
// Two kernels take this form; both keep the values and returns of their envs on chip through the whole launch, so the
// normalisation reads neither the advantages nor the values back and the raw advantages are never written:
//   gae_staged_slots_kernel (round 6, default; N % 64 == 0): a 256-thread block owns 64 envs.  All four waves stage
//       the block's [T][64] values, rewards and dones tiles into LDS with 16-byte loads (every thread has ~5 loads in
//       flight, and N / 64 blocks fill the chip where one lane per env left the 16,384-env share on 64 CUs), wave 0
//       runs the serial reverse recurrence out of LDS (one lane per env, the reference's fp32 operation order), and
//       after the barrier all four waves write advantages and slots from the tiles as 16-byte units.
//   gae_fused_slots_kernel (round 5; any N): one env per lane, 256 envs per block, the tiles in registers.
// The block partials reproduce the two-launch scan's partition exactly: a staged block's partial is the Chan tree of
// ONE wave of a scan block, and the fold chains each group of four in the scan's wave order before fold_moments'
// order over the groups -- mean / std, returns, advantages and slots are bit-identical to gae_scan_kernel +
// adv_normalize_slots_kernel.
//
// Grid barrier + statistics (grid_stats): thread 0 of each block stores its partial as agent-scope atomic stores, reads
// the generation word and takes a ticket; the LAST arrival folds every partial (one block: no all-to-all partial
// reads), publishes (mean, std + eps), re-arms the ticket (0) and bumps the generation; the others spin on the
// generation with s_sleep.  No release / acquire fences: on gfx950 they write back / invalidate the XCD's whole L2 (the
// returns just written are in it); agent-scope atomics complete at the coherence point (vmcnt) and are read back by
// agent-scope atomic loads.
// Co-residency: the grid is sized to what the device holds at once (occupancy x CUs, checked on the host).  That is
// not a guarantee when another kernel or process holds CUs, so a waiting block gives up after `spin_limit` polls
// (seconds): it raises the workspace's status word and normalises with NaN statistics -- a barrier that could not
// complete shows as NaN advantages AND a status word that PPO.update reads with its loss statistics and raises on,
// never as silently wrong numbers.  A late block still arrives, folds and re-arms, so the words are consistent for the
// next call.  RSLRL_GAE_COOP=1 launches cooperatively instead (hipLaunchCooperativeKernel: the runtime refuses a grid
// it cannot hold, and the call falls back to the two-launch path) -- opt-in, since it costs more than the barrier.
// Workspace: [kMaxWaveParts double4 partials][ticket][-][status] then, per group of 64 blocks, a 256-byte piece holding
// the group's record {generation, mean, std + eps, check} and (128 bytes on) its arrival ticket; zero-filled before its
// first use, tickets left zero by every call.  One workspace per
// stream (two concurrent calls must not share a ticket).
constexpr int kStagedEnvs = 64;                 // envs per block of the staged kernel (one wave of the scan's blocks)
constexpr int kMaxWaveParts = 4 * kMaxPartials; // partials of the staged kernel: N / 64 <= 2048
constexpr int kBarOffset = sizeof(double4) * kMaxWaveParts;
constexpr int kStatusWord = 2;                  // index of the status word among the barrier words
constexpr unsigned kDefaultSpinLimit = 1u << 22;

__device__ __forceinline__ void store_partial(double4* partials, int i, const Moments& m) {
    unsigned long long* p = reinterpret_cast<unsigned long long*>(partials + i);
    __hip_atomic_store(p, __double_as_longlong(m.n), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p + 1, __double_as_longlong(m.mean), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p + 2, __double_as_longlong(m.m2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ Moments load_partial(const double4* partials, int i) {
    const unsigned long long* p = reinterpret_cast<const unsigned long long*>(partials + i);
    return {__longlong_as_double(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
            __longlong_as_double(__hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
            __longlong_as_double(__hip_atomic_load(p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))};
}

// The barrier's generation words: one per group of kGenGroup blocks, each in its own 256-byte piece (a different
// memory channel), so ~64 pollers share a word instead of every block of the grid hammering one address -- with 1,024
// pollers on one word the arrival of the last block and its fold waited behind their loads.
constexpr int kGenGroup = 64;
constexpr int kGenStride = 64;  // words (256 bytes)
constexpr int kGenOffset = 64;  // words after the barrier base
constexpr int kMaxGenGroups = kMaxWaveParts / kGenGroup;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned gen_check(unsigned g, unsigned m, unsigned d) {
    return (g * 0x9e3779b1u) ^ (m + 0x7f4a7c15u) ^ ((d << 7) | (d >> 25)) ^ 0x5bd1e995u;
}

// Every block calls this after thread 0 stored its partial (partials[blockIdx.x]).  G partials make one scan-block
// partial (chained in index order, as block_chan chains a scan block's waves); those are folded in fold_moments'
// order.  Returns (mean, std + eps) in every thread; (NaN, NaN) after a barrier time-out.
template <int G, int NT>
__device__ float2 grid_stats(const double4* partials, int64_t total, float eps, unsigned* bar, unsigned spin_limit,
                             unsigned sleep_units, double (*scratch)[3]) {
    static_assert(NT == kBlock || NT == kWave, "256- or 64-thread blocks");
    // the fold runs in fold_moments' 256-thread order whatever the block size: real thread r plays the virtual threads
    // r + NT k (k < V), i.e. lane r of virtual wave k
    constexpr int V = kBlock / NT;
    constexpr int R = NT == kBlock ? kMaxPartials / kBlock : 1;  // rounds of 256 groups (the narrow form: N <= 65536)
    __shared__ float2 s_res;
    __shared__ int s_last;
    __shared__ unsigned s_gen;
    unsigned* ticket = bar;
    const unsigned nb = gridDim.x;
    unsigned* gen = bar + kGenOffset + kGenStride * (blockIdx.x / kGenGroup);
    __syncthreads();
    if (threadIdx.x == 0) {
        // two-level arrival: a ticket per group of kGenGroup blocks (its own line), the group's last arrival takes a
        // ticket of the grid -- at most 64 atomics queue on one address (1,024 on one word cost ~17 us at C3's
        // staged grid, profiles/r6_gae_probe.json)
        const unsigned grp = blockIdx.x / kGenGroup;
        const unsigned gsize = min(static_cast<unsigned>(kGenGroup), nb - grp * kGenGroup);
        unsigned* gticket = bar + kGenOffset + kGenStride * grp + kGenStride / 2;
        const unsigned g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's partial (and the generation read) complete
        int last = 0;
        if (__hip_atomic_fetch_add(gticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
            __hip_atomic_store(gticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the group has arrived
            const unsigned ngroups = (nb + kGenGroup - 1) / kGenGroup;
            // one group (<= 64 blocks): its last arrival is the grid's, no second hop
            last = ngroups == 1 ||
                   __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1;
        }
        s_last = last;
        s_gen = g0;
    }
    __syncthreads();
    const unsigned g0 = s_gen;
#ifdef RSLRL_GAE_STAMPS
    if (g_gae_stamps && threadIdx.x == 0) g_gae_stamps[static_cast<int64_t>(blockIdx.x) * 8 + 7] = s_last;
#endif
    if (s_last) {
        // every partial this thread folds is loaded before the first chan (one memory round trip; sc1: read at the
        // coherence point, where the other XCDs' atomic stores went)
        constexpr int kPer = V * R * G;  // partials per thread
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<double4*>(partials), 0, static_cast<int>(sizeof(double4) * nb), 0x00020000);
        double3 q[kPer];
#pragma unroll
        for (int i = 0; i < kPer; ++i) {  // i = ((k R) + j) G + member
            const int k = i / (R * G), j = (i / G) % R;
            const int idx = (threadIdx.x + NT * k + kBlock * j) * G + (i % G);
            const int off = idx < static_cast<int>(nb) ? idx * 32 : 0x7ffffff0;  // out of range reads 0
            const auto lo = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 16 /* sc1 */);
            const auto hi = __builtin_amdgcn_raw_buffer_load_b64(rsrc, off + 16, 0, 16 /* sc1 */);
            q[i] = make_double3(__builtin_bit_cast(double, make_uint2(lo[0], lo[1])),
                                __builtin_bit_cast(double, make_uint2(lo[2], lo[3])), __builtin_bit_cast(double, hi));
        }
        const int ngroups = static_cast<int>((nb + G - 1) / G);
        Moments mv[V];
#pragma unroll
        for (int k = 0; k < V; ++k) {
            mv[k] = Moments{0.0, 0.0, 0.0};
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const int gi = threadIdx.x + NT * k + kBlock * j;
                const double3* qq = q + (k * R + j) * G;
                if (gi < ngroups) {
                    Moments p{qq[0].x, qq[0].y, qq[0].z};
#pragma unroll
                    for (int u = 1; u < G; ++u)
                        if (gi * G + u < static_cast<int>(nb)) p = chan(p, Moments{qq[u].x, qq[u].y, qq[u].z});
                    mv[k] = chan(mv[k], p);
                }
            }
        }
        Moments m;
        if constexpr (V == 1) {
            m = block_chan(mv[0], scratch);
        } else {  // one real wave: each virtual wave's tree (block_chan's), then the virtual waves in order (lane 0)
#pragma unroll
            for (int k = 0; k < V; ++k) {
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    const Moments o{__shfl_down(mv[k].n, off, kWave), __shfl_down(mv[k].mean, off, kWave),
                                    __shfl_down(mv[k].m2, off, kWave)};
                    if (static_cast<int>(threadIdx.x) < off) mv[k] = chan(mv[k], o);
                }
            }
            m = mv[0];
#pragma unroll
            for (int k = 1; k < V; ++k) m = chan(m, mv[k]);
        }
        if (threadIdx.x == 0) {
            const double var = total > 1 ? m.m2 / static_cast<double>(total - 1) : __builtin_nan("");
            s_res = make_float2(static_cast<float>(m.mean),
                                __fadd_rn(static_cast<float>(sqrt(var)), eps));  // rollout_storage.py:149
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed (lands by kernel end)
        }
        __syncthreads();
        // publish {generation, mean, std + eps, check} as ONE 16-byte write-through store per group word: the waiters
        // read the statistics with the generation (one poll load, no second round trip).  EVERY group's record moves
        // (not only this grid's), so the generations stay equal whatever grid sizes share the workspace: a waiter
        // compares against its own group's word, and lagging words could equal a waiter's snapshot.
        if (threadIdx.x < kMaxGenGroups) {
            const unsigned g1 = g0 + 1u;
            const unsigned um = __float_as_uint(s_res.x), ud = __float_as_uint(s_res.y);
            const u32x4 rec = {g1, um, ud, gen_check(g1, um, ud)};
            unsigned* dst = bar + kGenOffset + kGenStride * threadIdx.x;
            asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst), "v"(rec) : "memory");
        }
    } else if (threadIdx.x == 0) {
        unsigned polls = 0;
        bool ok = true;
        u32x4 rec;
        for (;;) {
            // one 16-byte write-through load of the group's record; taken only with a new generation and a matching
            // check word (a torn read of the two halves fails the check and polls again)
            asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(rec) : "v"(gen) : "memory");
            if (rec.x != g0 && rec.w == gen_check(rec.x, rec.y, rec.z)) break;
            if (polls++ >= spin_limit) {
                ok = false;
                break;
            }
            for (unsigned z = 0; z < sleep_units; ++z) __builtin_amdgcn_s_sleep(2);
        }
        if (ok) {
            s_res = make_float2(__uint_as_float(rec.y), __uint_as_float(rec.z));
        } else {
            __hip_atomic_store(bar + kStatusWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_res = make_float2(__builtin_nanf(""), __builtin_nanf(""));
        }
    }
    __syncthreads();
    return s_res;
}

template <int T, int NT>
__global__ __launch_bounds__(NT) void gae_fused_slots_kernel(
    const float* __restrict__ values, const float* __restrict__ rewards, const uint8_t* __restrict__ dones,
    const float* __restrict__ last_values, float gamma, float lam, int64_t N, float eps, float* __restrict__ returns,
    float* __restrict__ advantages, const float* __restrict__ logp, float4* __restrict__ slots,
    double4* __restrict__ partials, unsigned* __restrict__ bar, unsigned spin_limit,
    unsigned sleep_units) {
    __shared__ double scratch[NT / kWave][3];
    const int64_t n = static_cast<int64_t>(blockIdx.x) * NT + threadIdx.x;
    const bool ok = n < N;
    float v[T], ret[T];
    Moments m{0.0, 0.0, 0.0};
    GAE_STAMP(0);
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
    if constexpr (NT == kBlock) {
        m = block_chan(m, scratch);
    } else {  // one wave per block: its partial is the wave tree of a 256-thread block's wave
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const Moments o{__shfl_down(m.n, off, kWave), __shfl_down(m.mean, off, kWave), __shfl_down(m.m2, off, kWave)};
            if (static_cast<int>(threadIdx.x) < off) m = chan(m, o);
        }
    }
    GAE_STAMP(1);
    if (threadIdx.x == 0) store_partial(partials, blockIdx.x, m);
    GAE_STAMP(2);
    float lp[T];  // the log-probs load while the grid gathers
    if (ok) {
#pragma unroll
        for (int t = 0; t < T; ++t) lp[t] = logp[static_cast<int64_t>(t) * N + n];
    }
    GAE_STAMP(3);
    const float2 st = grid_stats<kBlock / NT, NT>(partials, static_cast<int64_t>(T) * N, eps, bar, spin_limit, sleep_units, scratch);
    GAE_STAMP(4);
    if (ok) {
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int64_t i = static_cast<int64_t>(t) * N + n;
            const float a = __fdiv_rn(__fsub_rn(__fsub_rn(ret[t], v[t]), st.x), st.y);
            advantages[i] = a;
            slots[i] = make_float4(v[t], lp[t], ret[t], a);
        }
    }
    GAE_STAMP(5);
}

template <int T>
__global__ __launch_bounds__(kBlock) void gae_staged_slots_kernel(
    const float* __restrict__ values, const float* __restrict__ rewards, const uint8_t* __restrict__ dones,
    const float* __restrict__ last_values, float gamma, float lam, int64_t N, float eps, float* __restrict__ returns,
    float* __restrict__ advantages, const float* __restrict__ logp, float4* __restrict__ slots,
    double4* __restrict__ partials, unsigned* __restrict__ bar, unsigned spin_limit,
    unsigned sleep_units) {
    constexpr int E = kStagedEnvs;
    constexpr int U = T * E / 4;                    // 16-byte units of a [T][64] fp32 tile (16 per row)
    constexpr int UD = T * E / 16;                  // 16-byte units of the [T][64] uint8 dones tile (4 per row)
    constexpr int J = (U + kBlock - 1) / kBlock;    // fp32 units per thread
    constexpr int JD = (UD + kBlock - 1) / kBlock;  // dones units per thread
    __shared__ float4 s_v[U];
    __shared__ float4 s_r[U];  // rewards, overwritten by the returns as the scan consumes them
    __shared__ uint4 s_d[UD];
    __shared__ double scratch[kBlock / kWave][3];
    const int tid = threadIdx.x;
    const int64_t n0 = static_cast<int64_t>(blockIdx.x) * E;
    // ---- stage: every load of the block in flight at once (rows of 64 envs = 256 contiguous bytes) ----
    float4 v4[J], r4[J], l4[J];
    uint4 d4[JD];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int u = tid + j * kBlock;
        if (U % kBlock == 0 || u < U) {
            const int64_t g = static_cast<int64_t>(u >> 4) * N + n0 + 4 * (u & 15);
            v4[j] = *reinterpret_cast<const float4*>(values + g);
            r4[j] = *reinterpret_cast<const float4*>(rewards + g);
            l4[j] = *reinterpret_cast<const float4*>(logp + g);  // for this thread's slots after the barrier
        }
    }
#pragma unroll
    for (int j = 0; j < JD; ++j) {
        const int u = tid + j * kBlock;
        if (UD % kBlock == 0 || u < UD)
            d4[j] = *reinterpret_cast<const uint4*>(dones + static_cast<int64_t>(u >> 2) * N + n0 + 16 * (u & 3));
    }
    const float lv = tid < E ? last_values[n0 + tid] : 0.0f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int u = tid + j * kBlock;
        if (U % kBlock == 0 || u < U) {
            s_v[u] = v4[j];
            s_r[u] = r4[j];
        }
    }
#pragma unroll
    for (int j = 0; j < JD; ++j) {
        const int u = tid + j * kBlock;
        if (UD % kBlock == 0 || u < UD) s_d[u] = d4[j];
    }
    __syncthreads();
    // ---- wave 0: the reverse recurrence of rollout_storage.py:128-145, one lane per env ----
    if (tid < E) {
        const float* sv = reinterpret_cast<const float*>(s_v);
        float* sr = reinterpret_cast<float*>(s_r);
        const uint8_t* sd = reinterpret_cast<const uint8_t*>(s_d);
        float next_v = lv;
        float adv = 0.0f;
        double s = 0.0;
#pragma unroll
        for (int t = T - 1; t >= 0; --t) {
            const float v = sv[t * E + tid];
            adv = GaeStep::step(v, sr[t * E + tid], sd[t * E + tid], next_v, adv, gamma, lam);
            const float ret = __fadd_rn(adv, v);  // :142
            sr[t * E + tid] = ret;
            returns[static_cast<int64_t>(t) * N + n0 + tid] = ret;
            s += static_cast<double>(__fsub_rn(ret, v));  // :145
            next_v = v;
        }
        const double mean = s / static_cast<double>(T);
        double m2 = 0.0;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const double dlt = static_cast<double>(__fsub_rn(sr[t * E + tid], sv[t * E + tid])) - mean;
            m2 += dlt * dlt;
        }
        Moments m = chan(Moments{0.0, 0.0, 0.0}, Moments{static_cast<double>(T), mean, m2});
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {  // block_chan's wave tree
            const Moments o{__shfl_down(m.n, off, kWave), __shfl_down(m.mean, off, kWave),
                            __shfl_down(m.m2, off, kWave)};
            if (tid < off) m = chan(m, o);
        }
        if (tid == 0) store_partial(partials, blockIdx.x, m);
    }
    // ---- statistics over the grid (4 staged blocks = one scan block) ----
    const float2 st = grid_stats<4, kBlock>(partials, static_cast<int64_t>(T) * N, eps, bar, spin_limit, sleep_units, scratch);
    // ---- normalise and write: per thread its units of the tiles (the barrier's __syncthreads published s_r) ----
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int u = tid + j * kBlock;
        if (U % kBlock == 0 || u < U) {
            const int64_t g = static_cast<int64_t>(u >> 4) * N + n0 + 4 * (u & 15);
            const float4 v = s_v[u];
            const float4 rt = s_r[u];
            float4 a;
            a.x = __fdiv_rn(__fsub_rn(__fsub_rn(rt.x, v.x), st.x), st.y);
            a.y = __fdiv_rn(__fsub_rn(__fsub_rn(rt.y, v.y), st.x), st.y);
            a.z = __fdiv_rn(__fsub_rn(__fsub_rn(rt.z, v.z), st.x), st.y);
            a.w = __fdiv_rn(__fsub_rn(__fsub_rn(rt.w, v.w), st.x), st.y);
            *reinterpret_cast<float4*>(advantages + g) = a;
            float4* sl = slots + g;
            sl[0] = make_float4(v.x, l4[j].x, rt.x, a.x);
            sl[1] = make_float4(v.y, l4[j].y, rt.y, a.y);
            sl[2] = make_float4(v.z, l4[j].z, rt.z, a.z);
            sl[3] = make_float4(v.w, l4[j].w, rt.w, a.w);
        }
    }
}

// ---- host side: which form a call takes, device capacities, the debug knobs ----
enum GaeForm { kFormTwoLaunch = 0, kFormOneLaunch = 1, kFormStaged = 2, kFormNarrow = 3 };
constexpr int kNarrowMaxN = 65536;  // the narrow form's fold holds one round of 256 groups

std::atomic<int64_t> g_knob_form{-1};       // -1 auto; 0 / 1 / 2 / 3 force that form where it applies (else 0)
std::atomic<int64_t> g_knob_coop{-1};       // -1 RSLRL_GAE_COOP (default 0), 0 plain launch, 1 cooperative
std::atomic<int64_t> g_knob_spin{kDefaultSpinLimit};
std::atomic<int64_t> g_knob_sleep{1};       // s_sleep 2 rounds between two polls of a waiting block

template <int T>
const void* fused_fn(int form) {
    return form == kFormStaged   ? reinterpret_cast<const void*>(&gae_staged_slots_kernel<T>)
           : form == kFormNarrow ? reinterpret_cast<const void*>(&gae_fused_slots_kernel<T, kWave>)
                                 : reinterpret_cast<const void*>(&gae_fused_slots_kernel<T, kBlock>);
}

int form_threads(int form) { return form == kFormNarrow ? kWave : kBlock; }

int64_t form_blocks(int form, int64_t N) {
    return form == kFormStaged ? N / kStagedEnvs : ceil_div(N, form_threads(form));
}

const void* fused_fn_t(int T, int form) {
    return T == 8 ? fused_fn<8>(form) : T == 16 ? fused_fn<16>(form) : T == 24 ? fused_fn<24>(form) : fused_fn<32>(form);
}

// blocks of the form's kernel for T the current device holds at once (0: no such instance), computed once per
// (device, T, form); concurrent first calls compute the same value
int gae_fused_capacity(int T, int form) {
    constexpr int kMaxDev = 64;
    static std::atomic<int> cap[kMaxDev][4][4];
    static std::once_flag init;
    std::call_once(init, [] {
        for (auto& d : cap)
            for (auto& c : d)
                for (auto& f : c) f.store(-1, std::memory_order_relaxed);
    });
    const int k = T == 8 ? 0 : T == 16 ? 1 : T == 24 ? 2 : T == 32 ? 3 : -1;
    int dev = 0;
    if (k < 0 || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 0;
    const int fi = form;
    int c = cap[dev][k][fi].load(std::memory_order_relaxed);
    if (c < 0) {
        int cus = 0, per = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fused_fn_t(T, form), form_threads(form), 0) != hipSuccess)
            per = 0;
        c = per * cus;
        cap[dev][k][fi].store(c, std::memory_order_relaxed);
    }
    return c;
}

bool coop_supported() {
    constexpr int kMaxDev = 64;
    static std::atomic<int> sup[kMaxDev];
    static std::once_flag init;
    std::call_once(init, [] {
        for (auto& s : sup) s.store(-1, std::memory_order_relaxed);
    });
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return false;
    int s = sup[dev].load(std::memory_order_relaxed);
    if (s < 0) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeCooperativeLaunch, dev) != hipSuccess) v = 0;
        s = v != 0;
        sup[dev].store(s, std::memory_order_relaxed);
    }
    return s != 0;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// The form rslrl_compute_returns_slots takes for these arguments (rslrl_compute_returns_slots_form reports it).
int slots_form(int64_t T, int64_t N, const float* values, const float* rewards, const uint8_t* dones,
               const float* log_prob, const float* returns, const float* advantages) {
    static const bool fused_env = [] {
        const char* e = std::getenv("RSLRL_GAE_FUSED");
        return !(e && e[0] == '0');
    }();
    const int64_t knob = g_knob_form.load(std::memory_order_relaxed);
    if (!fused_env || knob == 0) return kFormTwoLaunch;
    if (!(T == 8 || T == 16 || T == 24 || T == 32) || N <= 0 || ceil_div(N, kBlock) > kMaxPartials)
        return kFormTwoLaunch;
    const int t = static_cast<int>(T);
    const bool aligned = aligned16(values) && aligned16(rewards) && aligned16(dones) && aligned16(log_prob) &&
                         aligned16(returns) && aligned16(advantages);
    auto fits = [&](int form) {
        if (form == kFormStaged && (N % kStagedEnvs != 0 || !aligned)) return false;
        if (form == kFormNarrow && N > kNarrowMaxN) return false;
        return form_blocks(form, N) <= gae_fused_capacity(t, form);
    };
    if (knob > 0) return knob <= kFormNarrow && fits(static_cast<int>(knob)) ? static_cast<int>(knob) : kFormTwoLaunch;
    // auto, by measurement (profiles/r6_gae_probe.json, rocprof kernel durations at 16,384 / 32,768 / 65,536 envs, T 24):
    // one env per lane in 256-thread blocks is the fastest form at every size (17.9 us at C3 vs 26.4 staged, 21.8
    // narrow; 12.2 us at 16,384 envs vs 14.3 / 14.1); the staged and narrow forms stay selectable (gae_form 2 / 3)
    if (fits(kFormOneLaunch)) return kFormOneLaunch;
    return kFormTwoLaunch;
}

// launches the one-launch form; false when the runtime refused it (the caller runs the two-launch path)
bool launch_fused(int form, int T, int64_t N, hipStream_t st, const float* values, const float* rewards,
                  const uint8_t* dones, const float* last_values, float gamma, float lam, float* returns,
                  float* advantages, const float* logp, float4* slots, double4* part, unsigned* bar) {
    const unsigned nb = static_cast<unsigned>(form_blocks(form, N));
    float eps = 1e-8f;
    unsigned spin = static_cast<unsigned>(g_knob_spin.load(std::memory_order_relaxed));
    unsigned sleep_units = static_cast<unsigned>(g_knob_sleep.load(std::memory_order_relaxed));
    void* args[] = {&values, &rewards, &dones, &last_values, &gamma, &lam, &N, &eps, &returns,
                    &advantages, &logp, &slots, &part, &bar, &spin, &sleep_units};
    // cooperative launches are opt-in (RSLRL_GAE_COOP=1): on this runtime one costs ~6-17 us more per call than the
    // whole kernel's barrier (profiles/r6_gae_probe*.json); the status word + NaN outputs are the default safety net
    static const bool coop_env = [] {
        const char* e = std::getenv("RSLRL_GAE_COOP");
        return e && e[0] == '1';
    }();
    const int64_t coop_knob = g_knob_coop.load(std::memory_order_relaxed);
    const bool coop = (coop_knob == 1 || (coop_knob < 0 && coop_env)) && coop_supported();
    const void* f = fused_fn_t(T, form);
    const dim3 block(form_threads(form));
    const hipError_t e = coop ? hipLaunchCooperativeKernel(f, dim3(nb), block, args, 0, st)
                              : hipLaunchKernel(f, dim3(nb), block, args, 0, st);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // clear the refused launch; nothing ran
        return false;
    }
    return true;
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
    // the partials, then the one-launch forms' barrier words (ticket, status, results; a generation word per group)
    return kBarOffset + 4 * (kGenOffset + kGenStride * kMaxGenGroups);
}

#ifdef RSLRL_GAE_STAMPS
extern "C" int rslrl_gae_debug_stamps(void* buf) {  // diagnostic build only
    uint64_t* p = static_cast<uint64_t*>(buf);
    return static_cast<int>(hipMemcpyToSymbol(HIP_SYMBOL(g_gae_stamps), &p, sizeof(p)));
}
#endif

extern "C" size_t rslrl_compute_returns_status_offset(void) { return kBarOffset + 4 * kStatusWord; }

extern "C" int rslrl_compute_returns_slots_form(int64_t T, int64_t N, const float* values, const float* rewards,
                                                const uint8_t* dones, const float* log_prob, const float* returns,
                                                const float* advantages) {
    if (T <= 0 || N <= 0) return kFormTwoLaunch;
    return slots_form(T, N, values, rewards, dones, log_prob, returns, advantages);
}

extern "C" int rslrl_debug_knob(const char* name, int64_t value, int64_t* previous) {
    if (!name) return RSLRL_E_INVALID_ARGUMENT;
    const std::string k(name);
    std::atomic<int64_t>* knob = k == "gae_form" ? &g_knob_form : k == "gae_coop" ? &g_knob_coop
                               : k == "gae_spin_limit" ? &g_knob_spin : k == "gae_sleep" ? &g_knob_sleep : nullptr;
    if (!knob) return RSLRL_E_INVALID_ARGUMENT;
    if ((k == "gae_spin_limit" || k == "gae_sleep") && (value < 0 || value > 0xffffffffll))
        return RSLRL_E_INVALID_ARGUMENT;
    const int64_t prev = knob->exchange(value);
    if (previous) *previous = prev;
    return RSLRL_OK;
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
    if (slot && slot->record_floats == 0) {
        const int form = slots_form(T, N, values, rewards, dones, slot->log_prob, returns, advantages);
        // one launch: scan + grid barrier + normalisation + slots (bit-identical to the two-launch path below); a
        // refused cooperative launch runs the two-launch path
        if (form != kFormTwoLaunch &&
            launch_fused(form, t, N, st, values, rewards, dones, last_values, gamma, lam, returns, advantages,
                         slot->log_prob, reinterpret_cast<float4*>(slot->records), part,
                         reinterpret_cast<unsigned*>(static_cast<char*>(workspace) + kBarOffset)))
            return RSLRL_OK;
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
