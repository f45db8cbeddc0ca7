// Rollout-side fusion: one launch per environment step replaces the tail of
// PPO.act + PPO.process_env_step + RolloutStorage.add_transitions + RND.get_intrinsic_reward:
//
//   logp      = sum_a Normal(mu, sigma).log_prob(actions)          actor_critic.py:150-151 (act, ppo.py:135)
//   r_int     = weight * || target(s) - predictor(s) ||_2          rnd.py:113-135 (s = normalised RND state)
//   reward    = (rewards + r_int) + gamma * (values * time_outs)   ppo.py:147-164
//   storage[t] <- obs groups, actions, reward, uint8(dones), values, logp, mu, sigma (expanded)
//                                                                   rollout_storage.py:77-103
//
// Two index spaces share the grid: the first `copy_blocks` workgroups stream the row-contiguous slabs
// (observation groups, actions, mu, sigma) with 16-byte accesses; the rest run one thread per env for
// the per-row work (log-prob over A, the two RND MLPs from LDS-resident weights, the reward arithmetic).
// Every fp32 operation of the reference expressions is issued separately in the reference's order
// (__f*_rn), except the RND MLP dot products (fmaf chain, fp32 GEMM-class rounding) and the sum over
// actions (sequential; torch's reduction order is unspecified).
#include <algorithm>

#include "common.h"
#include "launch_timing.h"
#include "rnd_mlp.h"

namespace rslrl {
namespace {

constexpr int kMaxRndIn = 64;
constexpr int kMaxRndHidden = 64;
constexpr int kMaxRndOut = 8;
constexpr int kMaxA = 64;

__device__ __forceinline__ float load_flag(const void* p, int dtype, int64_t i) {
    switch (dtype) {
        case RSLRL_DTYPE_U8: return static_cast<float>(static_cast<const uint8_t*>(p)[i]);
        case RSLRL_DTYPE_I32: return static_cast<float>(static_cast<const int32_t*>(p)[i]);
        case RSLRL_DTYPE_I64: return static_cast<float>(static_cast<const int64_t*>(p)[i]);
        default: return static_cast<const float*>(p)[i];
    }
}

// Record-mode copy segments (obs groups, actions, mu, sigma) in 16-byte units of a destination record
constexpr int kMaxSeg = RSLRL_ROLLOUT_MAX_OBS + 3;
#ifndef RSLRL_REC_ROWS
#define RSLRL_REC_ROWS 64
#endif
#ifndef RSLRL_REC_NT
#define RSLRL_REC_NT 1  // nontemporal record stores (0: plain stores, the round-4 form; an A/B knob)
#endif
#ifndef RSLRL_REC_ENV_FIRST
#define RSLRL_REC_ENV_FIRST 1  // the per-env blocks take the low block indices (dispatched first; 0: copy blocks first)
#endif
#ifndef RSLRL_REC_DIAG
#define RSLRL_REC_DIAG 0  // diagnostic builds only (wrong results): 1 skips the copy blocks' log-prob, 2 the per-env blocks
#endif
constexpr int kRecRows = RSLRL_REC_ROWS;  // records per copy block (<= 64: four lanes per record in the log-prob)
struct RecSegs {
    const float4* src[kMaxSeg];
    float4* dst0;                // record row 0 of step t (record start, 16-byte aligned)
    int32_t start[kMaxSeg];      // first unit of each segment inside the record
    int32_t end[kMaxSeg];        // one past its last unit
    int32_t src_units[kMaxSeg];  // source row stride in units (0: one row shared by all envs)
    int32_t nseg;
    int32_t r4;  // record stride in units: every unit of a record is written (zeros past the segments), so
                 // the copy leaves whole 64-byte sectors and no partial-line write-backs
    float rcp_r4;
};

// RND networks of the per-env part: 0 none, 1 config C5's 48 -> 48 -> 1 (exact widths), 2 any size the ABI admits
template <int RNDK>
struct RndShape {
    static constexpr int INP = RNDK == 1 ? 48 : 64, HP = RNDK == 1 ? 48 : 64, Q = RNDK == 1 ? 1 : kMaxRndOut;
    static constexpr bool EXACT = RNDK == 1;
};

template <int RNDK>
__global__ __launch_bounds__(kBlock) void rollout_record_kernel(rslrl_rollout_args_t a, int copy_blocks, RecSegs rs) {
    extern __shared__ __attribute__((aligned(16))) float lds_w[];  // RND target then predictor images (rnd_mlp.h)
    const int64_t N = a.N;
    // block index in the copy-blocks-first numbering; RSLRL_REC_ENV_FIRST=1 dispatches the per-env blocks first
#if RSLRL_REC_ENV_FIRST
    const int row_blocks = static_cast<int>(gridDim.x) - copy_blocks;
    const int bid = static_cast<int>(blockIdx.x) >= row_blocks ? static_cast<int>(blockIdx.x) - row_blocks
                                                               : static_cast<int>(blockIdx.x) + copy_blocks;
#else
    const int bid = static_cast<int>(blockIdx.x);
#endif
    if (bid < copy_blocks && a.record_floats > 0) {
        // ---- record mode: block b writes records [64 b, 64 b + 64) unit by unit (contiguous stores); the unit ->
        // segment map and the segment table live in LDS
        __shared__ int8_t useg[RSLRL_MAX_RECORD_FLOATS / 4];
        __shared__ const float4* ssrc[kMaxSeg];
        __shared__ int32_t sstart[kMaxSeg], ssu[kMaxSeg];
#pragma unroll
        for (int q = 0; q < kMaxSeg; ++q)
            if (static_cast<int>(threadIdx.x) == q) {
                ssrc[q] = rs.src[q];
                sstart[q] = rs.start[q];
                ssu[q] = rs.src_units[q];
            }
        for (int u = threadIdx.x; u < rs.r4; u += kBlock) {
            int sg = -1;
#pragma unroll
            for (int q = 0; q < kMaxSeg; ++q)
                if (q < rs.nseg && u >= rs.start[q] && u < rs.end[q]) sg = q;
            useg[u] = static_cast<int8_t>(sg);
        }
        __syncthreads();
        const int64_t n0 = static_cast<int64_t>(bid) * kRecRows;
        const int rows = static_cast<int>(min<int64_t>(kRecRows, N - n0));
        const int total = rows * rs.r4;  // <= 64 * 64: exact float division below
        float4* dst = rs.dst0 + n0 * rs.r4;
        // the actions / mu / sigma units of these records also go to LDS ([3][64][A], dynamic LDS): the log-prob is
        // computed here from the values the copy already loaded, instead of the per-env threads reading the actions
        // and mu rows a second time
        const int seg_x = rs.nseg - 3;  // segments: obs groups, then actions, mu, sigma (host order)
        const int A = a.A;
        // every load of a pass is issued before its stores (a store between two loads would order them)
        constexpr int kPass = 8;
        for (int k0 = threadIdx.x; k0 < total; k0 += kPass * kBlock) {
            float4 v[kPass];
#pragma unroll
            for (int j = 0; j < kPass; ++j) {
                const int k = k0 + j * kBlock;
                v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (k < total) {
                    const int r = static_cast<int>((static_cast<float>(k) + 0.5f) * rs.rcp_r4);
                    const int u = k - r * rs.r4;
                    const int sg = useg[u];
                    if (sg >= 0) v[j] = ssrc[sg][(n0 + r) * ssu[sg] + (u - sstart[sg])];
                }
            }
#pragma unroll
            for (int j = 0; j < kPass; ++j) {
                const int k = k0 + j * kBlock;
                if (k < total) {
#if RSLRL_REC_NT
                    // nontemporal: the records are read back only by the update's gather, T env steps later
                    __builtin_nontemporal_store(v[j].x, &dst[k].x);
                    __builtin_nontemporal_store(v[j].y, &dst[k].y);
                    __builtin_nontemporal_store(v[j].z, &dst[k].z);
                    __builtin_nontemporal_store(v[j].w, &dst[k].w);
#else
                    dst[k] = v[j];
#endif
                    const int r = static_cast<int>((static_cast<float>(k) + 0.5f) * rs.rcp_r4);
                    const int u = k - r * rs.r4;
                    const int sg = useg[u];
                    if (sg >= seg_x)
                        *reinterpret_cast<float4*>(lds_w + ((sg - seg_x) * kRecRows + r) * A + 4 * (u - sstart[sg])) = v[j];
                }
            }
        }
        if constexpr ((RSLRL_REC_DIAG & 1) != 0) return;
        __syncthreads();
        {
            // log-prob of the action under Normal(mu, sigma), torch's expression (see the per-env part below): the
            // per-action terms (a division and a log each) on the row's four lanes (action j on lane j & 3), then
            // summed in action order -- each group of four terms broadcast across the quad (DPP quad_perm, no LDS
            // round trip or second barrier), so every lane of the quad adds t_0, t_1, ... in sequence and lane 0
            // stores.  Quads past `rows` compute on stale LDS and store nothing (a whole quad is one row).
            const int r = threadIdx.x >> 2, q = threadIdx.x & 3;
            const float c = 0.918938533204672742f;
            const float* xr = lds_w + r * A;
            const float* mr = lds_w + (kRecRows + r) * A;
            const float* sr = lds_w + (2 * kRecRows + r) * A;
            float lp = 0.f;
            for (int j0 = 0; j0 < A; j0 += 4) {  // A % 4 == 0 in record mode (checked on the host)
                const int j = j0 + q;
                const float sj = sr[j];
                const float d = __fsub_rn(xr[j], mr[j]);
                const float num = -__fmul_rn(d, d);
                const float den = __fmul_rn(2.f, __fmul_rn(sj, sj));
                const int t = __builtin_bit_cast(int, __fsub_rn(__fsub_rn(__fdiv_rn(num, den), logf(sj)), c));
                lp = __fadd_rn(lp, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0x00, 0xF, 0xF, false)));
                lp = __fadd_rn(lp, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0x55, 0xF, 0xF, false)));
                lp = __fadd_rn(lp, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0xAA, 0xF, 0xF, false)));
                lp = __fadd_rn(lp, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(t, 0xFF, 0xF, 0xF, false)));
            }
            if (r < rows && q == 0) a.out_logp[n0 + r] = lp;
        }
        return;
    }
    if (bid < copy_blocks) {
        // ---- slab copies: obs groups [N, d], actions / mu [N, A], sigma expanded [N, A]
        const int64_t tid = static_cast<int64_t>(bid) * kBlock + threadIdx.x;
        const int64_t stride = static_cast<int64_t>(copy_blocks) * kBlock;
        for (int g = 0; g < a.n_obs; ++g) {
            const int64_t n4 = N * a.obs[g].row_floats / 4;  // row_floats % 4 == 0 checked on the host
            const float4* s = reinterpret_cast<const float4*>(a.obs[g].src);
            float4* d = reinterpret_cast<float4*>(a.obs[g].dst);
            for (int64_t i = tid; i < n4; i += stride) d[i] = s[i];
        }
        const int64_t na = N * a.A;
        if ((a.A & 3) == 0) {
            const int64_t n4 = na / 4;
            const float4* sa = reinterpret_cast<const float4*>(a.actions);
            const float4* sm = reinterpret_cast<const float4*>(a.mu);
            float4* da = reinterpret_cast<float4*>(a.out_actions);
            float4* dm = reinterpret_cast<float4*>(a.out_mu);
            float4* ds = reinterpret_cast<float4*>(a.out_sigma);
            const float4* ss = reinterpret_cast<const float4*>(a.sigma);
            const int a4 = a.A / 4;
            for (int64_t i = tid; i < n4; i += stride) {
                da[i] = sa[i];
                dm[i] = sm[i];
                ds[i] = a.sigma_mode ? ss[i] : ss[i % a4];
            }
        } else {
            for (int64_t i = tid; i < na; i += stride) {
                a.out_actions[i] = a.actions[i];
                a.out_mu[i] = a.mu[i];
                a.out_sigma[i] = a.sigma_mode ? a.sigma[i] : a.sigma[i % a.A];
            }
        }
        return;
    }

    // ---- per-env work
    if constexpr ((RSLRL_REC_DIAG & 2) != 0) return;
    using RS = RndShape<RNDK>;
    const int nw = rnd_net_floats(RS::INP, RS::HP, RNDK == 1 ? 1 : a.rnd_out);
    if constexpr (RNDK != 0) {
        const int Q = RNDK == 1 ? 1 : a.rnd_out;
        // the packed nets [W1 | b1 | W2 | b2] (rslrl_rollout_args_t) into their LDS images
        const int in = a.rnd_in, H = a.rnd_hidden;
        rnd_stage_net_t(lds_w, a.rnd_target, a.rnd_target + H * in, a.rnd_target + H * in + H,
                      a.rnd_target + H * in + H + Q * H, in, H, Q, RS::INP, RS::HP);
        rnd_stage_net_t(lds_w + nw, a.rnd_predictor, a.rnd_predictor + H * in, a.rnd_predictor + H * in + H,
                      a.rnd_predictor + H * in + H + Q * H, in, H, Q, RS::INP, RS::HP);
        __syncthreads();
    }
    const int64_t n = static_cast<int64_t>(bid - copy_blocks) * kBlock + threadIdx.x;
    if (n >= N) return;

    // log-prob of the action under Normal(mu, sigma): torch's
    //   -((x - mu) ** 2) / (2 * var) - log(sigma) - log(sqrt(2 pi)),  var = sigma ** 2, summed over A
    // (record mode: computed by the copy blocks above)
    const bool rec = a.record_floats > 0;
    float lp = 0.f;
    if (!rec) {
        const float c = 0.918938533204672742f;  // math.log(math.sqrt(2 * math.pi)) rounded to fp32
        const float* xr = a.actions + n * a.A;
        const float* mr = a.mu + n * a.A;
        const float* sr = a.sigma_mode ? a.sigma + n * a.A : a.sigma;
        for (int j = 0; j < a.A; ++j) {
            const float s = sr[j];
            const float d = __fsub_rn(xr[j], mr[j]);
            const float num = -__fmul_rn(d, d);
            const float den = __fmul_rn(2.f, __fmul_rn(s, s));
            const float t = __fsub_rn(__fsub_rn(__fdiv_rn(num, den), logf(s)), c);
            lp = __fadd_rn(lp, t);
        }
    }

    float reward = a.rewards[n];
    if (a.extra_reward) reward = __fadd_rn(reward, a.extra_reward[n]);
    if constexpr (RNDK != 0) {
        const int in = RS::EXACT ? RS::INP : a.rnd_in;
        const int Q = RNDK == 1 ? 1 : a.rnd_out;
        float x[RS::INP];
        const float* sx = a.rnd_obs + n * a.rnd_obs_stride;
        if constexpr (RS::EXACT) {  // 16-byte aligned rows (checked on the host): 16-byte loads
#pragma unroll
            for (int k = 0; k < RS::INP / 4; ++k) {
                const float4 v = reinterpret_cast<const float4*>(sx)[k];
                x[4 * k] = v.x;
                x[4 * k + 1] = v.y;
                x[4 * k + 2] = v.z;
                x[4 * k + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < RS::INP; ++i) x[i] = i < in ? sx[i] : 0.f;
        }
        if (a.rnd_state_mean) {  // (x - mean) / (std + eps), normalization.py forward
#pragma unroll
            for (int i = 0; i < RS::INP; ++i)
                if (i < in)
                    x[i] = __fdiv_rn(__fsub_rn(x[i], a.rnd_state_mean[i]), __fadd_rn(a.rnd_state_std[i], a.rnd_state_eps));
        }
        float yt[RS::Q], yp[RS::Q];
        {
            float h[RS::HP];
            rnd_hidden_t<RS::INP, RS::HP, RS::EXACT>(lds_w, in, x, h);
#pragma unroll
            for (int k = 0; k < RS::HP; ++k) h[k] = rnd_elu(h[k]);
            rnd_output<RS::INP, RS::HP, RS::Q>(lds_w, Q, h, yt);
        }
        {
            float h[RS::HP];
            rnd_hidden_t<RS::INP, RS::HP, RS::EXACT>(lds_w + nw, in, x, h);
#pragma unroll
            for (int k = 0; k < RS::HP; ++k) h[k] = rnd_elu(h[k]);
            rnd_output<RS::INP, RS::HP, RS::Q>(lds_w + nw, Q, h, yp);
        }
        float ss = 0.f;
#pragma unroll
        for (int q = 0; q < RS::Q; ++q)
            if (q < Q) {
                const float d = __fsub_rn(yt[q], yp[q]);
                ss = __fadd_rn(ss, __fmul_rn(d, d));
            }
        const float r_int = __fmul_rn(__fsqrt_rn(ss), a.rnd_weight);
        if (a.intrinsic_out) a.intrinsic_out[n] = r_int;
        reward = __fadd_rn(reward, r_int);
    }
    const float v = a.values[n];
    if (a.time_outs) reward = __fadd_rn(reward, __fmul_rn(a.gamma, __fmul_rn(v, load_flag(a.time_outs, a.time_outs_dtype, n))));

    a.out_rewards[n] = reward;
    a.out_values[n] = v;
    if (!rec) a.out_logp[n] = lp;
    a.out_dones[n] = load_flag(a.dones, a.dones_dtype, n) != 0.f ? 1 : 0;
}

}  // namespace
}  // namespace rslrl

using namespace rslrl;

extern "C" int rslrl_rollout_record(const rslrl_rollout_args_t* args, rslrl_stream_t stream) {
    if (!args) return RSLRL_E_INVALID_ARGUMENT;
    const rslrl_rollout_args_t& a = *args;
    if (a.N < 0 || a.A < 1 || a.A > kMaxA || a.n_obs < 0 || a.n_obs > RSLRL_ROLLOUT_MAX_OBS) return RSLRL_E_INVALID_ARGUMENT;
    if (a.N == 0) return RSLRL_OK;
    if (!a.actions || !a.mu || !a.sigma || !a.values || !a.rewards || !a.dones || !a.out_actions || !a.out_rewards ||
        !a.out_dones || !a.out_values || !a.out_logp || !a.out_mu || !a.out_sigma)
        return RSLRL_E_INVALID_ARGUMENT;
    for (int g = 0; g < a.n_obs; ++g) {
        if (!a.obs[g].src || !a.obs[g].dst || a.obs[g].row_floats < 1 || (a.obs[g].row_floats & 3))
            return RSLRL_E_INVALID_ARGUMENT;
        if ((reinterpret_cast<uintptr_t>(a.obs[g].src) | reinterpret_cast<uintptr_t>(a.obs[g].dst)) & 15)
            return RSLRL_E_MISALIGNED;
    }
    RecSegs rs{};
    if (a.record_floats > 0) {
        if ((a.record_floats & 3) || (a.A & 3) || a.record_floats > RSLRL_MAX_RECORD_FLOATS) return RSLRL_E_INVALID_ARGUMENT;
        // the destinations must be fields of the record at out_records, in order and not overlapping
        const float* base = a.out_records;
        if (!base || (reinterpret_cast<uintptr_t>(base) & 15)) return RSLRL_E_INVALID_ARGUMENT;
        int32_t units = 0;
        bool ok = true;
        auto add = [&](const float* src, const float* dst, int64_t floats, bool shared) {
            const int64_t off = dst - base;
            if (off < 0 || (off & 3) || off / 4 < units || off + floats > a.record_floats) ok = false;
            rs.src[rs.nseg] = reinterpret_cast<const float4*>(src);
            rs.start[rs.nseg] = static_cast<int32_t>(off / 4);
            rs.end[rs.nseg] = static_cast<int32_t>((off + floats) / 4);
            rs.src_units[rs.nseg] = shared ? 0 : static_cast<int32_t>(floats / 4);
            units = rs.end[rs.nseg];
            ++rs.nseg;
        };
        for (int g = 0; g < a.n_obs; ++g) add(a.obs[g].src, a.obs[g].dst, a.obs[g].row_floats, false);
        add(a.actions, a.out_actions, a.A, false);
        add(a.mu, a.out_mu, a.A, false);
        add(a.sigma, a.out_sigma, a.A, a.sigma_mode == 0);
        if (!ok) return RSLRL_E_INVALID_ARGUMENT;
        rs.dst0 = reinterpret_cast<float4*>(a.out_records);
        rs.r4 = static_cast<int32_t>(a.record_floats / 4);
        rs.rcp_r4 = 1.0f / static_cast<float>(rs.r4);
    }
    if (((a.A & 3) == 0 || a.record_floats > 0) && ((reinterpret_cast<uintptr_t>(a.actions) | reinterpret_cast<uintptr_t>(a.mu) |
                            reinterpret_cast<uintptr_t>(a.sigma) | reinterpret_cast<uintptr_t>(a.out_actions) |
                            reinterpret_cast<uintptr_t>(a.out_mu) | reinterpret_cast<uintptr_t>(a.out_sigma)) & 15))
        return RSLRL_E_MISALIGNED;
    size_t lds = 0;
    if (a.rnd_target) {
        if (!a.rnd_predictor || !a.rnd_obs || a.rnd_in < 1 || a.rnd_in > kMaxRndIn || a.rnd_hidden < 1 ||
            a.rnd_hidden > kMaxRndHidden || a.rnd_out < 1 || a.rnd_out > kMaxRndOut)
            return RSLRL_E_UNSUPPORTED;
        if ((a.rnd_state_mean == nullptr) != (a.rnd_state_std == nullptr)) return RSLRL_E_INVALID_ARGUMENT;
    }
    const bool c5 = a.rnd_target && a.rnd_in == 48 && a.rnd_hidden == 48 && a.rnd_out == 1 &&
                    (reinterpret_cast<uintptr_t>(a.rnd_obs) & 15) == 0 && (a.rnd_obs_stride & 3) == 0;
    if (a.rnd_target)
        lds = 2 * sizeof(float) * static_cast<size_t>(c5 ? rnd_net_floats(48, 48, 1) : rnd_net_floats(64, 64, a.rnd_out));
    int64_t copy_elems = a.N * a.A;
    for (int g = 0; g < a.n_obs; ++g) copy_elems += a.N * a.obs[g].row_floats;
    const int64_t cb = a.record_floats > 0 ? ceil_div(a.N, kRecRows)
                                           : std::min<int64_t>(1024, std::max<int64_t>(1, ceil_div(copy_elems / 4, kBlock * 4)));
    if (cb > INT32_MAX / 2) return RSLRL_E_INVALID_ARGUMENT;
    const int copy_blocks = static_cast<int>(cb);
    const int64_t row_blocks = ceil_div(a.N, kBlock);
    if (row_blocks + copy_blocks > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
    if (a.record_floats > 0)  // the copy blocks' [3][64][A] stage of actions / mu / sigma (log-prob)
        lds = std::max(lds, sizeof(float) * 3 * kRecRows * static_cast<size_t>(a.A));
#ifdef RSLRL_REC_LDS_PAD
    if (a.record_floats > 0) lds = std::max<size_t>(lds, RSLRL_REC_LDS_PAD);  // occupancy experiment
#endif
    const dim3 grid(static_cast<unsigned>(copy_blocks + row_blocks));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // (launch_timed: bound to a timing event pair while bench.py's timed region has the library's timing armed)
    if (!a.rnd_target)
        launch_timed(kTagRolloutRecord, rollout_record_kernel<0>, grid, dim3(kBlock), lds, st, a, copy_blocks, rs);
    else if (c5)
        launch_timed(kTagRolloutRecord, rollout_record_kernel<1>, grid, dim3(kBlock), lds, st, a, copy_blocks, rs);
    else
        launch_timed(kTagRolloutRecord, rollout_record_kernel<2>, grid, dim3(kBlock), lds, st, a, copy_blocks, rs);
    return launch_status();
}

// ---- the rollout's action sample (ActorCritic.act: Normal(mu, sigma).sample() = normal_(0, 1) * sigma + mu, the
// distribution.py sample of torch.normal): x <- x * scale + loc with torch's two roundings (mul, then add) -- one
// launch for the mul_ + add_ pair.  x [N, A] contiguous (the standard normals, drawn by the framework's generator so
// that the random stream is the reference's); scale / loc rows with their own strides (0: one row for all).
namespace rslrl {
namespace {
__global__ __launch_bounds__(kBlock) void normal_affine_kernel(float* __restrict__ x, const float* __restrict__ scale,
                                                               int64_t s_rs, const float* __restrict__ loc,
                                                               int64_t l_rs, int64_t N, int A) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (t >= N * A) return;
    const int64_t n = t / A;
    const int a = static_cast<int>(t - n * A);
    x[t] = __fadd_rn(__fmul_rn(x[t], scale[n * s_rs + a]), loc[n * l_rs + a]);
}
}  // namespace
}  // namespace rslrl

extern "C" int rslrl_normal_affine(float* x, const float* scale, int64_t scale_row_stride, const float* loc,
                                   int64_t loc_row_stride, int64_t N, int32_t A, rslrl_stream_t stream) {
    if (N < 0 || A < 1 || scale_row_stride < 0 || loc_row_stride < 0) return RSLRL_E_INVALID_ARGUMENT;
    if (N == 0) return RSLRL_OK;
    if (!x || !scale || !loc) return RSLRL_E_INVALID_ARGUMENT;
    hipLaunchKernelGGL(normal_affine_kernel, dim3(static_cast<unsigned>(ceil_div(N * A, kBlock))), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), x, scale, scale_row_stride, loc, loc_row_stride, N, A);
    return launch_status();
}
