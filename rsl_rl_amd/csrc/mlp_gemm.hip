// fp32 MFMA GEMMs with fused epilogues for the actor/critic MLP.
//
// Replaces, for the hidden layers of rsl_rl/networks/mlp.py:106-114 (nn.Linear + ELU), the three
// kernels torch runs per layer and direction -- GEMM, ELU, and in backward ELU' plus the bias-grad
// reduction -- with one kernel each:
//   linear_fwd   Y = act(X W^T + b)                 (act = identity | ELU, alpha 1)
//   linear_dgrad dZp = (dZ W) * ELU'(H)             (H = this layer's input = previous ELU output)
//                + per-tile column sums of dZp      (bias gradient of the previous layer)
// The pre-activation never reaches HBM in forward, dH never reaches HBM in backward.  The weight
// gradients stay split-K batched GEMMs (networks/linear.py).
//
// Exact fp32 arithmetic on v_mfma_f32_32x32x2_f32 (a k-ordered f32 fma chain, MI355X_MICROARCH.md);
// the k order inside a 4-deep group differs from a plain GEMM, i.e. rounding differs at fp32 epsilon.
//
// Tile: 128 rows x 256 columns per 512-thread workgroup (8 waves as 2 (M) x 4 (N), each wave 64 x 64 =
// 2 x 2 MFMA tiles), K staged in 16-deep chunks through double-buffered LDS (rows padded to 18 floats:
// the 8-byte operand reads of 32 lanes hit 32 distinct bank pairs).  For a k-group of 4 each lane reads
// A[i][4t + 2h .. +1] and B[j][4t + 2h .. +1] with one ds_read_b64 each and feeds two MFMA k-steps
// (step 2t uses k = 4t + 2h, step 2t+1 uses k = 4t + 2h + 1 -- the same mapping for A and B).

#include <algorithm>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "common.h"
#include "amax.h"
#include "fwd_stream.h"
#include "x6_split.h"
#include "ppo_loss_common.h"

namespace rslrl {
namespace {


constexpr int kBM = 128;
constexpr int kBN = 256;
constexpr int kKC = 16;
constexpr int kPad = 2;
constexpr int kLd = kKC + kPad;  // LDS row stride (floats)
constexpr int kThreads = 512;

// kEpiEluGradWgrad: kEpiEluGrad for a short reduction (Nred <= 16, one chunk: the output layer) that also
// accumulates that layer's weight gradient dZ^T H from the same H tile (x6 path only)
// kEpiBiasEluOut: kEpiBiasElu for the last hidden layer that also applies the (<= 32 wide) output layer to
// the activation tile while it is in registers (x6 path only; the main loop computes C^T tiles)
enum Epilogue { kEpiBias = 0, kEpiBiasElu = 1, kEpiEluGrad = 2, kEpiEluGradWgrad = 3, kEpiBiasEluOut = 4 };
constexpr int kH0StageBytes = 4096;  // kEpiEluGrad: one wave's first H block staged in LDS (stage_h_block0)
constexpr int kMaxWgradRows = 16;
constexpr int kMaxOutWidth = 32;     // kEpiBiasEluOut
constexpr int kStagedOutWidth = 20;  // kEpiBiasEluOut: widths whose reduction tiles fit beside the h stage

struct GemmParams {
    const float* a;    // [M, K] row-major (lda = K)
    const float* bw;   // [N, K] row-major (the nn.Linear weight layout; for dgrad: W^T)
    const float* bias; // [N] (fwd)
    const float* h;    // [M, N] (dgrad: the activation whose ELU' gates the output)
    float* c;          // [M, N] row-major
    float* colsum;     // [gridDim.x, N] (dgrad)
    int64_t M;
    int K;
    int N;
    int64_t ctiles;    // dgrad: columns of colsum (= rslrl_linear_tiles(M), 128-row tiles)
    float* wpart;      // kEpiEluGradWgrad: per-tile weight-gradient partials [tiles][K][N]
    const uint4* oimg;   // kEpiBiasEluOut: output-layer image (out_image_kernel layout)
    const float* obias;  // kEpiBiasEluOut: output bias [nout]
    float* y;            // kEpiBiasEluOut: output [M, nout]
    int nout;            // kEpiBiasEluOut: output width <= 32
    int nt;              // kEpiBiasEluOut: streaming stores for h
    const float* a_amax;  // h3: max |A| (device scalar written by A's producer) -> A's power-of-two scale
    float* amax_out;      // optional: max |C| over the stored output (device scalar, for an h3 consumer)
    unsigned* amax_ws;    // with amax_out: {running max bits, arrival ticket}, zero before and after the launch
    int deep;             // K = 256: the unrolled look-ahead main loop (h3_deep_loop; x6 and h3)
    // value head with its backward (mlp_gemm_x6_value_head_kernel, rslrl_value_head_fwd_bwd)
    const float* vh_tv;   // [M] target values (the rollout's values)
    const float* vh_ret;  // [M] returns
    const float* vh_w;    // [N] the value head's fp32 weight row
    float vh_clip;        // clip_param
    float vh_g;           // value_loss_coef / M
    int vh_clipped;       // use_clipped_value_loss
};

// The actor head with the PPO loss and its backward (mlp_gemm_x6_actor_head_kernel, rslrl_actor_head_fwd_bwd): the
// loss inputs of the mini-batch, the output layer's transposed image and the loss outputs.
constexpr int kActA = 12;                              // actions: 3 per lane of a row's quad
constexpr int kActCols = 4 + kActA;                    // loss partial columns: surrogate, value, entropy, KL, d sigma
constexpr int kActTileFloats = kActA * kBN + kActA;    // per-tile [dW (12 x 256) | db (12)] (a multiple of 4)
struct ActorParams {
    const float* actions;    // [M, 12]
    const float* old_mu;     // [M, 12]
    const float* old_sigma;  // [M, 12]
    const float* sigma;      // [12] shared std
    const float* old_logp;   // [M]
    const float* adv;        // [M]
    const float* values;     // [M]
    const float* target_values;  // [M]
    const float* returns;    // [M]
    const uint4* w_t_img;    // x6 image of W_out^T (layout 0): row n = hidden column, k = action
    float* wpart;            // [tiles][kActTileFloats]
    float* grad_sigma;       // [12]
    float* stats;            // [8]
    float* grad_mu;          // [M, 12] or null
    double* partials;        // [kActCols][tiles], then [kActCols][groups]
    unsigned* tickets;       // 1 + groups, zero between launches
    float clip, ratio_lo, ratio_hi, g_surr, g_ent, value_loss_coef, entropy_coef;
    int clipped_value, compute_kl, kl_fast;
};

// global -> registers for one K chunk: A: 128 x 16 floats = 512 float4 (1 per thread); B: 256 x 16 = 1024
// float4 (2 per thread, only the first N rows real).  Rows >= M / N and k >= K read as zero.
struct Stage {
    float4 a, b0, b1;
};

// Branch-free masked 16-byte load: out-of-range rows / k-groups read a valid address (the row base) and
// are zeroed by a select, so the load stream has no control flow.  Needs K % 4 == 0.
__device__ __forceinline__ float4 load4_masked(const float* __restrict__ row_base, bool ok, int k) {
    const float4 v = *reinterpret_cast<const float4*>(ok ? row_base + k : row_base);
    return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}

__device__ __forceinline__ Stage load_chunk(const GemmParams& p, int64_t row0, int k0) {
    const int t = threadIdx.x;
    const int k = k0 + 4 * (t & 3);
    const bool k_ok = k < p.K;
    Stage s;
    const int r = t >> 2;  // 0..127
    const int64_t row = row0 + r;
    const bool row_ok = row < p.M;
    s.a = load4_masked(p.a + (row_ok ? row : row0) * p.K, row_ok && k_ok, k);
    const int n0 = r, n1 = r + 128;
    s.b0 = load4_masked(p.bw + static_cast<int64_t>(n0 < p.N ? n0 : 0) * p.K, n0 < p.N && k_ok, k);
    s.b1 = load4_masked(p.bw + static_cast<int64_t>(n1 < p.N ? n1 : 0) * p.K, n1 < p.N && k_ok, k);
    return s;
}

__device__ __forceinline__ void store_chunk(const Stage& s, float* __restrict__ a_lds, float* __restrict__ b_lds) {
    const int t = threadIdx.x;
    const int q = t & 3;
    const int r = t >> 2;
    float2* pa = reinterpret_cast<float2*>(a_lds + r * kLd + 4 * q);
    pa[0] = make_float2(s.a.x, s.a.y);
    pa[1] = make_float2(s.a.z, s.a.w);
    float2* pb0 = reinterpret_cast<float2*>(b_lds + r * kLd + 4 * q);
    pb0[0] = make_float2(s.b0.x, s.b0.y);
    pb0[1] = make_float2(s.b0.z, s.b0.w);
    float2* pb1 = reinterpret_cast<float2*>(b_lds + (r + 128) * kLd + 4 * q);
    pb1[0] = make_float2(s.b1.x, s.b1.y);
    pb1[1] = make_float2(s.b1.z, s.b1.w);
}

// expm1(v) for v <= 0 (the ELU's negative branch) in ~9 VALU instead of libm expm1f's ~27: a degree-5 polynomial
// (Horner, explicit fma) on [-0.5, 0], exp(v) - 1 below (the subtraction is exact there, error = exp's ~1 ulp of a
// value <= 0.61 -> <= 2 ulp of the result).
__device__ __forceinline__ float elu_neg(float v) {
    // minimax fit of expm1(v) / v on [-0.5, 0] (degree 5, Horner with explicit fma; round 6): 1.26 ulp at most against
    // expm1 over every 7th fp32 in [-0.5, 0) (the degree-9 Taylor form it replaced: 1.14 ulp) in 3 fewer FMAs
    float t = __fmaf_rn(v, 0.0011216326f, 0.008187376f);
    t = __fmaf_rn(v, t, 0.04162908f);
    t = __fmaf_rn(v, t, 0.16666223f);
    t = __fmaf_rn(v, t, 0.49999982f);
    t = __fmaf_rn(v, t, 1.0f);
    const float poly = v * t;
    const float e = __expf(v) - 1.0f;
    return v > -0.5f ? poly : e;
}

// ---- epilogue of one wave's I x J grid of 32x32 tiles at (wrow0, wcol0).  C/D map of a tile:
// col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).  Tiles are processed in order b = J i + j;
// for the ELU' epilogue the 16 h values of tile b + 1 are loaded before tile b is finished, so no h load
// waits alone.  colpart[j] returns this lane's sum over its rows of column wcol0 + 32 j + (lane & 31).
template <int EPI, int I, int J, bool FULLT, int NR>
__device__ __forceinline__ void epilogue_tiles_impl(const GemmParams& p, f32x16 (&acc)[I][J], int64_t wrow0,
                                                    int wcol0, float (&colpart)[J], const float* dzo, int dzo_row0,
                                                    f32x2 (&wacc)[NR], float& amx) {
    constexpr bool full = FULLT;
    constexpr bool GRAD = EPI == kEpiEluGrad || EPI == kEpiEluGradWgrad;
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5;
    const int l32 = lane & 31;
#pragma unroll
    for (int j = 0; j < J; ++j) colpart[j] = 0.f;
    float hcur[16], hnext[16], hsave[16];
    // full tiles (N == kBN): wave-uniform base pointers (SGPRs) + 32-bit lane offsets with a compile-time row
    // stride -> saddr-form loads/stores whose row-in-group steps fold into the immediate.  A 64-bit address per
    // row (runtime stride) needs 32 VGPRs per tile and spilled ~70 B/lane to scratch around the epilogue.
    const int wr = full ? __builtin_amdgcn_readfirstlane(static_cast<int>(wrow0)) : 0;  // rows < 2^31 (launch)
    const int wc = full ? __builtin_amdgcn_readfirstlane(wcol0) : 0;
    const int64_t ubase = static_cast<int64_t>(wr) * kBN + wc;
    auto lane_off = [&](int i, int j, int roff) -> uint32_t {
        return static_cast<uint32_t>((i * 32 + 4 * h + roff) * kBN + j * 32 + l32);
    };
    auto load_h = [&](int b, float (&dst)[16]) {
        const int i = b / J, j = b % J;
        if constexpr (full) {
            const float* hb = p.h + ubase;
#pragma unroll
            for (int r = 0; r < 16; ++r) dst[r] = hb[lane_off(i, j, (r & 3) + 8 * (r >> 2))];
            return;
        }
        const int col = wcol0 + j * 32 + l32;
        const int64_t rbase = wrow0 + i * 32 + 4 * h;
        const float* hp = p.h + rbase * p.N + col;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int roff = (r & 3) + 8 * (r >> 2);
            dst[r] = (rbase + roff < p.M && col < p.N) ? hp[static_cast<int64_t>(roff) * p.N] : 0.f;
        }
    };
    if constexpr (full && EPI != kEpiEluGradWgrad) {
        // Full tiles: every access through a buffer resource over the wave's rows (wave-uniform base): the
        // lane part of the offset is one VGPR per column tile, the 8-row group step rides in soffset (an SGPR
        // constant) and the row within the group in the 12-bit immediate -- no per-store address arithmetic
        // (the 64-bit vaddr form spent two VALU per store).  The ELU is evaluated branch-free on every lane:
        // as a guarded call the compiler wrapped each element in an exec-mask branch (3 SALU + a skip each).
        const uint32_t rbytes = static_cast<uint32_t>(I * 32 * kBN * 4);
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(p.c + ubase, 0, rbytes, 0x00020000);
        const __amdgpu_buffer_rsrc_t rh =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(GRAD ? p.h + ubase : p.c), 0, rbytes, 0x00020000);
        auto voff = [&](int j, int r) { return static_cast<int>(((4 * h + (r & 3)) * kBN + j * 32 + l32) * 4); };
        auto soff = [&](int i, int r) { return (i * 32 + 8 * (r >> 2)) * kBN * 4; };
        auto load_hb = [&](int b, float (&dst)[16]) {
            const int i = b / J, j = b % J;
#ifdef RSLRL_DBG_NOHLOAD  // diagnostic build only: the input gradient's H loads replaced by register values
#pragma unroll
            for (int r = 0; r < 16; ++r) dst[r] = __builtin_bit_cast(float, voff(j, r) ^ soff(i, r)) - 0.5f;
#else
#pragma unroll
            for (int r = 0; r < 16; ++r)
                dst[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rh, voff(j, r), soff(i, r), 0));
#endif
        };
        if constexpr (EPI == kEpiEluGrad) {
            if (dzo) {  // block 0 was staged in LDS during the last main-loop chunk (row-major 32 x 32)
                // this wave's own DMA must have landed: the barrier after the main loop does not wait for loads
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const float* hs = dzo + (threadIdx.x >> 6) * (kH0StageBytes / 4);
#pragma unroll
                for (int r = 0; r < 16; ++r) hcur[r] = hs[(4 * h + (r & 3) + 8 * (r >> 2)) * 32 + l32];
            } else {
                load_hb(0, hcur);
            }
        } else if constexpr (GRAD) {
            load_hb(0, hcur);
        }
#pragma unroll
        for (int b = 0; b < I * J; ++b) {
            const int i = b / J, j = b % J;
            if constexpr (GRAD) {
                if (b + 1 < I * J) load_hb(b + 1, hnext);
            }
            float bias = 0.f;
            if constexpr (!GRAD) bias = p.bias[wcol0 + j * 32 + l32];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float v = acc[i][j][r];
                if constexpr (EPI == kEpiBias) {
                    v = v + bias;
                } else if constexpr (EPI == kEpiBiasElu) {
                    v = v + bias;
                    const float n = elu_neg(fminf(v, 0.f));  // evaluated on every lane: a select, not a branch
                    v = v > 0.f ? v : n;
                } else {
                    const float hv = hcur[r];
                    const float g = v * (hv + 1.f);
                    v = hv > 0.f ? v : g;
                    colpart[j] += v;
                }
                amx = fmaxf(amx, fabsf(v));
#ifdef RSLRL_DBG_NOSTORE  // diagnostic build only: the full-tile epilogue's stores skipped (values kept live)
                asm volatile("" ::"v"(v));
#else
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rc, voff(j, r), soff(i, r),
                                                      2 /* nt */);
#endif
            }
            if constexpr (GRAD) {
#pragma unroll
                for (int r = 0; r < 16; ++r) hcur[r] = hnext[r];
            }
        }
        return;
    }
    if constexpr (GRAD) load_h(0, hcur);
#pragma unroll
    for (int b = 0; b < I * J; ++b) {
        const int i = b / J, j = b % J;
        if constexpr (GRAD) {
            if (b + 1 < I * J) load_h(b + 1, hnext);
        }
        const int col = wcol0 + j * 32 + l32;
        const bool col_ok = col < p.N;
        float bias = 0.f;
        if constexpr (!GRAD) bias = col_ok ? p.bias[col] : 0.f;
        const int64_t rbase = wrow0 + i * 32 + 4 * h;
        float* cp = p.c + rbase * p.N + col;
        float* cb = p.c + ubase;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int roff = (r & 3) + 8 * (r >> 2);
            if (full || (rbase + roff < p.M && col_ok)) {
                float v = acc[i][j][r];
                if constexpr (EPI == kEpiBias) {
                    v = v + bias;
                } else if constexpr (EPI == kEpiBiasElu) {
                    v = v + bias;
                    v = v > 0.f ? v : elu_neg(v);  // torch ELU, alpha = 1
                } else {  // kEpiEluGrad / kEpiEluGradWgrad
                    const float hv = hcur[r];  // ELU'(z) = 1 if z > 0 else hv + 1
                    v = hv > 0.f ? v : v * (hv + 1.f);
                    colpart[j] += v;
                }
                amx = fmaxf(amx, fabsf(v));
                // streaming store: the outputs are not re-read by this kernel, and keeping them out of L2
                // keeps the B image and the A stream resident (-7% kernel time measured)
                if constexpr (full)
                    __builtin_nontemporal_store(v, cb + lane_off(i, j, roff));
                else
                    __builtin_nontemporal_store(v, cp + static_cast<int64_t>(roff) * p.N);
            }
        }
        if constexpr (EPI == kEpiEluGradWgrad) {
            // dW[o][col] += dZ[row][o] * H[row][col] over this lane's 16 rows (H = 0 outside the matrix); the two
            // column tiles of row tile i share each dZ read and one packed FMA (v_pk_fma_f32)
            static_assert(J == 2, "the fused weight gradient pairs the wave's two column tiles");
            if (j == 0) {
#pragma unroll
                for (int r = 0; r < 16; ++r) hsave[r] = hcur[r];
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int roff = (r & 3) + 8 * (r >> 2);
                    const float4* d =
                        reinterpret_cast<const float4*>(dzo + (dzo_row0 + i * 32 + 4 * h + roff) * kMaxWgradRows);
                    const f32x2 hh = {hsave[r], hcur[r]};
#pragma unroll
                    for (int o4 = 0; o4 < NR / 4; ++o4) {
                        const float4 dv = d[o4];
                        wacc[4 * o4 + 0] = __builtin_elementwise_fma(f32x2{dv.x, dv.x}, hh, wacc[4 * o4 + 0]);
                        wacc[4 * o4 + 1] = __builtin_elementwise_fma(f32x2{dv.y, dv.y}, hh, wacc[4 * o4 + 1]);
                        wacc[4 * o4 + 2] = __builtin_elementwise_fma(f32x2{dv.z, dv.z}, hh, wacc[4 * o4 + 2]);
                        wacc[4 * o4 + 3] = __builtin_elementwise_fma(f32x2{dv.w, dv.w}, hh, wacc[4 * o4 + 3]);
                    }
                }
            }
        }
        if constexpr (GRAD) {
#pragma unroll
            for (int r = 0; r < 16; ++r) hcur[r] = hnext[r];
        }
    }
}

// Full-tile forward (bias + ELU) / input-gradient (ELU') epilogue through a per-wave LDS stage of 4 KiB: each 32 x 32
// block is written in the MFMA's C layout (lane = column, ds_write_b32), read back as 8 rows x 128 B per instruction
// (lane: row 8 k + (lane >> 3), column quad lane & 7; quads XOR-swizzled by (row >> 1) & 7 -- conflict-free both ways)
// and meets HBM as 16-byte accesses: per block 4 loads of H and 4 stores where the C-layout epilogue issues 16 + 16
// 4-byte ones.  The elementwise operations are epilogue_tiles_impl's: the same bits.  Plain launches only (no column
// sums, no amax).  Measured on the input-gradient pair: skipping its H loads and stores altogether took it from 662 to
// 526 us at 393,216 rows (diagnostic builds, RSLRL_DBG_NOSTORE / RSLRL_DBG_NOHLOAD), the I/O's share this attacks --
// but the 16-byte form measured no faster than the 4-byte C-layout one (dgrad pair 629-631 vs 623-624 us, forward
// 634-637 vs 622-626 us, the K = 48 first layer 230 vs 211 us; profiles/r4_staged_epilogue_ab.json): the epilogue's
// cost is its bytes (the clock falls 9 % with them, profiles/r4_epilogue_io_diag.json), not its instruction count.
// Kept as a build knob (RSLRL_STAGED_EPI=1), bit-identical to the default epilogue.
#ifndef RSLRL_STAGED_EPI
#define RSLRL_STAGED_EPI 0  // measured no faster (profiles/r4_staged_epilogue_ab.json): a build knob, off
#endif
constexpr bool kStagedEpi = RSLRL_STAGED_EPI != 0;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

template <int EPI, int I, int J>
__device__ __forceinline__ void epilogue_tiles_staged(const GemmParams& p, f32x16 (&acc)[I][J], int64_t wrow0,
                                                      int wcol0, float* __restrict__ stage) {
    static_assert(EPI == kEpiBiasElu || EPI == kEpiEluGrad, "staged epilogue: forward ELU or input gradient");
    constexpr bool GRAD = EPI == kEpiEluGrad;
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const int cq = lane & 7;   // read layout: column quad
    const int rr = lane >> 3;  // read layout: row within an 8-row group
    const int wr = __builtin_amdgcn_readfirstlane(static_cast<int>(wrow0));  // rows < 2^31 (launch)
    const int wc = __builtin_amdgcn_readfirstlane(wcol0);
    const int64_t ubase = static_cast<int64_t>(wr) * kBN + wc;
    const uint32_t rbytes = static_cast<uint32_t>(I * 32 * kBN * 4);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(p.c + ubase, 0, rbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rh =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(GRAD ? p.h + ubase : p.c), 0, rbytes, 0x00020000);
    auto voff = [&](int j) { return static_cast<int>((rr * kBN + j * 32 + 4 * cq) * 4); };
    auto soff = [&](int i, int k) { return (i * 32 + 8 * k) * kBN * 4; };
    f32x4 hcur[4], hnext[4];
    auto load_h = [&](int b, f32x4 (&dst)[4]) {
        const int i = b / J, j = b % J;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            dst[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rh, voff(j), soff(i, k), 0));
    };
    f32x4 bias[J];
    if constexpr (!GRAD) {
#pragma unroll
        for (int j = 0; j < J; ++j) bias[j] = *reinterpret_cast<const f32x4*>(p.bias + wc + j * 32 + 4 * cq);
    } else {
        load_h(0, hcur);
    }
#pragma unroll
    for (int b = 0; b < I * J; ++b) {
        const int i = b / J, j = b % J;
        if constexpr (GRAD) {
            if (b + 1 < I * J) load_h(b + 1, hnext);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = 4 * h + (r & 3) + 8 * (r >> 2);
#ifdef RSLRL_STAGE_NOSWZ  // diagnostic
            stage[row * 32 + l32] = acc[i][j][r];
#else
            stage[row * 32 + 4 * ((l32 >> 2) ^ ((row >> 1) & 7)) + (l32 & 3)] = acc[i][j][r];
#endif
        }
        // the stage's dword writes retire before its 16-byte reads (without this wait a few elements per tile read
        // stale data on the box: a b32-write / b128-read order is not kept by the LDS on its own)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int row = 8 * k + rr;
#ifdef RSLRL_STAGE_NOSWZ
            f32x4 v = *reinterpret_cast<const f32x4*>(stage + row * 32 + 4 * cq);
#else
            f32x4 v = *reinterpret_cast<const f32x4*>(stage + row * 32 + 4 * (cq ^ ((row >> 1) & 7)));
#endif
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if constexpr (GRAD) {
                    const float hv = hcur[k][e];
                    const float g = v[e] * (hv + 1.f);
                    v[e] = hv > 0.f ? v[e] : g;
                } else {
                    const float t = v[e] + bias[j][e];
                    const float n = elu_neg(fminf(t, 0.f));  // evaluated on every lane: a select, not a branch
                    v[e] = t > 0.f ? t : n;
                }
            }
            const u32x4 sv = __builtin_bit_cast(u32x4, v);
            __builtin_amdgcn_raw_buffer_store_b128(sv, rc, voff(j), soff(i, k), 2 /* nt */);
            // VMEM store-data hazard: the 16-byte store reads its data VGPRs after it issues, and hipcc (ROCm 7.2,
            // gfx950) put a VALU write of the first data register right behind it with no wait state -- the stored
            // element 0 of some lanes then came from the next computation (non-deterministic outputs on the box).
            // The asm keeps the data registers live past wait states of its own (ordered after the store by the
            // memory clobber).
            asm volatile("s_nop 3" ::"v"(sv) : "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the stage's reads are done before the next writes
        if constexpr (GRAD) {
#pragma unroll
            for (int k = 0; k < 4; ++k) hcur[k] = hnext[k];
        }
    }
}

// full (wave-uniform): every row and column of the tile exists.  The two paths are separate code: a
// runtime `full ||` test per element puts a branch around every store, and the compiler then waits
// vmcnt(0) before each store (64 serialised stores per wave: the epilogue ran 3x longer).
// h0 (kEpiEluGrad, full tiles): the LDS copy of each wave's first H block (stage_h_block0), or nullptr
template <int EPI, int I, int J>
__device__ __forceinline__ void epilogue_tiles(const GemmParams& p, f32x16 (&acc)[I][J], int64_t wrow0, int wcol0,
                                               bool full, float (&colpart)[J], float& amx, const float* h0 = nullptr) {
    f32x2 wacc[1];  // unused (no weight-gradient accumulation)
    if (full)
        epilogue_tiles_impl<EPI, I, J, true, 1>(p, acc, wrow0, wcol0, colpart, h0, 0, wacc, amx);
    else
        epilogue_tiles_impl<EPI, I, J, false, 1>(p, acc, wrow0, wcol0, colpart, nullptr, 0, wacc, amx);
}

template <int EPI, int I, int J, int NR>
__device__ __forceinline__ void epilogue_tiles_w(const GemmParams& p, f32x16 (&acc)[I][J], int64_t wrow0, int wcol0,
                                                 bool full, float (&colpart)[J], const float* dzo, int dzo_row0,
                                                 f32x2 (&wacc)[NR], float& amx) {
#pragma unroll
    for (int o = 0; o < NR; ++o) wacc[o] = f32x2{0.f, 0.f};
    if (full)
        epilogue_tiles_impl<EPI, I, J, true, NR>(p, acc, wrow0, wcol0, colpart, dzo, dzo_row0, wacc, amx);
    else
        epilogue_tiles_impl<EPI, I, J, false, NR>(p, acc, wrow0, wcol0, colpart, dzo, dzo_row0, wacc, amx);
}

// f32 kernel epilogue: 128-row tile, waves 2 (m) x 4 (n) of 64 x 64; column sums over the tile's 128 rows
// (lanes l and l+32 hold the two row halves, the two wm waves the two 64-row halves; fixed combine order)
// -> colsum[col][blockIdx.x].  colred: 2 x kBN floats of LDS the caller no longer reads.
template <int EPI>
__device__ __forceinline__ void epilogue(const GemmParams& p, f32x16 (&acc)[2][2], int64_t row0, float* colred) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave >> 2;
    const int wn = wave & 3;
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const bool full = (row0 + kBM <= p.M) && (p.N == kBN);  // wave-uniform: no per-element bounds checks
    float colpart[2];
    float amx = 0.f;
    epilogue_tiles<EPI, 2, 2>(p, acc, row0 + wm * 64, wn * 64, full, colpart, amx);
    if constexpr (EPI == kEpiEluGrad) {
        __syncthreads();  // the LDS tiles are no longer read
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float s = colpart[j] + __shfl_xor(colpart[j], 32, 64);
            if (h == 0) colred[wm * kBN + wn * 64 + j * 32 + l32] = s;
        }
        __syncthreads();
        // tile-major partials [tiles][N]: one contiguous row per workgroup (column-major rows of 4-byte
        // pieces scattered over the whole buffer cost a read-modify-write of a line each)
        for (int col = threadIdx.x; col < p.N && col < kBN; col += kThreads)
            p.colsum[static_cast<int64_t>(blockIdx.x) * p.N + col] = colred[col] + colred[kBN + col];
    }
}

// MINW = minimum waves per SIMD the register allocation must allow (4: two workgroups per CU, <= 128
// VGPRs; 2: one workgroup per CU, <= 256 VGPRs).
template <int EPI, int MINW>
__global__ __launch_bounds__(kThreads, MINW) void mlp_gemm_kernel(GemmParams p) {
    __shared__ __attribute__((aligned(16))) float lds[2][(kBM + kBN) * kLd];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave >> 2;  // 0..1 -> rows wm*64
    const int wn = wave & 3;   // 0..3 -> cols wn*64
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * kBM;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

    const int nchunks = (p.K + kKC - 1) / kKC;
    Stage st = load_chunk(p, row0, 0);
    store_chunk(st, lds[0], lds[0] + kBM * kLd);
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
        const int buf = c & 1;
        const bool more = c + 1 < nchunks;
        if (more) st = load_chunk(p, row0, (c + 1) * kKC);  // in flight during this chunk's MFMAs
        const float* a_lds = lds[buf];
        const float* b_lds = lds[buf] + kBM * kLd;
#pragma unroll
        for (int t = 0; t < kKC / 4; ++t) {
            float2 av[2], bv[2];
#pragma unroll
            for (int i = 0; i < 2; ++i)
                av[i] = *reinterpret_cast<const float2*>(a_lds + (wm * 64 + i * 32 + l32) * kLd + 4 * t + 2 * h);
#pragma unroll
            for (int j = 0; j < 2; ++j)
                bv[j] = *reinterpret_cast<const float2*>(b_lds + (wn * 64 + j * 32 + l32) * kLd + 4 * t + 2 * h);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].x, bv[j].x, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].y, bv[j].y, acc[i][j], 0, 0, 0);
                }
        }
        if (more) {
            // the other buffer was last read in chunk c-1, and every wave passed the barrier after it
            store_chunk(st, lds[buf ^ 1], lds[buf ^ 1] + kBM * kLd);
        }
        __syncthreads();
    }
    epilogue<EPI>(p, acc, row0, lds[0]);
}

// ---- split-bf16 main loop ("x6"): fp32-accurate products on the bf16 MFMA (16x the f32 MFMA rate).
// Every fp32 operand is split into three bf16 planes (x6_split.h); per 16-deep k step and 32x32 tile six
// bf16 MFMAs accumulate a0b0 + a0b1 + a1b0 + a1b1 + a0b2 + a2b0 in fp32 -- the error of an fp32 GEMM
// (tests/test_gpu_fused_mlp.py measures both against fp64) at 2.67x fewer MFMA cycles than
// v_mfma_f32_32x32x2_f32.
//
// Tile: 256 rows x 256 columns per 512-thread workgroup (one per CU), 8 waves as 2 (M) x 4 (N), each wave
// 128 x 64 = 4 x 2 MFMA tiles.  Operands: A (activations, fp32, read once from HBM) is fetched two chunks
// ahead into registers and split while it is stored into LDS; B (the weights, re-read by every
// workgroup from L2) is split once per call by bimage_kernel into an image that is byte-for-byte the
// kernel's LDS image (three 16-B loads + ds_write_b128 per thread and chunk, no VALU).
//
// LDS image per buffer: [A plane 0..2][B plane 0..2], each plane [rows][16 bf16] = 32 B per row; the two
// 16-B halves of a row are swapped on rows with (row >> 3) & 1, which makes both the staging stores
// (ds_write_b64, 16-lane groups) and the fragment reads (ds_read_b128: lane l reads row l & 31, half l >> 5)
// bank-conflict free.
#ifdef RSLRL_STAMPS
__device__ uint64_t* g_stamps;
#endif
constexpr int kX6RowB = 32;
constexpr int kX6PlaneB = kBN * kX6RowB;  // 8 KiB
constexpr int kX6ChunkB = 3 * kX6PlaneB;  // 24 KiB: one chunk of the B image
// h3 B image (RSLRL_BIMAGE_LAYOUT_H3): [chunk][2 fp16 planes][256 rows][32 B swizzled] of t_n B[n][k] (t_n a
// power of two per row n from max_k |B[n][k]|), then 1 / t_n for the 256 rows (fp32).
constexpr int kH3ChunkB = 2 * kX6PlaneB;
__host__ __device__ inline int64_t h3_image_scales_offset(int depth) { return ((depth + kKC - 1) / kKC) * int64_t{kH3ChunkB}; }

__device__ __forceinline__ int swz(int row, int half) { return row * kX6RowB + 16 * (half ^ ((row >> 3) & 1)); }

// B image: [chunk][plane][256 rows][32 B swizzled]; element (row n, k) = transposed ? src[k * rows + n] :
// src[n * depth + k], zero for n >= rows or k >= depth.  One thread per (chunk, row, physical half);
// blockIdx.y selects the image of a batch (one launch builds every image an MLP pass needs).
constexpr int kMaxImages = 16;
struct BImageBatch {
    rslrl_bimage_desc_t d[kMaxImages];
};

// Output-layer image (layout 1, rslrl_linear_fwd_out): for wave column group wn (64 columns), column tile j,
// k step s, plane q, lane half h and output o: 8 bf16 of W_out[o][c], c = 64 wn + 32 j + 4 h + (t & 3) +
// 8 (2 s + (t >> 2)), t < 8 -- the columns lane half h of the C^T epilogue holds in registers 8 s .. 8 s + 7.
// Unit (16 B) index ((((wn * 2 + j) * 2 + s) * 3 + q) * 2 + h) * 32 + o; zero for o >= rows, c >= depth.
// Followed by the same weights in fp32 for the VALU path (<= 4 outputs): 8 floats per (wn, j, s, h, o) at
// unit kOutImagePlaneUnits + 2 ((((wn * 2 + j) * 2 + s) * 2 + h) * 32 + o).
constexpr int kOutImagePlaneUnits = 4 * 2 * 2 * 3 * 2 * 32;
constexpr int kOutImageThreads = 4 * 2 * 2 * 2 * 32;
constexpr int kOutImageUnits = kOutImagePlaneUnits + 2 * kOutImageThreads;

__device__ __forceinline__ void out_image_thread(const rslrl_bimage_desc_t& dsc, int id) {
    if (id >= kOutImageThreads) return;
    const int o = id & 31, h = (id >> 5) & 1, s = (id >> 6) & 1, j = (id >> 7) & 1, wn = id >> 8;
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const int c = wn * 64 + j * 32 + 4 * h + (t & 3) + 8 * (2 * s + (t >> 2));
        v[t] = (o < dsc.rows && c < dsc.depth) ? dsc.src[static_cast<int64_t>(o) * dsc.depth + c] : 0.f;
    }
    uint2 lo[3], hi[3];
    split4(make_float4(v[0], v[1], v[2], v[3]), lo[0], lo[1], lo[2]);
    split4(make_float4(v[4], v[5], v[6], v[7]), hi[0], hi[1], hi[2]);
    uint4* img = static_cast<uint4*>(dsc.image);
#pragma unroll
    for (int q = 0; q < 3; ++q)
        img[((((wn * 2 + j) * 2 + s) * 3 + q) * 2 + h) * 32 + o] = make_uint4(lo[q].x, lo[q].y, hi[q].x, hi[q].y);
    float4* f = reinterpret_cast<float4*>(img + kOutImagePlaneUnits) + 2 * id;
    f[0] = make_float4(v[0], v[1], v[2], v[3]);
    f[1] = make_float4(v[4], v[5], v[6], v[7]);
}

__global__ __launch_bounds__(kBlock) void bimage_kernel(BImageBatch batch) {
    const rslrl_bimage_desc_t& dsc = batch.d[blockIdx.y];
    if (dsc.layout == RSLRL_BIMAGE_LAYOUT_OUT) {
        out_image_thread(dsc, blockIdx.x * kBlock + threadIdx.x);
        return;
    }
    const int rows = dsc.rows, depth = dsc.depth;
    const float* __restrict__ src = dsc.src;
    const int nchunks = (depth + kKC - 1) / kKC;
    const int id = blockIdx.x * kBlock + threadIdx.x;
    if (dsc.layout == RSLRL_BIMAGE_LAYOUT_H3) {
        // depth <= 256: the 16 chunks x 2 halves of row n are the 32 lanes of a half wave, so the row's max
        // (-> its scale t_n) is a 32-lane shuffle reduction of the lanes' own 8 values
        if (id >= kBN * 32) return;  // whole half waves exit together
        const int n = id >> 5;
        const int c = (id >> 1) & 15;
        const int ph = id & 1;
        const int lh = ph ^ ((n >> 3) & 1);
        float v[8];
        float m = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 16 * c + 8 * lh + j;
            v[j] = (n < rows && k < depth) ? src[dsc.transposed ? static_cast<int64_t>(k) * rows + n
                                                                : static_cast<int64_t>(n) * depth + k]
                                           : 0.f;
            m = fmaxf(m, fabsf(v[j]));
        }
#pragma unroll
        for (int off = 16; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 32));
        const float t = h3_scale(m);
        if (c < nchunks) {
            uint2 lo[2], hi[2];
            split4_h(make_float4(v[0] * t, v[1] * t, v[2] * t, v[3] * t), lo[0], lo[1]);
            split4_h(make_float4(v[4] * t, v[5] * t, v[6] * t, v[7] * t), hi[0], hi[1]);
            uint4* base = static_cast<uint4*>(dsc.image) + static_cast<int64_t>(c) * (kH3ChunkB / 16) +
                          (n * kX6RowB + 16 * ph) / 16;
#pragma unroll
            for (int q = 0; q < 2; ++q) base[q * (kX6PlaneB / 16)] = make_uint4(lo[q].x, lo[q].y, hi[q].x, hi[q].y);
        }
        if (c == 0 && ph == 0)
            reinterpret_cast<float*>(static_cast<char*>(dsc.image) + h3_image_scales_offset(depth))[n] = 1.f / t;
        return;
    }
    if (id >= nchunks * kBN * 2) return;
    const int c = id / (kBN * 2);
    const int n = (id >> 1) % kBN;
    const int ph = id & 1;
    const int lh = ph ^ ((n >> 3) & 1);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = 16 * c + 8 * lh + j;
        v[j] = (n < rows && k < depth) ? src[dsc.transposed ? static_cast<int64_t>(k) * rows + n
                                                            : static_cast<int64_t>(n) * depth + k]
                                       : 0.f;
    }
    uint2 lo[3], hi[3];
    split4(make_float4(v[0], v[1], v[2], v[3]), lo[0], lo[1], lo[2]);
    split4(make_float4(v[4], v[5], v[6], v[7]), hi[0], hi[1], hi[2]);
    uint4* base = static_cast<uint4*>(dsc.image) + static_cast<int64_t>(c) * (kX6ChunkB / 16) +
                  (n * kX6RowB + 16 * ph) / 16;
#pragma unroll
    for (int q = 0; q < 3; ++q) base[q * (kX6PlaneB / 16)] = make_uint4(lo[q].x, lo[q].y, hi[q].x, hi[q].y);
}

// A chunk: BM rows x 16 k = BM / 128 float4 per thread (unit u = t + 512 i: row u >> 2, k-quad u & 3).
// FULL: the tile's rows exist and K % 16 == 0 -> no masks.
template <int BM, int NT = kThreads>
struct AStage {
    float4 v[BM * 4 / NT];
};

template <int BM, bool FULL, int NT = kThreads>
__device__ __forceinline__ AStage<BM, NT> load_a(const GemmParams& p, int64_t row0, int k0) {
    AStage<BM, NT> s;
#pragma unroll
    for (int i = 0; i < BM * 4 / NT; ++i) {
        const int u = threadIdx.x + NT * i;
        const int k = k0 + 4 * (u & 3);
        const int64_t row = row0 + (u >> 2);
        if constexpr (FULL) {
            s.v[i] = *reinterpret_cast<const float4*>(p.a + row * p.K + k);
        } else {
            const bool row_ok = row < p.M;
            s.v[i] = load4_masked(p.a + (row_ok ? row : row0) * p.K, row_ok && k < p.K, k);
        }
    }
    return s;
}

// PL planes (3: x6 bf16, 2: h3 fp16 of the operand scaled by sc, a power of two)
template <int BM, int PL, int NT = kThreads>
__device__ __forceinline__ void store_a_split(const AStage<BM, NT>& s, char* __restrict__ a_lds, float sc) {
    constexpr int plane = BM * kX6RowB;
#pragma unroll
    for (int i = 0; i < BM * 4 / NT; ++i) {
        const int u = threadIdx.x + NT * i;
        const int q = u & 3;
        const int r = u >> 2;
        const int off = swz(r, q >> 1) + 8 * (q & 1);
        uint2 w[PL];
        float4 v = s.v[i];
        if constexpr (PL == 2) v = make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc);
        Arith<PL>::split(v, w);
#pragma unroll
        for (int q2 = 0; q2 < PL; ++q2) *reinterpret_cast<uint2*>(a_lds + q2 * plane + off) = w[q2];
    }
}

// B chunk c of the image -> LDS: PL x 512 16-B units, thread t copies units t, t + 512, ...; the LDS
// destination of a wave's global_load_lds is (wave-uniform base) + 16 * lane.
template <int PL>
__device__ __forceinline__ void load_b_lds(const uint4* __restrict__ img, int c, char* b_lds) {
    const int t = threadIdx.x;
    const uint4* src = img + static_cast<int64_t>(c) * (PL * kX6PlaneB / 16);
#pragma unroll
    for (int i = 0; i < PL; ++i) {
        const int u = t + kThreads * i;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + u),
                                         (__attribute__((address_space(3))) void*)(b_lds + 16 * (u & ~63)), 16, 0, 0);
    }
}

template <typename F = bf16x8>
__device__ __forceinline__ F read_frag(const char* __restrict__ plane, int row, int h) {
    return __builtin_bit_cast(F, *reinterpret_cast<const uint4*>(plane + swz(row, h)));
}


#ifndef RSLRL_H3_DEPTH
#define RSLRL_H3_DEPTH 3
#endif
constexpr int kH3Depth = RSLRL_H3_DEPTH;  // A look-ahead (chunks) of the unrolled h3 main loop
#ifndef RSLRL_X6_DEPTH
#define RSLRL_X6_DEPTH 1
#endif
// the same loop on x6 operands (three planes: more fragment registers).  Measured at M = 393,216 (one process
// per build, scripts/x6_probe.py): depth 1 / 2 / 3 -> fwd 329 / 352 / 335 us, dgrad 359 / 375 / 375 us against
// 466-494 us for the generic one-chunk loop; depth 1 is the only one without spills at two workgroups per CU.
constexpr int kX6Depth = RSLRL_X6_DEPTH;
constexpr int kH3DeepDefault = (1 << RSLRL_LINEAR_FWD) | (1 << RSLRL_LINEAR_FWD_ELU) | (1 << RSLRL_LINEAR_DGRAD_ELU) |
                               (1 << RSLRL_LINEAR_FWD_OUT);
__device__ __forceinline__ void amax_commit(const GemmParams& p, float amx) {
    amax_publish<kThreads>(p.amax_out, p.amax_ws, amx);
}

// h3 main loop for a compile-time chunk count (K = 16 NCH, full tiles), fully unrolled so the A operand can be
// fetched D chunks ahead into registers (sa_[k % D] holds chunk k) -- the one-chunk look-ahead of the generic
// loop leaves each chunk waiting out an HBM load latency.  The B image chunk goes through registers as well
// (16-byte loads + ds_write_b128, one chunk ahead): with a global_load_lds DMA in flight the compiler waits
// vmcnt(0) before every LDS read (it cannot tell the DMA's buffer from the one being read), which would drain
// the A look-ahead every chunk.  Per chunk c: read every fragment of chunk c, write A(c+1) and B(c+1) into the
// other buffer, fetch A(c+1+D) and B(c+2), MFMAs, barrier (LDS writes only: lgkmcnt(0)).
template <int PL, int NT = kThreads>
struct BStage {
    uint4 u[PL * kThreads / NT];
};

template <int PL, int NT = kThreads>
__device__ __forceinline__ BStage<PL, NT> load_b_regs(const uint4* __restrict__ img, int c) {
    const uint4* src = img + static_cast<int64_t>(c) * (PL * kX6PlaneB / 16);
    BStage<PL, NT> b;
#pragma unroll
    for (int i = 0; i < PL * kThreads / NT; ++i) b.u[i] = src[threadIdx.x + NT * i];
    return b;
}

template <int PL, int NT = kThreads>
__device__ __forceinline__ void store_b_regs(BStage<PL, NT>& b, char* b_lds) {
#pragma unroll
    for (int i = 0; i < PL * kThreads / NT; ++i) {
        asm volatile("" : "+v"(b.u[i].x), "+v"(b.u[i].y), "+v"(b.u[i].z), "+v"(b.u[i].w));
        *reinterpret_cast<uint4*>(b_lds + 16 * (threadIdx.x + NT * i)) = b.u[i];
    }
}

#ifndef RSLRL_B_FIRST
#define RSLRL_B_FIRST 1
#endif
constexpr bool kBFirst = RSLRL_B_FIRST != 0;  // deep_pipeline's issue order of the look-ahead loads (A/B build knob)

// The pipeline alone, for any fragment schedule: compute(a_lds, b_lds) reads one chunk's fragments from the
// LDS buffer and issues its MFMAs.
struct NoHook {
    __device__ void operator()(char*) const {}
};

// last_hook(free_buffer): called before the last chunk's compute with the LDS buffer no chunk reads any more
// (a compile-time object: a DMA into it does not make the compiler wait for it before the other buffer's reads)
template <int BM, int PL, int NCH, int D, typename Compute, typename Hook = NoHook, int NT = kThreads>
__device__ __forceinline__ void deep_pipeline(const GemmParams& p, int64_t row0, const uint4* __restrict__ bimg,
                                              char* (&lds)[2], float sa, Compute&& compute, Hook&& last_hook = Hook{}) {
    constexpr int planeA = BM * kX6RowB;
    AStage<BM, NT> sa_[D];
    BStage<PL, NT> sb;
    {
        BStage<PL, NT> b0 = load_b_regs<PL, NT>(bimg, 0);
        store_b_regs<PL, NT>(b0, lds[0] + PL * planeA);
    }
    store_a_split<BM, PL, NT>(load_a<BM, true, NT>(p, row0, 0), lds[0], sa);
#pragma unroll
    for (int d = 1; d <= D; ++d)
        if (d < NCH) sa_[d % D] = load_a<BM, true, NT>(p, row0, d * kKC);
    if (NCH > 1) sb = load_b_regs<PL, NT>(bimg, 1);
    __syncthreads();
    constexpr bool kHook = !std::is_same_v<std::decay_t<Hook>, NoHook>;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        if (c + 1 == NCH) last_hook(lds[(c + 1) & 1]);
        compute(lds[c & 1], lds[c & 1] + PL * planeA);
        if (c + 1 < NCH) {  // buffer (c+1)&1 was last read in chunk c-1; every wave passed the barrier after it
            // pin the use of the prefetched registers here: otherwise the scheduler hoists the scaling
            // multiply right behind the load and the wave waits out the look-ahead right away
#pragma unroll
            for (int u = 0; u < BM * 4 / NT; ++u) {
                float4& v = sa_[(c + 1) % D].v[u];
                asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
            }
            store_a_split<BM, PL, NT>(sa_[(c + 1) % D], lds[(c + 1) & 1], sa);
            store_b_regs<PL, NT>(sb, lds[(c + 1) & 1] + PL * planeA);
            if constexpr (kBFirst) {
                // B (one chunk ahead) issued before A (D chunks ahead): vmcnt retires in issue order, so the next
                // chunk's wait for this B leaves the younger A loads in flight.  Issued after A, that wait was a
                // vmcnt(0) every chunk -- the A look-ahead drained down to one chunk (the .s of the w4 kernel).
                if (c + 2 < NCH) sb = load_b_regs<PL, NT>(bimg, c + 2);
                if (c + 1 + D < NCH) sa_[(c + 1) % D] = load_a<BM, true, NT>(p, row0, (c + 1 + D) * kKC);
            } else {
                if (c + 1 + D < NCH) sa_[(c + 1) % D] = load_a<BM, true, NT>(p, row0, (c + 1 + D) * kKC);
                if (c + 2 < NCH) sb = load_b_regs<PL, NT>(bimg, c + 2);
            }
        }
        // only LDS writes to retire (lgkmcnt); __syncthreads' release fence would also wait vmcnt(0) and drain
        // the look-ahead every chunk
        if (c + 1 < NCH) {
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        } else {
            // a hook's LDS DMA may be read by other waves after the barrier, which does not wait for loads
            if constexpr (kHook) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();  // the epilogue may reuse the LDS
        }
    }
}

// Input-gradient epilogue: H block (i = 0, j = 0) of each wave (32 x 32 fp32, row-major, kH0StageBytes at wave *
// kH0StageBytes) DMA'd into the free LDS buffer during the last chunk, so the epilogue's first ELU' does not wait
// out an HBM load (the later blocks are prefetched one ahead in registers).  Full tiles only (the caller checks).
__device__ __forceinline__ void stage_h_block0(const GemmParams& p, int64_t row0, int wm, int wn, char* buf) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const float* hb = p.h + (row0 + wm * 64) * kBN + wn * 64;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int r = 8 * k + (lane >> 3), c4 = lane & 7;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(hb + r * kBN + 4 * c4),
                                         (__attribute__((address_space(3))) void*)(buf + wave * kH0StageBytes + k * 1024),
                                         16, 0, 0);
    }
}

template <int EPI, int BM, int PL, int NCH, int D, typename Frag>
__device__ __forceinline__ void h3_deep_loop(const GemmParams& p, int64_t row0, const uint4* __restrict__ bimg,
                                             char* (&lds)[2], f32x16 (&acc)[BM / 64][2], float sa, int wm,
                                             int wn, int l32, int h, bool stage_h0 = false) {
    constexpr int I = BM / 64;
    constexpr int planeA = BM * kX6RowB;
    auto hook = [&](char* free_buf) {
        // (the forward's biases staged the same way measured 2-4 % slower: kept as L2 loads)
        if constexpr (EPI == kEpiEluGrad && PL == 3)
            if (stage_h0) stage_h_block0(p, row0, wm, wn, free_buf);
    };
    deep_pipeline<BM, PL, NCH, D>(p, row0, bimg, lds, sa, [&](const char* a_lds, const char* b_lds) {
        Frag bf[2][PL];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < PL; ++q) bf[j][q] = read_frag<Frag>(b_lds + q * kX6PlaneB, wn * 64 + j * 32 + l32, h);
#pragma unroll
        for (int i = 0; i < I; ++i) {
            Frag af[PL];
#pragma unroll
            for (int q = 0; q < PL; ++q) af[q] = read_frag<Frag>(a_lds + q * planeA, wm * (BM / 2) + i * 32 + l32, h);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if constexpr (EPI == kEpiBiasEluOut)
                    acc[i][j] = Arith<PL>::mfma(bf[j], af, acc[i][j]);
                else
                    acc[i][j] = Arith<PL>::mfma(af, bf[j], acc[i][j]);
            }
        }
    }, hook);
}

// 128 rows x 256 columns per workgroup: waves 2 (M) x 4 (N) of 64 x 64 (2 x 2 MFMA tiles); MINW = 4:
// two workgroups per CU (<= 128 VGPRs), 2: one (the register-hungrier short-K dgrad epilogues).
// NR: rows of the fused weight gradient (kEpiEluGradWgrad: Nred rounded up to 4); kEpiBiasEluOut: 1 = VALU output
// layer (<= 4 outputs), 4 = MFMA output layer (separate code: one register allocation for both spilled).
// PL: operand planes (3: x6 bf16 on a layout-0 image; 2: h3 fp16 on a layout-2 image, A scaled from *p.a_amax).
// KCH = 3: a kernel for K = 48 only (the first layer), whose look-ahead loop is its only main loop (one body with
// both loop instances ran the K = 256 forward ~2 % slower)
// bytes of each of the two LDS buffers of the x6 GEMM body
template <int EPI, int PL>
constexpr int x6_buf_bytes() {
    // the fused output layer's epilogue needs 40 KiB per buffer (h stage in one, reduction tiles in the other)
    return EPI == kEpiBiasEluOut ? 40960 : (PL * kBM * kX6RowB + PL * kX6PlaneB);
}

// ---- The actor head: last hidden layer + output layer + PPO loss + output-layer backward (one 128-row tile) ----------
// Called after the main loop of a full x6 C^T tile (acc: lane (l32, h) holds row l32 of block i, columns (r & 3) +
// 8 (r >> 2) + 4 h of block j).  Phases (LDS: buffer 0 = b0, buffer 1 = b1, 40 KiB each):
//  1. H = ELU(acc + b) in place; the output layer's partial tiles (x6 MFMA, the fused forward's epilogue: the same
//     bits) -> red [wm][wn][i][12][32] (b0 [0, 24K)).
//  2. mu of row t >> 2, actions 3 (t & 3) .. +2 (the wn partials added in the fused forward's order), then the loss of
//     the row on its quad of lanes: ppo_loss_quad_kernel's arithmetic (shared std; same d mu bits) -> d mu tile
//     [128][16] (b1 [32K, 40K), columns 12..15 zero) and per-wave fp64 loss partials (b0 [32K, 33K)).  The i = 1
//     half of H waits in LDS meanwhile (32 registers fewer through the loss).
//  3. per half i (1, then 0): H staged as [32 rows][256] per wave row wm (b0 / b1 [0, 32K), float4 quads XOR-swizzled
//     in their 8-quad group by row & 7); dW[o][c] += d mu[r][o] H[r][c] over the half's 64 rows, thread (c, o half)
//     with 6 accumulators; then dZ = (d mu W_out) * ELU'(H): x6 MFMA of the W_out^T image (A) and the split d mu
//     rows (B) gives the C^T layout of acc, ELU' from H, and the result leaves in place through the stage as
//     whole-line stores.
//  4. per-tile [dW | db] partials; loss partials folded over the grid (fold_grid_partials) -> stats, d sigma.
__device__ __forceinline__ int act_stage_idx(int l, int quad) { return l * kBN + 4 * (quad ^ (l & 7)); }

__device__ __forceinline__ void actor_head_epilogue(const GemmParams& p, const ActorParams& ap, f32x16 (&acc)[2][2],
                                                    char* lds0, char* lds1, const float* xsb, int wm, int wn, int lane,
                                                    int wave, int64_t row0) {
    const int l32 = lane & 31, h = lane >> 5;
    const int t = threadIdx.x;
    float* red = reinterpret_cast<float*>(lds0);
    float* dmu = reinterpret_cast<float*>(lds1 + 32768);
    double* wstat = reinterpret_cast<double*>(lds0 + 32768);  // [8 waves][kActCols]
    double* folded = wstat + 8 * kActCols;                    // [kActCols]
    int* flag = reinterpret_cast<int*>(folded + kActCols);
    float* const stg = reinterpret_cast<float*>(wm ? lds1 : lds0);  // this wave row's half-tile H stage
    // ---- 1. H and the output layer's partials
    const uint4* oimg = p.oimg + wn * (2 * 2 * 3 * 64);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        f32x16 oacc = f32x16{};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int cb = wn * 64 + j * 32 + 4 * h;
            float v[16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 b4 = *reinterpret_cast<const float4*>(xsb + cb + 8 * g);
                float tt[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                tt[0] += b4.x;
                tt[1] += b4.y;
                tt[2] += b4.z;
                tt[3] += b4.w;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float n = elu_neg(fminf(tt[e], 0.f));
                    v[4 * g + e] = tt[e] > 0.f ? tt[e] : n;
                    acc[i][j][4 * g + e] = v[4 * g + e];
                }
            }
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                bf16x8 vb[3], wa[3];
                uint2 lo[3], hi[3];
                split4(make_float4(v[8 * s2], v[8 * s2 + 1], v[8 * s2 + 2], v[8 * s2 + 3]), lo[0], lo[1], lo[2]);
                split4(make_float4(v[8 * s2 + 4], v[8 * s2 + 5], v[8 * s2 + 6], v[8 * s2 + 7]), hi[0], hi[1], hi[2]);
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    vb[q] = __builtin_bit_cast(bf16x8, make_uint4(lo[q].x, lo[q].y, hi[q].x, hi[q].y));
                    wa[q] = __builtin_bit_cast(bf16x8, oimg[((j * 2 + s2) * 3 + q) * 64 + lane]);
                }
                oacc = mfma_x6(wa, vb, oacc);
                __builtin_amdgcn_sched_barrier(0);  // one k step at a time: its planes die before the next split
            }
        }
        float* rd = red + ((wm * 4 + wn) * 2 + i) * (kActA * 32);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int o = (r & 3) + 8 * (r >> 2) + 4 * h;
            if (o < kActA) rd[o * 32 + l32] = oacc[r];
        }
    }
    // ---- 2. mu and the loss of row rl on lanes q = 0..3 (actions a0 .. a0 + 2)
    const int rl = t >> 2, q = t & 3, a0 = 3 * q;
    const int64_t row = row0 + rl;
    const float* xact = xsb + kBN;  // [obias | sigma | old_sigma of sample 0] x 12 (prologue)
    __syncthreads();  // red complete
    float mu[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float* b = red + ((rl >> 6) * 4 * 2 + ((rl & 63) >> 5)) * (kActA * 32) + (a0 + k) * 32 + (rl & 31);
        const float sum = ((b[0] + b[2 * kActA * 32]) + b[4 * kActA * 32]) + b[6 * kActA * 32];
        mu[k] = sum + xact[a0 + k];
        p.y[row * kActA + a0 + k] = mu[k];
    }
    float x[3], om[3], os[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        x[k] = ap.actions[row * kActA + a0 + k];
        om[k] = ap.old_mu[row * kActA + a0 + k];
        os[k] = ap.old_sigma[row * kActA + a0 + k];
    }
    const float old_logp = ap.old_logp[row], adv = ap.adv[row], V = ap.values[row], tv = ap.target_values[row],
                R = ap.returns[row];
    __syncthreads();  // red read: buffer 0 takes the H stage
    auto stage_half = [&](int i) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 hv = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                *reinterpret_cast<f32x4*>(stg + act_stage_idx(l32, wn * 16 + j * 8 + 2 * g + h)) = hv;
            }
    };
    stage_half(1);
    // per-action constants (ppo_loss_quad_kernel, SHARED = true)
    float c_s[3], c_ls[3], c_inv_den[3], c_inv_s[3], c_inv_s3[3], c_os[3], c_t1[3], c_D[3], c_rD[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float s = xact[kActA + a0 + k], os0 = xact[2 * kActA + a0 + k];
        const float inv_s = 1.0f / s;
        c_s[k] = s;
        c_ls[k] = logf(s);
        c_inv_den[k] = 1.0f / __fmul_rn(2.0f, __fmul_rn(s, s));
        c_inv_s[k] = inv_s;
        c_inv_s3[k] = inv_s * inv_s * inv_s;
        const float D = __fmul_rn(2.0f, __fmul_rn(s, s));
        const bool d_ok = D >= 0x1p-60f && D <= 0x1p60f;
        c_os[k] = (d_ok && ap.kl_fast) ? os0 : __builtin_nanf("");
        c_t1[k] = logf(__fadd_rn(__fdiv_rn(s, os0), 1.0e-5f));
        c_D[k] = D;
        c_rD[k] = __fdiv_rn(1.0f, D);
    }
    float ent_shared = 0.0f;  // sum over the 12 actions in order (the quad's lanes hold 3 each)
#pragma unroll
    for (int a = 0; a < kActA; ++a)
        ent_shared = __fadd_rn(ent_shared, __fadd_rn(kEntC, __shfl(c_ls[a % 3], (lane & ~3) + a / 3, kWave)));
    float d[3], lpart = 0.0f, klpart = 0.0f;
    bool kl_slow = false;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float dd = x[k] - mu[k];
        d[k] = dd;
        lpart += (-(dd * dd) * c_inv_den[k] - c_ls[k]) - kLogSqrt2Pi;
        const float osk = os[k];
        const float dm = __fsub_rn(om[k], mu[k]);
        const float n = __fadd_rn(__fmul_rn(osk, osk), __fmul_rn(dm, dm));
        const float t1 = c_t1[k];
        const float q0 = __fmul_rn(n, c_rD[k]);
        const float t2 = __builtin_fmaf(__builtin_fmaf(-q0, c_D[k], n), c_rD[k], q0);
        kl_slow |= !(osk == c_os[k] && n >= 0x1p-60f && n <= 0x1p60f);
        klpart = __fadd_rn(klpart, __fsub_rn(__fadd_rn(t1, t2), 0.5f));
    }
    if (ap.compute_kl && kl_slow) {  // the reference's exact expression for every element of this lane (rare)
        klpart = 0.0f;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float s = c_s[k], osk = os[k];
            const float dm = __fsub_rn(om[k], mu[k]);
            const float t1 = logf(__fadd_rn(__fdiv_rn(s, osk), 1.0e-5f));
            const float t2 = __fdiv_rn(__fadd_rn(__fmul_rn(osk, osk), __fmul_rn(dm, dm)), __fmul_rn(2.0f, __fmul_rn(s, s)));
            klpart = __fadd_rn(klpart, __fsub_rn(__fadd_rn(t1, t2), 0.5f));
        }
    }
    const float logp = quad_sum(lpart);
    // surrogate (ppo.py:297-302)
    const float ratio = expf(logp - old_logp);
    const float nadv = -adv;
    const float surr = nadv * ratio;
    const float rc = fminf(fmaxf(ratio, ap.ratio_lo), ap.ratio_hi);
    const float surr_c = nadv * rc;
    float g_s, g_sc;
    max_grads(surr, surr_c, ap.g_surr, g_s, g_sc);
    const bool in_clip = (ratio >= ap.ratio_lo) && (ratio <= ap.ratio_hi);
    const float g_ratio = g_s * nadv + (in_clip ? g_sc * nadv : 0.0f);
    const float gj = g_ratio * ratio;
    // value loss term (ppo.py:305-313; its gradient is the critic head's, rslrl_value_head_fwd_bwd)
    float vterm;
    if (ap.clipped_value) {
        const float dv = V - tv;
        const float vc = tv + fminf(fmaxf(dv, -ap.clip), ap.clip);
        const float e1 = V - R;
        const float e2 = vc - R;
        vterm = fmaxf(e1 * e1, e2 * e2);
    } else {
        const float e = R - V;
        vterm = e * e;
    }
    const float g2 = 2.0f * gj;
    float gsg[3];
    {
        float gm[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float dd = d[k];
            gm[k] = g2 * dd * c_inv_den[k];
            gsg[k] = gj * (dd * dd * c_inv_s3[k] - c_inv_s[k]) + ap.g_ent * c_inv_s[k];
            dmu[rl * 16 + a0 + k] = gm[k];
            if (ap.grad_mu) ap.grad_mu[row * kActA + a0 + k] = gm[k];
        }
        if (q == 3) *reinterpret_cast<float4*>(dmu + rl * 16 + kActA) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    {
        const double s_surr = wave_sum(static_cast<double>(q == 0 ? fmaxf(surr, surr_c) : 0.0f));
        const double s_val = wave_sum(static_cast<double>(q == 0 ? vterm : 0.0f));
        const double s_ent = wave_sum(static_cast<double>(q == 0 ? ent_shared : 0.0f));
        const double s_kl = wave_sum(static_cast<double>(ap.compute_kl ? klpart : 0.0f));
        if (lane == 0) {
            wstat[wave * kActCols + 0] = s_surr;
            wstat[wave * kActCols + 1] = s_val;
            wstat[wave * kActCols + 2] = s_ent;
            wstat[wave * kActCols + 3] = s_kl;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            double v = static_cast<double>(gsg[k]);
#pragma unroll
            for (int off = 4; off < kWave; off <<= 1) v += __shfl_xor(v, off, kWave);
            if (lane < 4) wstat[wave * kActCols + 4 + 3 * lane + k] = v;
        }
    }
    __syncthreads();  // the d mu tile and the i = 1 stage complete
    // ---- 3. output-layer backward, half i = 1 (staged) then i = 0 (registers)
    float* wp = ap.wpart + static_cast<int64_t>(blockIdx.x) * kActTileFloats;
    if (wave == 0) {  // db = column sums of d mu: lane (o, quarter) adds its 32 rows in order, then the quarters
        const int o = lane & 15, part = lane >> 4;
        float s = 0.f;
#pragma unroll 8
        for (int r = 32 * part; r < 32 * part + 32; ++r) s += dmu[r * 16 + o];
        s += __shfl_xor(s, 16, kWave);
        s += __shfl_xor(s, 32, kWave);
        if (lane < kActA) wp[kActA * kBN + lane] = s;
    }
    const int c = t & (kBN - 1), rh = t >> 8;  // dW column c over the 32 rows of buffer rh (wave-uniform)
    float wacc[kActA];
#pragma unroll
    for (int o = 0; o < kActA; ++o) wacc[o] = 0.f;
    auto dw_pass = [&](int i) {  // 3 broadcast d mu reads + 1 H read per 12 FMAs
        const float* sb = reinterpret_cast<const float*>(rh ? lds1 : lds0);
#pragma unroll 4
        for (int l = 0; l < 32; ++l) {
            const float hv = sb[act_stage_idx(l, c >> 2) + (c & 3)];
            const float4* dr = reinterpret_cast<const float4*>(dmu + (rh * 64 + i * 32 + l) * 16);
            const float4 d0 = dr[0], d1 = dr[1], d2 = dr[2];
            const float dd[kActA] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w, d2.x, d2.y, d2.z, d2.w};
#pragma unroll
            for (int o = 0; o < kActA; ++o) wacc[o] = fmaf(dd[o], hv, wacc[o]);
        }
    };
    bf16x8 wa[2][3];
    auto load_wa = [&]() {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int qq = 0; qq < 3; ++qq)
                wa[j][qq] = read_frag<bf16x8>(reinterpret_cast<const char*>(ap.w_t_img) + qq * kX6PlaneB,
                                              wn * 64 + j * 32 + l32, h);
    };
    auto dmu_frag = [&](int i, bf16x8 (&vb)[3]) {
        const float* r = dmu + (wm * 64 + i * 32 + l32) * 16 + 8 * h;
        const float4 v0 = *reinterpret_cast<const float4*>(r);
        const float4 v1 = *reinterpret_cast<const float4*>(r + 4);
        uint2 lo[3], hi[3];
        split4(v0, lo[0], lo[1], lo[2]);
        split4(v1, hi[0], hi[1], hi[2]);
#pragma unroll
        for (int qq = 0; qq < 3; ++qq) vb[qq] = __builtin_bit_cast(bf16x8, make_uint4(lo[qq].x, lo[qq].y, hi[qq].x, hi[qq].y));
    };
    // dZ of block (i, j) from H values hv (C^T layout): in place over the wave's stage positions, then whole lines out
    auto dz_block = [&](int i, int j, const bf16x8 (&vb)[3], const f32x16& hv) {
        const f32x16 dacc = mfma_x6(wa[j], vb, f32x16{});
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            f32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float z = dacc[4 * g + e], hh = hv[4 * g + e];
                o[e] = hh > 0.f ? z : z * (hh + 1.f);  // ELU'(x) = 1 if h > 0 else h + 1
            }
            *reinterpret_cast<f32x4*>(stg + act_stage_idx(l32, wn * 16 + j * 8 + 2 * g + h)) = o;
        }
        __builtin_amdgcn_wave_barrier();  // one wave's LDS accesses execute in order
        float* ct = p.c + (row0 + wm * 64 + i * 32) * kBN + (wn * 64 + j * 32);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int sr = 8 * k + (lane >> 3), cq = lane & 7;
            const f32x4 v = *reinterpret_cast<const f32x4*>(stg + act_stage_idx(sr, wn * 16 + j * 8 + cq));
            f32x4* dst = reinterpret_cast<f32x4*>(ct + static_cast<uint32_t>(sr * kBN + 4 * cq));
            if (p.nt) __builtin_nontemporal_store(v, dst);
            else *dst = v;
        }
        __builtin_amdgcn_wave_barrier();
    };
    load_wa();
    dw_pass(1);
    __syncthreads();  // every wave's reads of the i = 1 stage done
    {
        bf16x8 vb[3];
        dmu_frag(1, vb);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            f32x16 hv;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 h4 = *reinterpret_cast<const f32x4*>(stg + act_stage_idx(l32, wn * 16 + j * 8 + 2 * g + h));
#pragma unroll
                for (int e = 0; e < 4; ++e) hv[4 * g + e] = h4[e];
            }
            dz_block(1, j, vb, hv);
        }
    }
    stage_half(0);
    __syncthreads();  // the i = 0 stage complete
    dw_pass(0);
    __syncthreads();  // every wave's reads of the i = 0 stage done
    {
        bf16x8 vb[3];
        dmu_frag(0, vb);
#pragma unroll
        for (int j = 0; j < 2; ++j) dz_block(0, j, vb, acc[0][j]);
    }
    // ---- 4. per-tile partials: dW rows (coalesced over c), then the loss terms over the grid
    __syncthreads();  // the stages are no longer read: the buffer-1 half of dW goes through LDS
    float* dwx = reinterpret_cast<float*>(lds0);  // [12][256]
    if (rh == 1)
#pragma unroll
        for (int o = 0; o < kActA; ++o) dwx[o * kBN + c] = wacc[o];
    __syncthreads();
    if (rh == 0)
#pragma unroll
        for (int o = 0; o < kActA; ++o) wp[o * kBN + c] = wacc[o] + dwx[o * kBN + c];
    double v = 0.0;
    if (t < kActCols) {
        v = wstat[t];
#pragma unroll
        for (int w = 1; w < 8; ++w) v += wstat[w * kActCols + t];
    }
    // groups of 64 tiles up to 4096 tiles (C3's 3072), of 128 above (C4's 131,072 envs on one GPU: 6144 tiles)
    const bool folded_ok = gridDim.x > kFoldGroup * kFoldGroup
                               ? fold_grid_partials<kActCols, 2 * kFoldGroup>(ap.partials, ap.tickets,
                                                                               static_cast<int>(gridDim.x), kActCols, v,
                                                                               folded, flag)
                               : fold_grid_partials<kActCols>(ap.partials, ap.tickets, static_cast<int>(gridDim.x),
                                                              kActCols, v, folded, flag);
    if (folded_ok) {
        if (t == 0) {
            const double Bd = static_cast<double>(p.M);
            float* stats = ap.stats;
            stats[1] = static_cast<float>(folded[0] / Bd);
            stats[2] = static_cast<float>(folded[1] / Bd);
            stats[3] = static_cast<float>(folded[2] / Bd);
            stats[4] = static_cast<float>(folded[3] / Bd);
            stats[0] = __fsub_rn(__fadd_rn(stats[1], __fmul_rn(ap.value_loss_coef, stats[2])),
                                 __fmul_rn(ap.entropy_coef, stats[3]));
            stats[5] = 0.0f;
            stats[6] = 0.0f;
            stats[7] = 0.0f;
            __hip_atomic_store(ap.tickets, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm (stream-ordered)
        }
        if (t < kActA) ap.grad_sigma[t] = static_cast<float>(folded[4 + t]);
    }
}

// lds_b0 / lds_b1: the kernel's two LDS buffers (x6_buf_bytes<EPI, PL>() each).  Two LDS objects, not one [2][bytes]
// array: the waitcnt pass can then tell a DMA into one buffer from reads of the other (distinct alias scopes) where
// the buffer index is a compile-time constant.  Declared by the kernel so that two bodies in one kernel (the
// output-layer pair) share them.
// HEAD (kEpiBiasEluOut, NR 1, full tiles): the value head's backward fused behind it (mlp_gemm_x6_value_head_kernel)
template <int EPI, bool FULL, int NR, int PL, bool STAGE = true, int KCH = 0, int HEAD = 0>
__device__ __forceinline__ void mlp_gemm_x6_body(GemmParams p, const uint4* __restrict__ bimg, char* lds_b0,
                                                 char* lds_b1, const ActorParams* ap = nullptr) {
    static_assert(PL == 3 || EPI != kEpiEluGradWgrad, "the fused output-layer backward is x6 only");
    using Frag = typename Arith<PL>::frag;
    constexpr int BM = kBM;
    constexpr int I = BM / 64;
    constexpr int planeA = BM * kX6RowB;
    constexpr int bufBytes = x6_buf_bytes<EPI, PL>();
    static_assert(bufBytes >= PL * planeA + PL * kX6PlaneB, "LDS buffer");
    char* lds[2];
    lds[0] = lds_b0;
    lds[1] = lds_b1;
    // kEpiBiasEluOut: the bias and (1 output on the VALU: the value head) the fp32 output weights live in the 4 KiB of buffer 0
    // that neither the main loop nor the epilogue uses, so the epilogue's dependent chain reads them from LDS
    // instead of waiting on L2 loads (xs: [256] bias, then [32 (wn, j, s, h)][kXsOut][8] weights)
    // past the main loop's operands and past the epilogue's H stage / reduction tiles (8 waves x 4 KiB)
    constexpr int kXsOff = PL * planeA + PL * kX6PlaneB > 8 * 4096 ? PL * planeA + PL * kX6PlaneB : 8 * 4096;
    constexpr int kXsOut = 1;  // the value head
    constexpr int kVhWOff = kBN + kOutImageThreads / 32 * kXsOut * 8;  // HEAD: floats from xs to the value weights
    if constexpr (EPI == kEpiBiasEluOut) {
        static_assert(kXsOff + 4 * (kBN + kOutImageThreads / 32 * kXsOut * 8) <= bufBytes, "LDS side area");
        float* xs = reinterpret_cast<float*>(lds_b0 + kXsOff);
        const int t = threadIdx.x;
        if (t < kBN / 4)
            reinterpret_cast<float4*>(xs)[t] =
                4 * t < p.N ? *reinterpret_cast<const float4*>(p.bias + 4 * t) : make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (NR == 1) {
            // the fp32 section holds kOutImageThreads / 32 = 32 (wn, j, s, h) combinations x 32 outputs
            if (p.nout <= kXsOut && t >= 64 && t < 64 + kOutImageThreads / 32 * kXsOut) {
                const int e = t - 64, combo = e / kXsOut, o = e % kXsOut;
                const float4* src = reinterpret_cast<const float4*>(p.oimg + kOutImagePlaneUnits) + 2 * (combo * 32 + o);
                float4* dst = reinterpret_cast<float4*>(xs + kBN) + 2 * e;
                const bool ok = o < p.nout;
                dst[0] = ok ? src[0] : make_float4(0.f, 0.f, 0.f, 0.f);
                dst[1] = ok ? src[1] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        if constexpr (HEAD == 2) {
            // the actor head: [output bias | shared std | old std of the mini-batch's sample 0] per action after the bias
            // (actor_head_epilogue's mu and per-action loss constants)
            if (t >= 64 && t < 64 + kActA) {
                const int a = t - 64;
                xs[kBN + a] = p.obias[a];
                xs[kBN + kActA + a] = ap->sigma[a];
                xs[kBN + 2 * kActA + a] = ap->old_sigma[a];
            }
        }
        if constexpr (HEAD == 1) {
            // after the side area: the value weight row in column order [N], then the tile's target values and returns
            // [BM] each, DMA'd now (no registers held through the main loop; its final barrier drains them) -- the
            // epilogue replaces the targets by dV
            static_assert(kXsOff + 4 * (kVhWOff + kBN + 2 * BM) <= bufBytes, "LDS side area (value head)");
            if (t >= 128 && t < 128 + kBN / 4)
                reinterpret_cast<float4*>(xs + kVhWOff)[t - 128] = *reinterpret_cast<const float4*>(p.vh_w + 4 * (t - 128));
            if (t < BM) {
                const int w = t >> 6;  // waves 0 and 1: 64 rows each, lane l -> row 64 w + l
                const int64_t r = static_cast<int64_t>(blockIdx.x) * BM + t;
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(p.vh_tv + r),
                    (__attribute__((address_space(3))) void*)(xs + kVhWOff + kBN + 64 * w), 4, 0, 0);
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(p.vh_ret + r),
                    (__attribute__((address_space(3))) void*)(xs + kVhWOff + kBN + BM + 64 * w), 4, 0, 0);
            }
        }
    }
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: SGPR arithmetic
    const int wm = wave >> 2;  // rows wm * BM / 2
    const int wn = wave & 3;   // cols wn * 64
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * BM;
#ifdef RSLRL_STAMPS  // diagnostic build only (scripts/experiments/gemm_timeline.hip)
    uint64_t st0 = __builtin_amdgcn_s_memrealtime();
    uint64_t ct0 = __builtin_amdgcn_s_memtime();
#endif

    f32x16 acc[I][2];
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

    const float sa = PL == 2 ? h3_scale(*p.a_amax) : 1.f;
    bool deep = false;
    // x6 input gradient on a full tile: each wave's first H block goes to the free LDS buffer during the last
    // chunk (stage_h_block0); lds[0] is that buffer for the 16-chunk loop (the last chunk reads lds[1])
    // (the same condition as the deep loop below: FULL, K = 256, p.deep -- the DMA is issued from that loop)
    // STAGE = false (the pair kernel): a spill at its register budget cost more than the staged loads save
    const bool stage_h0 = STAGE && FULL && EPI == kEpiEluGrad && PL == 3 && p.h != nullptr && (row0 + BM <= p.M) &&
                          p.N == kBN && p.K == 16 * kKC && p.deep;
    static_assert(EPI != kEpiEluGrad || PL != 3 || 8 * kH0StageBytes <= bufBytes, "H block stage");
    if constexpr (FULL && KCH == 3) {
        // the first layer (K = 48: three chunks) on the look-ahead loop: the generic loop's per-chunk __syncthreads
        // drains every load, which a three-chunk tile pays in full (the host launches KCH = 3 for K = 48 only)
        h3_deep_loop<EPI, BM, PL, 3, 1, Frag>(p, row0, bimg, lds, acc, sa, wm, wn, l32, h);
        deep = true;
    } else if constexpr (FULL) {
        if (p.K == 16 * kKC && p.deep) {
            h3_deep_loop<EPI, BM, PL, 16, PL == 2 ? kH3Depth : kX6Depth, Frag>(p, row0, bimg, lds, acc, sa, wm, wn, l32, h,
                                                                            stage_h0);
            deep = true;
        }
    }
    // Pipeline: B of chunk c+1 is copied (global_load_lds) and A of chunk c+1 fetched into registers at
    // the start of chunk c; A is split into the other LDS buffer at its end.
    const int nchunks = deep ? 0 : (p.K + kKC - 1) / kKC;
    if (!deep) {
    load_b_lds<PL>(bimg, 0, lds[0] + PL * planeA);
    store_a_split<BM, PL>(load_a<BM, FULL>(p, row0, 0), lds[0], sa);
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
        const int buf = c & 1;
        const bool more = c + 1 < nchunks;
        const char* a_lds = lds[buf];
        const char* b_lds = lds[buf] + PL * planeA;
        AStage<BM> an;
        Frag bf[2][PL];
        if constexpr (PL == 2) {
            // h3: every fragment of the chunk is read before the next chunk's loads issue -- the compiler
            // cannot tell the global_load_lds destination (the other buffer) from this one and waits
            // vmcnt(0) before any LDS read that follows it, which would expose the loads' full latency
            Frag af[I][PL];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < PL; ++q)
                    bf[j][q] = read_frag<Frag>(b_lds + q * kX6PlaneB, wn * 64 + j * 32 + l32, h);
#pragma unroll
            for (int i = 0; i < I; ++i)
#pragma unroll
                for (int q = 0; q < PL; ++q)
                    af[i][q] = read_frag<Frag>(a_lds + q * planeA, wm * (BM / 2) + i * 32 + l32, h);
            if (more) {  // the other buffer was last read in chunk c-1, and every wave passed the barrier after it
                load_b_lds<PL>(bimg, c + 1, lds[buf ^ 1] + PL * planeA);
                an = load_a<BM, FULL>(p, row0, (c + 1) * kKC);
            }
#pragma unroll
            for (int i = 0; i < I; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if constexpr (EPI == kEpiBiasEluOut)  // C^T tile: the weight fragment is the MFMA's A operand
                        acc[i][j] = Arith<PL>::mfma(bf[j], af[i], acc[i][j]);
                    else
                        acc[i][j] = Arith<PL>::mfma(af[i], bf[j], acc[i][j]);
                }
        } else {
            if (more) {  // the other buffer was last read in chunk c-1, and every wave passed the barrier after it
                load_b_lds<PL>(bimg, c + 1, lds[buf ^ 1] + PL * planeA);
                an = load_a<BM, FULL>(p, row0, (c + 1) * kKC);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < PL; ++q)
                    bf[j][q] = read_frag<Frag>(b_lds + q * kX6PlaneB, wn * 64 + j * 32 + l32, h);
#pragma unroll
            for (int i = 0; i < I; ++i) {
                Frag af[PL];
#pragma unroll
                for (int q = 0; q < PL; ++q)
                    af[q] = read_frag<Frag>(a_lds + q * planeA, wm * (BM / 2) + i * 32 + l32, h);
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if constexpr (EPI == kEpiBiasEluOut)  // C^T tile: the weight fragment is the MFMA's A operand
                        acc[i][j] = Arith<PL>::mfma(bf[j], af, acc[i][j]);
                    else
                        acc[i][j] = Arith<PL>::mfma(af, bf[j], acc[i][j]);
                }
            }
        }
        if (more) store_a_split<BM, PL>(an, lds[buf ^ 1], sa);
        __syncthreads();  // also retires the global_load_lds of chunk c+1 (vmcnt(0))
    }
    }  // !deep
    const float inv_sa = 1.f / sa;
    if constexpr (PL == 2) {
        // undo the operand scales: C[m][n] = acc / (s_a t_n), exact (powers of two)
        const float* inv_t =
            reinterpret_cast<const float*>(reinterpret_cast<const char*>(bimg) + h3_image_scales_offset(p.K));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if constexpr (EPI == kEpiBiasEluOut) {
                // C^T tiles: unscaled column by column in the epilogue below (its bias loads)
            } else {
                const float f = inv_t[wn * 64 + j * 32 + l32] * inv_sa;
#pragma unroll
                for (int i = 0; i < I; ++i)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[i][j][r] *= f;
            }
        }
    }

    const bool full = (row0 + BM <= p.M) && (p.N == kBN);
    float colpart[2];
    float amx = 0.f;  // max |stored output| of this lane (amax_commit)
#ifdef RSLRL_STAMPS
    uint64_t st1 = __builtin_amdgcn_s_memrealtime();
    uint64_t ct1 = __builtin_amdgcn_s_memtime();
#endif
    if constexpr (EPI == kEpiEluGradWgrad) {
        // one chunk (K <= 16): buffer 0 holds the tile's dZ planes; rebuild the fp32 rows (p0 + p1 + p2 is
        // exact) into buffer 1 as [128][16] for the weight-gradient accumulation
        float* dzo = reinterpret_cast<float*>(lds[1]);
        {
            const int r = threadIdx.x >> 2, q = threadIdx.x & 3;
            const int off = swz(r, q >> 1) + 8 * (q & 1);
            const uint2 p0 = *reinterpret_cast<const uint2*>(lds[0] + off);
            const uint2 p1 = *reinterpret_cast<const uint2*>(lds[0] + planeA + off);
            const uint2 p2 = *reinterpret_cast<const uint2*>(lds[0] + 2 * planeA + off);
            auto lo = [](uint32_t w) { return __uint_as_float(w << 16); };
            auto hi = [](uint32_t w) { return __uint_as_float(w & 0xffff0000u); };
            float4 v;
            v.x = (lo(p0.x) + lo(p1.x)) + lo(p2.x);
            v.y = (hi(p0.x) + hi(p1.x)) + hi(p2.x);
            v.z = (lo(p0.y) + lo(p1.y)) + lo(p2.y);
            v.w = (hi(p0.y) + hi(p1.y)) + hi(p2.y);
            *reinterpret_cast<float4*>(dzo + r * kMaxWgradRows + 4 * q) = v;
        }
        __syncthreads();
        f32x2 wacc[NR];
        epilogue_tiles_w<EPI, I, 2, NR>(p, acc, row0 + wm * (BM / 2), wn * 64, full, colpart, dzo, wm * (BM / 2), wacc,
                                        amx);
        // per-tile partial dW[o][col]: lane halves (rows 4h..) by shuffle, then the two wave rows in a fixed
        // order through LDS (the B region of buffer 0 is free after the main loop)
        float* red = reinterpret_cast<float*>(lds[0] + 3 * planeA);  // [16][256]
#pragma unroll
        for (int o = 0; o < NR; ++o)
#pragma unroll
            for (int j = 0; j < 2; ++j) wacc[o][j] += __shfl_xor(wacc[o][j], 32, 64);
        if (wm == 0 && h == 0) {
#pragma unroll
            for (int o = 0; o < NR; ++o)
#pragma unroll
                for (int j = 0; j < 2; ++j) red[o * kBN + wn * 64 + j * 32 + l32] = wacc[o][j];
        }
        __syncthreads();
        // per-tile partial sums of dZ itself (the layer's bias gradient): wave 0, lane (q, c) sums rows
        // 32 q .. 32 q + 31 of column c in order, the four quarters are added in order
        const int64_t tile_floats = static_cast<int64_t>(p.K) * p.N + p.K;
        if (threadIdx.x < 64) {
            const int c = threadIdx.x & 15, q = threadIdx.x >> 4;
            float sz = 0.f;
            for (int r = 32 * q; r < 32 * q + 32; ++r) sz += dzo[r * kMaxWgradRows + c];
            const float s1 = __shfl(sz, c + 16, 64), s2 = __shfl(sz, c + 32, 64), s3 = __shfl(sz, c + 48, 64);
            if (q == 0 && c < p.K)
                p.wpart[static_cast<int64_t>(blockIdx.x) * tile_floats + static_cast<int64_t>(p.K) * p.N + c] =
                    ((sz + s1) + s2) + s3;
        }
        if (wm == 1 && h == 0) {
            float* out = p.wpart + static_cast<int64_t>(blockIdx.x) * tile_floats;
#pragma unroll
            for (int o = 0; o < NR; ++o)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int col = wn * 64 + j * 32 + l32;
                    if (o < p.K && col < p.N) out[o * p.N + col] = red[o * kBN + col] + wacc[o][j];
                }
        }
    } else if constexpr (EPI == kEpiBiasEluOut && HEAD == 2) {
        static_assert(FULL && PL == 3, "actor head: full x6 tiles");
        actor_head_epilogue(p, *ap, acc, lds_b0, lds_b1, reinterpret_cast<const float*>(lds_b0 + kXsOff), wm, wn, lane,
                            wave, row0);
    } else if constexpr (EPI == kEpiBiasEluOut && HEAD == 1) {
        // The critic's head with its backward.  V = ELU(acc + b) w^T + b_out exactly as the plain value-head epilogue
        // below computes it (same operations, same order: the same bits), then dV = d loss / dV per row
        // (value_loss_grad), then the output layer's backward over the H tile still in registers (acc holds H after
        // the first pass): dZ = (dV w) * ELU'(H) -> p.c through the per-wave stage (whole-line stores), and this
        // tile's partial row of p.wpart = [dW = sum dV H | db = sum dV | 0 pad] (out_bwd_valu_body's layout; the
        // reduction order over the tile's rows differs).  dZ per element is out_bwd_valu_body's expression: the same
        // bits.  H never reaches HBM, and the output layer's backward reads nothing back.
        static_assert(NR == 1 && FULL && PL == 3, "value head: full x6 tiles, the VALU value head");
        float* xsb = reinterpret_cast<float*>(lds_b0 + kXsOff);
        float* wvl = xsb + kVhWOff;  // [N] value weights, column order
        float* dvl = wvl + kBN;      // [BM] the tile's target values (prologue DMA), replaced by dV
        const float* retl = dvl + BM;  // [BM] the tile's returns (prologue DMA)
        float* red = reinterpret_cast<float*>(lds[1]);  // [wm][wn][i][32] V partials (2 KiB)
        float* hred = reinterpret_cast<float*>(lds[1]) + 1024;  // [dZ sums wm 0, 1 | dW sums wm 0, 1][N] (4 KiB)
        // two 32 x 32 H blocks per wave in LDS (the i = 1 row of blocks, written in the first pass: 32 registers fewer
        // held through the dV step): area A = buffer 0 (block j = 1), area B = buffer 1 past red / hred (block j = 0);
        // each later stages one of the wave's i = 0 blocks.  Layout of the whole-line store stage: float4 column quads
        // XOR-swizzled by (row >> 1) & 7.
        float* const area0 = reinterpret_cast<float*>(lds[1] + 8192) + wave * 1024;
        float* const area1 = reinterpret_cast<float*>(lds[0]) + wave * 1024;
        static_assert(8192 + 8 * 4096 <= bufBytes, "value head: H blocks in LDS");
        auto stage_block = [&](float* blk, f32x16 v) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 hv = {v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
                *reinterpret_cast<f32x4*>(blk + l32 * 32 + 4 * ((2 * g + h) ^ ((l32 >> 1) & 7))) = hv;
            }
        };
#pragma unroll
        for (int ii = 0; ii < I; ++ii) {
            const int i = I - 1 - ii;  // the parked row of blocks first: its registers die before the other's H forms
            float oval = 0.f;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int cb = wn * 64 + j * 32 + 4 * h;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float4 b4 = *reinterpret_cast<const float4*>(xsb + cb + 8 * g);
                    float t[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                    t[0] += b4.x;
                    t[1] += b4.y;
                    t[2] += b4.z;
                    t[3] += b4.w;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float n = elu_neg(fminf(t[e], 0.f));
                        acc[i][j][4 * g + e] = t[e] > 0.f ? t[e] : n;
                    }
                }
                const float4* wl = reinterpret_cast<const float4*>(xsb + kBN) + 2 * ((((wn * 2 + j) * 2) * 2 + h) * kXsOut);
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const float4* q = wl + 2 * (s2 * 2 * kXsOut);
                    const float4 w0 = q[0], w1 = q[1];
                    const float w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
                    for (int t = 0; t < 8; ++t) oval = fmaf(acc[i][j][8 * s2 + t], w[t], oval);
                }
                if (i == I - 1) stage_block(j ? area1 : area0, acc[i][j]);
            }
            const float tsum = oval + __shfl_xor(oval, 32, 64);
            if (h == 0) red[((wm * 4 + wn) * I + i) * 32 + l32] = tsum;
        }
        __syncthreads();
        if (threadIdx.x < BM) {  // the four wn partials in the plain epilogue's order
            const int rl = threadIdx.x;
            const float tv = dvl[rl], ret = retl[rl];
            const float* b = red + (rl >> 6) * 4 * I * 32 + ((rl & 63) >> 5) * 32 + (rl & 31);
            const float sum = ((b[0] + b[I * 32]) + b[2 * I * 32]) + b[3 * I * 32];
            const float V = sum + p.obias[0];
            p.y[row0 + rl] = V;
            dvl[rl] = value_loss_grad(V, tv, ret, p.vh_clipped, p.vh_clip, p.vh_g);
        }
        __syncthreads();
        const int cq = lane & 7;
        // dZ of one staged block (i, j): lane (row 8 k + lane >> 3, column quad cq) -> whole-line stores
        auto block_bwd = [&](const float* blk, int i, int j, float (&cs)[4], float (&wsum)[4]) {
            const int64_t trow = row0 + wm * (BM / 2) + i * 32;
            float* ct = p.c + trow * p.N + (wn * 64 + j * 32);
            const float4 w4 = *reinterpret_cast<const float4*>(wvl + wn * 64 + j * 32 + 4 * cq);
            const float w[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll 1
            for (int k = 0; k < 4; ++k) {
                const int sr = 8 * k + (lane >> 3);
                const f32x4 hq = *reinterpret_cast<const f32x4*>(blk + sr * 32 + 4 * (cq ^ ((sr >> 1) & 7)));
                const float hh4[4] = {hq[0], hq[1], hq[2], hq[3]};
                const float dv = dvl[wm * (BM / 2) + i * 32 + sr];
                float o[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float hh = hh4[e];
                    const float z = __fmaf_rn(dv, w[e], 0.f);  // out_bwd_valu_body's fma chain of one term
                    const float v = hh > 0.f ? z : z * (hh + 1.f);  // ELU'(x) = 1 if h > 0 else h + 1
                    o[e] = v;
                    cs[e] += v;
                    wsum[e] = fmaf(dv, hh, wsum[e]);
                }
                const f32x4 ov = {o[0], o[1], o[2], o[3]};
                f32x4* dst = reinterpret_cast<f32x4*>(ct + static_cast<uint32_t>(sr * p.N + 4 * cq));
                if (p.nt) __builtin_nontemporal_store(ov, dst);
                else *dst = ov;
            }
        };
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            float cs[4] = {0.f, 0.f, 0.f, 0.f}, wsum[4] = {0.f, 0.f, 0.f, 0.f};
            float* const blk = j ? area1 : area0;
            block_bwd(blk, I - 1, j, cs, wsum);  // the block parked in the first pass
            __builtin_amdgcn_wave_barrier();     // one wave's LDS accesses execute in order
            stage_block(blk, acc[0][j]);         // then block (0, j) through the same area
            __builtin_amdgcn_wave_barrier();
            block_bwd(blk, 0, j, cs, wsum);
            // column sums over the wave's 64 rows: lanes of one column quad (lane & 7) differ in lane >> 3
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int off = 8; off < 64; off <<= 1) {
                    cs[e] += __shfl_xor(cs[e], off, 64);
                    wsum[e] += __shfl_xor(wsum[e], off, 64);
                }
            if (lane < 8) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int col = wn * 64 + j * 32 + 4 * lane + e;
                    hred[wm * kBN + col] = cs[e];
                    hred[(2 + wm) * kBN + col] = wsum[e];
                }
            }
        }
        __syncthreads();
        const int64_t tile_floats = (static_cast<int64_t>(p.N) + 1 + 3) / 4 * 4;  // dgrad_wgrad_tile_floats(1, N)
        float* wp = p.wpart + static_cast<int64_t>(blockIdx.x) * tile_floats;
        if (threadIdx.x < kBN) {
            const int c = threadIdx.x;
            wp[c] = hred[2 * kBN + c] + hred[3 * kBN + c];
            if (p.colsum) p.colsum[static_cast<int64_t>(blockIdx.x) * p.N + c] = hred[c] + hred[kBN + c];
        }
        if (threadIdx.x < 64) {  // db = sum of the tile's dV (fixed butterfly order)
            float sv = dvl[lane] + dvl[lane + 64];
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) sv += __shfl_xor(sv, off, 64);
            if (lane == 0) wp[kBN] = sv;
            else if (lane < static_cast<int>(tile_floats - kBN)) wp[kBN + lane] = 0.f;
        }
    } else if constexpr (EPI == kEpiBiasEluOut) {
        // C^T tiles: lane (l32, h) holds row l32 of the tile, columns (r & 3) + 8 (r >> 2) + 4 h (r < 16).
        // h = ELU(acc + b) is stored (when wanted) as float4 column quads, split into bf16 planes in
        // registers and multiplied by the output weight: Y'[o][row] = sum over this wave's 64 columns,
        // 2 k steps of 16 per 32-column tile (lane half h carries columns {0-3, 8-11} + 4 h, then
        // {16-19, 24-27} + 4 h; the image orders the weight the same way).  The four wn waves' partial
        // Y' tiles are added in a fixed order through LDS.
        // h leaves through a per-wave LDS stage (32 x 32 floats, float4 quads XOR-swizzled by (row >> 1) & 7):
        // written as the C^T quads, read back as 8 rows x 128 B per instruction -> whole-line stores (direct
        // C^T stores write 32-B pieces: +48 us per launch at M = 393216).  red: [wm][wn][i][o][32 rows].
        const bool staged = p.c != nullptr && p.nout <= kStagedOutWidth;
        const int red_rows = staged ? kStagedOutWidth : 32;
        // stage: buffer 0 (32 KiB); red: [wm][wn][i][o][32] in buffer 1 when staged (<= 40 KiB), else wave row wm
        // in buffer wm (32 KiB each)
        float* stage = reinterpret_cast<float*>(lds[0]) + wave * 1024;
        const int tile = red_rows * 32;
        auto red_of = [&](int w) {
            return staged ? reinterpret_cast<float*>(lds[1]) + w * 4 * I * tile : reinterpret_cast<float*>(lds[w]);
        };
        const uint4* oimg = p.oimg + wn * (2 * 2 * 3 * 64);
        constexpr bool valu = NR == 1;  // the critic's value head: VALU dot products beat 32-row MFMA tiles
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const int64_t row = row0 + wm * (BM / 2) + i * 32 + l32;
            const bool row_ok = row < p.M;
            f32x16 oacc = f32x16{};
            float oval[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int cb = wn * 64 + j * 32 + 4 * h;
                float v[16];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int col = cb + 8 * g;
                    const bool col_ok = col < p.N;  // N % 4 == 0
                    // (zero past N in the LDS copy)
                    const float4 b4 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(lds[0] + kXsOff) + col);
                    float t[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                    if constexpr (PL == 2) {  // h3: C = acc / (s_a t_n), exact
                        const float4 f4 = *reinterpret_cast<const float4*>(
                            reinterpret_cast<const float*>(reinterpret_cast<const char*>(bimg) +
                                                           h3_image_scales_offset(p.K)) + col);
                        t[0] *= f4.x * inv_sa;
                        t[1] *= f4.y * inv_sa;
                        t[2] *= f4.z * inv_sa;
                        t[3] *= f4.w * inv_sa;
                    }
                    t[0] += b4.x;
                    t[1] += b4.y;
                    t[2] += b4.z;
                    t[3] += b4.w;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {  // branch-free (see the full-tile epilogue)
                        const float n = elu_neg(fminf(t[e], 0.f));
                        v[4 * g + e] = t[e] > 0.f ? t[e] : n;
                    }
                    const f32x4 hv = {v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
                    if (staged) {
                        *reinterpret_cast<f32x4*>(stage + l32 * 32 + 4 * ((2 * g + h) ^ ((l32 >> 1) & 7))) = hv;
                    } else if (p.c && row_ok && col_ok) {
                        *reinterpret_cast<f32x4*>(p.c + row * p.N + col) = hv;
                    }
                }
                if (staged) {
                    __builtin_amdgcn_wave_barrier();  // one wave's LDS accesses execute in order
                    // wave-uniform tile base + 32-bit lane offsets (one VGPR per store, not a 64-bit address)
                    const int64_t trow = row0 + wm * (BM / 2) + i * 32;
                    float* ct = p.c + trow * p.N + (wn * 64 + j * 32);
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int sr = 8 * k + (lane >> 3);
                        const int cq = lane & 7;
                        const f32x4 hv = *reinterpret_cast<const f32x4*>(stage + sr * 32 + 4 * (cq ^ ((sr >> 1) & 7)));
                        const int gcol = wn * 64 + j * 32 + 4 * cq;
                        if (trow + sr < p.M && gcol < p.N) {
                            f32x4* dst = reinterpret_cast<f32x4*>(ct + static_cast<uint32_t>(sr * p.N + 4 * cq));
                            if (p.nt) __builtin_nontemporal_store(hv, dst);
                            else *dst = hv;
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                }
                if constexpr (valu) {
                    // <= 4 outputs: fp32 FMA chains over the lane's 16 columns (the image's fp32 copy; for 1
                    // output the copy in LDS, kXsOut entries per (wn, j, s, h))
                    const bool in_lds = p.nout <= kXsOut;
                    const float4* wf = reinterpret_cast<const float4*>(p.oimg + kOutImagePlaneUnits) +
                                       2 * ((((wn * 2 + j) * 2) * 2 + h) * 32);
                    const float4* wl = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(lds[0] + kXsOff) +
                                                                       kBN) + 2 * ((((wn * 2 + j) * 2) * 2 + h) * kXsOut);
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                        for (int o = 0; o < 4; ++o) {
                            if (o >= p.nout) break;
                            const float4* q = in_lds ? wl + 2 * (s2 * 2 * kXsOut + o) : wf + 2 * (s2 * 64 + o);
                            const float4 w0 = q[0], w1 = q[1];
                            const float w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
                            for (int t = 0; t < 8; ++t) oval[o] = fmaf(v[8 * s2 + t], w[t], oval[o]);
                        }
                    continue;
                }
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    bf16x8 vb[3], wa[3];
                    uint2 lo[3], hi[3];
                    split4(make_float4(v[8 * s2], v[8 * s2 + 1], v[8 * s2 + 2], v[8 * s2 + 3]), lo[0], lo[1], lo[2]);
                    split4(make_float4(v[8 * s2 + 4], v[8 * s2 + 5], v[8 * s2 + 6], v[8 * s2 + 7]), hi[0], hi[1],
                           hi[2]);
#pragma unroll
                    for (int q = 0; q < 3; ++q) {
                        vb[q] = __builtin_bit_cast(bf16x8, make_uint4(lo[q].x, lo[q].y, hi[q].x, hi[q].y));
                        wa[q] = __builtin_bit_cast(bf16x8, oimg[((j * 2 + s2) * 3 + q) * 64 + lane]);
                    }
                    oacc = mfma_x6(wa, vb, oacc);
                }
            }
            float* rd = red_of(wm) + (wn * I + i) * tile;
            if constexpr (valu) {  // the two lane halves hold different columns of the same row
#pragma unroll
                for (int o = 0; o < 4; ++o) {
                    const float t = oval[o] + __shfl_xor(oval[o], 32, 64);
                    if (h == 0 && o < p.nout) rd[o * 32 + l32] = t;
                }
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int o = (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (o < red_rows) rd[o * 32 + l32] = oacc[r];
                }
            }
        }
        __syncthreads();
        const int nout = p.nout;
        for (int idx = threadIdx.x; idx < BM * nout; idx += kThreads) {
            const int rl = idx / nout;
            const int o = idx - rl * nout;
            const float* b = red_of(rl >> 6) + ((rl & 63) >> 5) * tile + o * 32 + (rl & 31);
            const float sum = ((b[0] + b[I * tile]) + b[2 * I * tile]) + b[3 * I * tile];
            const int64_t row = row0 + rl;
            if (row < p.M) p.y[row * nout + o] = sum + p.obias[o];
        }
    } else {
        bool staged = false;
        if constexpr (kStagedEpi && PL == 3 && EPI == kEpiBiasElu) {
            // plain full tiles (the paired update launches): 16-byte I/O through a per-wave stage in buffer 0 (the
            // input gradient takes the w4 kernel's staged epilogue instead: beside the 128-register one here it spilled)
            staged = full && p.colsum == nullptr && p.amax_out == nullptr && !stage_h0;
            if (staged)
                epilogue_tiles_staged<EPI, I, 2>(p, acc, row0 + wm * (BM / 2), wn * 64,
                                                 reinterpret_cast<float*>(lds[0]) + wave * 1024);
        }
        if (!staged)
            epilogue_tiles<EPI, I, 2>(p, acc, row0 + wm * (BM / 2), wn * 64, full, colpart, amx,
                                      stage_h0 && full ? reinterpret_cast<const float*>(lds[0]) : nullptr);
    }
#ifdef RSLRL_STAMPS
    {
        uint64_t st2 = __builtin_amdgcn_s_memrealtime();
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        if (threadIdx.x == 0 || threadIdx.x == 448) {
            uint64_t* o = g_stamps + (static_cast<int64_t>(blockIdx.x) * 2 + (threadIdx.x ? 1 : 0)) * 6;
            o[0] = st0; o[1] = st1; o[2] = st2; o[3] = (static_cast<uint64_t>(xcc) << 32) | hw;
            o[4] = ct0; o[5] = ct1;
        }
    }
#endif
    // (colsum == nullptr: the previous layer's bias gradient comes from its weight-gradient kernel instead)
    if (EPI == kEpiEluGrad || EPI == kEpiEluGradWgrad) if (p.colsum) {
        // column sums over the tile's 128 rows -> colsum[tile][col]: lanes l and l + 32 hold the two row
        // halves of a column, the two wave rows (wm) are combined in a fixed order through LDS
        float s[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) s[j] = colpart[j] + __shfl_xor(colpart[j], 32, 64);
        float* colred = reinterpret_cast<float*>(lds[0]);
        __syncthreads();  // the LDS tiles are no longer read
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (h == 0) colred[wm * kBN + wn * 64 + j * 32 + l32] = s[j];
        __syncthreads();
        for (int col = threadIdx.x; col < p.N && col < kBN; col += kThreads)
            p.colsum[static_cast<int64_t>(blockIdx.x) * p.N + col] = colred[col] + colred[kBN + col];
    }
    if constexpr (EPI != kEpiBiasEluOut) amax_commit(p, amx);
}

template <int EPI, bool FULL, int MINW, int NR = 4, int PL = 3, int KCH = 0>
__global__ __launch_bounds__(kThreads, MINW) void mlp_gemm_x6_kernel(GemmParams p, const uint4* __restrict__ bimg) {
    __shared__ __attribute__((aligned(16))) char lds_b0[x6_buf_bytes<EPI, PL>()];
    __shared__ __attribute__((aligned(16))) char lds_b1[x6_buf_bytes<EPI, PL>()];
    mlp_gemm_x6_body<EPI, FULL, NR, PL, true, KCH>(p, bimg, lds_b0, lds_b1);
}

// The critic's last hidden layer + value head + d(value loss)/dV + the value head's backward (dZ of the last hidden
// layer and the head's weight-gradient partials) in one launch (rslrl_value_head_fwd_bwd): full 128-row tiles, x6.
__global__ __launch_bounds__(kThreads, 4) void mlp_gemm_x6_value_head_kernel(GemmParams p, const uint4* __restrict__ bimg) {
    __shared__ __attribute__((aligned(16))) char lds_b0[x6_buf_bytes<kEpiBiasEluOut, 3>()];
    __shared__ __attribute__((aligned(16))) char lds_b1[x6_buf_bytes<kEpiBiasEluOut, 3>()];
    mlp_gemm_x6_body<kEpiBiasEluOut, true, 1, 3, true, 0, 1>(p, bimg, lds_b0, lds_b1);
}

// The actor's last hidden layer + output layer + the PPO loss + the output layer's backward in one launch
// (rslrl_actor_head_fwd_bwd; actor_head_epilogue): full 128-row tiles, x6.
__global__ __launch_bounds__(kThreads, 4) void mlp_gemm_x6_actor_head_kernel(GemmParams p, const uint4* __restrict__ bimg,
                                                                           ActorParams ap) {
    __shared__ __attribute__((aligned(16))) char lds_b0[x6_buf_bytes<kEpiBiasEluOut, 3>()];
    __shared__ __attribute__((aligned(16))) char lds_b1[x6_buf_bytes<kEpiBiasEluOut, 3>()];
    mlp_gemm_x6_body<kEpiBiasEluOut, true, 4, 3, true, 0, 2>(p, bimg, lds_b0, lds_b1, &ap);
}

// the K = 48 kernel applies to full tiles of a forward on x6 operands with the deep loop enabled
template <int EPI>
bool k48_deep(const GemmParams& p, bool fullm, int pl) {
    return (EPI == kEpiBias || EPI == kEpiBiasElu) && pl == 3 && fullm && p.K == 3 * kKC && p.deep;
}

// Two independent problems of one shape in one launch (blockIdx.y picks the problem): the rollout's actor and
// critic layers, whose 512-tile launches (M = 65536) leave half of the 2-per-CU workgroup slots idle.  Each
// problem keeps its own amax output and workspace (the protocol counts gridDim.x workgroups per problem).
struct GemmPair {
    GemmParams p[2];
    const uint4* img[2];
};

template <int EPI, bool FULL, int PL, int KCH = 0, bool STAGE = false>
__global__ __launch_bounds__(kThreads, 4) void mlp_gemm_x6_pair_kernel(GemmPair b) {
    __shared__ __attribute__((aligned(16))) char lds_b0[x6_buf_bytes<EPI, PL>()];
    __shared__ __attribute__((aligned(16))) char lds_b1[x6_buf_bytes<EPI, PL>()];
    const int y = blockIdx.y;
    mlp_gemm_x6_body<EPI, FULL, 4, PL, STAGE, KCH>(b.p[y], b.img[y], lds_b0, lds_b1);
}

// The actor's and the critic's fused last hidden + output layer in one launch (blockIdx.y): the two output widths
// take different epilogues (NR 4: MFMA output layer, e.g. 12 actions; NR 1: VALU, <= 4 outputs, e.g. the value
// head), one body each over the shared LDS buffers.  At the rollout's 16,384 rows per GPU each alone fills a
// quarter of the workgroup slots.
template <bool FULL, int MINW, int NR0, int NR1, int PL>
__global__ __launch_bounds__(kThreads, MINW) void mlp_gemm_x6_out_pair_kernel(GemmPair b) {
    __shared__ __attribute__((aligned(16))) char lds_b0[x6_buf_bytes<kEpiBiasEluOut, PL>()];
    __shared__ __attribute__((aligned(16))) char lds_b1[x6_buf_bytes<kEpiBiasEluOut, PL>()];
    // (distinct opaque markers open the two branches: otherwise the bodies' common index arithmetic is hoisted
    // above the branch, lives through either body and spills)
    if (blockIdx.y == 0) {
        asm volatile("; out pair: problem 0" ::: "memory");
        mlp_gemm_x6_body<kEpiBiasEluOut, FULL, NR0, PL>(b.p[0], b.img[0], lds_b0, lds_b1);
    } else {
        asm volatile("; out pair: problem 1" ::: "memory");
        mlp_gemm_x6_body<kEpiBiasEluOut, FULL, NR1, PL>(b.p[1], b.img[1], lds_b0, lds_b1);
    }
}

// ---- the same x6 GEMM on v_mfma_f32_16x16x32_bf16 ("paired" x6).  Under load the chip holds a higher
// clock on the 16x16x32 shape than on 32x32x16 at equal cycles per FLOP (MI355X_MICROARCH.md, DVFS
// give-back item 7).  Its k = 32 is spent on two plane products of the same 16-deep chunk: lanes 0-31
// carry the first product of a pair, lanes 32-63 the second (a dot product does not care which lanes
// hold which k), so three MFMAs per 16x16 tile and chunk accumulate, smallest terms first,
//   P1 = a0b2 + a2b0,  P2 = a1b1 + a0b1,  P3 = a1b0 + a0b0.
// A fragments: P1 reads plane (0 | 2), P2 and P3 share plane (1 | 0); B fragments: (2 | 0), 1, 0.  Lane l
// reads row (l & 15) of its 16-row block, k half (l >> 4) & 1 -- each 16-lane group covers all 64 banks
// through the same row-half swizzle, so the LDS image and its staging are the 32x32x16 kernel's.
// The MFMAs take the weight fragment as their A operand and the activation fragment as B, so they
// produce C^T tiles: lane l holds row (l & 15) of its 16-row block and the four consecutive columns
// 4 (l >> 4) .. +3 of its 16-column block -> 16-byte stores and h loads in the epilogue.  Wave tile 64 x 64.
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

template <int EPI, bool FULLT, bool NT>
__device__ __forceinline__ void epilogue16_impl(const GemmParams& p, f32x4 (&acc)[4][4], int64_t wrow0, int wcol0,
                                                f32x4 (&colpart)[4]) {
    constexpr bool full = FULLT;
    constexpr bool GRAD = EPI == kEpiEluGrad;
    const int lane = threadIdx.x & 63;
    const int l16 = lane & 15;
    const int cq = 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) colpart[j] = f32x4{};
    f32x4 bias[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int col = wcol0 + 16 * j + cq;  // N % 4 == 0 (launch)
        bias[j] = f32x4{};
        if constexpr (!GRAD) {
            if (col < p.N) {
                const float4 b = ld4(p.bias + col);
                bias[j] = f32x4{b.x, b.y, b.z, b.w};
            }
        }
    }
    // h of row block i (4 column quads), loaded at the block's start: a prefetch of block i + 1 would
    // push the 128-register allocation into scratch
    f32x4 hcur[4];
    auto load_h = [&](int i, f32x4 (&dst)[4]) {
        const int64_t row = wrow0 + 16 * i + l16;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = wcol0 + 16 * j + cq;
            dst[j] = f32x4{};
            if (full || (row < p.M && col < p.N)) {
                const float4 v = ld4(p.h + row * p.N + col);
                dst[j] = f32x4{v.x, v.y, v.z, v.w};
            }
        }
    };
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if constexpr (GRAD) load_h(i, hcur);
        const int64_t row = wrow0 + 16 * i + l16;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = wcol0 + 16 * j + cq;
            f32x4 v = acc[i][j];
            if constexpr (EPI == kEpiBias) {
                v = v + bias[j];
            } else if constexpr (EPI == kEpiBiasElu) {
                v = v + bias[j];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : elu_neg(v[r]);
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float hv = hcur[j][r];
                    v[r] = hv > 0.f ? v[r] : v[r] * (hv + 1.f);
                }
            }
            if (full || (row < p.M && col < p.N)) {
                if constexpr (GRAD) colpart[j] = colpart[j] + v;
                f32x4* dst = reinterpret_cast<f32x4*>(p.c + row * p.N + col);
                if constexpr (NT) __builtin_nontemporal_store(v, dst);
                else *dst = v;
            }
        }
    }
}

template <int EPI, bool FULL, int MINW, bool NT>
__global__ __launch_bounds__(kThreads, MINW) void mlp_gemm_x6s_kernel(GemmParams p, const uint4* __restrict__ bimg) {
    constexpr int BM = kBM;
    constexpr int planeA = BM * kX6RowB;
    constexpr int bufBytes = 3 * planeA + kX6ChunkB;
    static_assert(EPI == kEpiBias || EPI == kEpiBiasElu || EPI == kEpiEluGrad, "no fused weight gradient here");
    __shared__ __attribute__((aligned(16))) char lds[2][bufBytes];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave >> 2;  // rows wm * 64
    const int wn = wave & 3;   // cols wn * 64
    const int hs = lane >> 5;          // which product of a pair
    const int hk = (lane >> 4) & 1;    // k half of the chunk
    const int l16 = lane & 15;
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * BM;
    const int offA0 = (hs ? 2 : 0) * planeA;     // P1: a0 | a2
    const int offA1 = (hs ? 0 : 1) * planeA;     // P2, P3: a1 | a0
    const int offB0 = (hs ? 0 : 2) * kX6PlaneB;  // P1: b2 | b0

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

    // one chunk's fragments and MFMAs (a_lds / b_lds: the chunk's A planes and B image in LDS)
    auto compute = [&](const char* a_lds, const char* b_lds) {
        bf16x8 af[4][2];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = wm * 64 + 16 * i + l16;
            af[i][0] = read_frag(a_lds + offA0, row, hk);
            af[i][1] = read_frag(a_lds + offA1, row, hk);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = wn * 64 + 16 * j + l16;
            const bf16x8 b0 = read_frag(b_lds + offB0, col, hk);
            const bf16x8 b1 = read_frag(b_lds + kX6PlaneB, col, hk);
            const bf16x8 b2 = read_frag(b_lds, col, hk);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0, af[i][0], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1, af[i][1], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b2, af[i][1], acc[i][j], 0, 0, 0);
            }
        }
    };
    bool deep = false;
    if constexpr (FULL) {
        if (p.K == 16 * kKC && p.deep) {  // the unrolled look-ahead pipeline (K = 256)
            char* ldsp[2] = {lds[0], lds[1]};
            deep_pipeline<BM, 3, 16, kX6Depth>(p, row0, bimg, ldsp, 1.f, compute);
            deep = true;
        }
    }
    const int nchunks = deep ? 0 : (p.K + kKC - 1) / kKC;
    if (!deep) {
    load_b_lds<3>(bimg, 0, lds[0] + 3 * planeA);
    store_a_split<BM, 3>(load_a<BM, FULL>(p, row0, 0), lds[0], 1.f);
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
        const int buf = c & 1;
        const bool more = c + 1 < nchunks;
        AStage<BM> an;
        if (more) {
            load_b_lds<3>(bimg, c + 1, lds[buf ^ 1] + 3 * planeA);
            an = load_a<BM, FULL>(p, row0, (c + 1) * kKC);
        }
        compute(lds[buf], lds[buf] + 3 * planeA);
        if (more) store_a_split<BM, 3>(an, lds[buf ^ 1], 1.f);
        __syncthreads();
    }
    }  // !deep

    const bool full = (row0 + BM <= p.M) && (p.N == kBN);
    f32x4 colpart[4];
    if (full)
        epilogue16_impl<EPI, true, NT>(p, acc, row0 + wm * 64, wn * 64, colpart);
    else
        epilogue16_impl<EPI, false, NT>(p, acc, row0 + wm * 64, wn * 64, colpart);
    if constexpr (EPI == kEpiEluGrad) {
        // column sums over the tile's 128 rows: the 16 lanes of a group hold 16 rows of the same columns
        // (butterfly over lane bits 0-3, a fixed order), the two wave rows (wm) are combined through LDS
#pragma unroll
        for (int m = 1; m < 16; m <<= 1)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) colpart[j][r] += __shfl_xor(colpart[j][r], m, 64);
        float* colred = reinterpret_cast<float*>(lds[0]);
        __syncthreads();  // the LDS tiles are no longer read
        if ((lane & 15) == 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                *reinterpret_cast<f32x4*>(colred + wm * kBN + wn * 64 + 16 * j + 4 * (lane >> 4)) = colpart[j];
        }
        __syncthreads();
        for (int col = threadIdx.x; col < p.N && col < kBN; col += kThreads)
            p.colsum[static_cast<int64_t>(blockIdx.x) * p.N + col] = colred[col] + colred[kBN + col];
    }
}

// tuning knob: RSLRL_X6S_NT=0|1 (default 0): streaming stores in the 16x16 epilogue.  Its 64-byte row
// pieces are better served by ordinary stores (K=48 forward 126 vs 159 us; the 32x32 epilogue writes whole
// 128-byte lines per instruction and gains from streaming stores instead)
bool x6s_nontemporal() {
    static const bool v = [] {
        const char* e = std::getenv("RSLRL_X6S_NT");
        return e && std::atoi(e) == 1;
    }();
    return v;
}

// tuning knob: RSLRL_X6_SHAPE=16|32 (default 32): MFMA shape of the long-K x6 forward GEMMs.  Measured at
// C3 (bench.py, 3 x 20 iterations each): 16x16x32 13.10 M vs 32x32x16 13.05 M env-steps/s -- on par; the
// forward kernels gain 2-7 % per launch, the dgrad epilogue does not fit 128 registers on the 16x16 tiling
// (acc spills in the main loop: 1.2 ms per launch) and stays on 32x32x16.
int x6_shape() {  // read per call (A/B measurements in one process)
    const char* e = std::getenv("RSLRL_X6_SHAPE");
    return (e && std::atoi(e) == 16) ? 16 : 32;
}

// Bias gradient: out[col] = sum over tiles of part[tiles][N], in two launches and a fixed order.  Pass 1:
// workgroup (column group of 64, slice s) sums the slice's tiles (4 phases of 64 columns, fp64, phases
// folded in order) and leaves the slice sum in the slice's first row (that element was read by the same
// thread); pass 2 adds the slice sums in order.  The partials are scratch: pass 1 overwrites them.
constexpr int kFoldCols = 64;
constexpr int kFoldPhases = kBlock / kFoldCols;
constexpr int kFoldSlices = 64;
__global__ __launch_bounds__(kBlock) void colsum_slice_kernel(float* __restrict__ part, int tiles, int n, int per) {
    __shared__ double scratch[kFoldPhases][kFoldCols];
    const int c = threadIdx.x % kFoldCols, ph = threadIdx.x / kFoldCols;
    const int col = blockIdx.x * kFoldCols + c;
    const int t0 = blockIdx.y * per;
    const int t1 = t0 + per < tiles ? t0 + per : tiles;
    double s = 0.0;
    if (col < n) {
#pragma unroll 4
        for (int t = t0 + ph; t < t1; t += kFoldPhases) s += static_cast<double>(part[static_cast<int64_t>(t) * n + col]);
    }
    scratch[ph][c] = s;
    __syncthreads();
    if (ph == 0 && col < n) {
        double tot = 0.0;
        for (int q = 0; q < kFoldPhases; ++q) tot += scratch[q][c];
        part[static_cast<int64_t>(t0) * n + col] = static_cast<float>(tot);
    }
}

// pass 2: thread (group g, column c) loads slices g, g + 4, ... (<= 16, all loads issued before the adds) and the
// four group sums are added in g order
__global__ __launch_bounds__(kBlock) void colsum_fold_kernel(const float* __restrict__ part, int slices, int n,
                                                             int per, float* __restrict__ out) {
    __shared__ double scratch[kFoldPhases][kFoldCols];
    const int c = threadIdx.x % kFoldCols, g = threadIdx.x / kFoldCols;
    const int col = blockIdx.x * kFoldCols + c;
    constexpr int kMaxPer = kFoldSlices / kFoldPhases;
    float v[kMaxPer];
#pragma unroll
    for (int i = 0; i < kMaxPer; ++i) {
        const int s = g + kFoldPhases * i;
        v[i] = (col < n && s < slices) ? part[static_cast<int64_t>(s) * per * n + col] : 0.f;
    }
    double tot = 0.0;
#pragma unroll
    for (int i = 0; i < kMaxPer; ++i) tot += static_cast<double>(v[i]);
    scratch[g][c] = tot;
    __syncthreads();
    if (g == 0 && col < n) {
        double t = 0.0;
        for (int q = 0; q < kFoldPhases; ++q) t += scratch[q][c];
        out[col] = static_cast<float>(t);
    }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int dgrad_occupancy() {  // tuning knob: RSLRL_DGRAD_OCC=2|4 (default 4)
    static const int v = [] {
        const char* e = std::getenv("RSLRL_DGRAD_OCC");
        return (e && std::atoi(e) == 2) ? 2 : 4;
    }();
    return v;
}

// the opt-in 16x16x32 forward (RSLRL_X6_SHAPE=16); false: not taken
template <int EPI>
bool launch_x6s(const GemmParams& p, const uint4* img, bool fullm, dim3 g, hipStream_t st) {
    if constexpr (EPI == kEpiBias || EPI == kEpiBiasElu) {
        if (x6_shape() != 16 || (p.N & 3) || !aligned16(p.c) || !aligned16(p.bias) || p.amax_out)
            return false;  // 16-B epilogue, no amax
        const dim3 b(kThreads);
        const char* mw = std::getenv("RSLRL_X6S_MINW");  // tuning knob, read per call: 2 = one workgroup per CU
        if (mw && std::atoi(mw) == 2) {
            if (fullm) hipLaunchKernelGGL((mlp_gemm_x6s_kernel<EPI, true, 2, false>), g, b, 0, st, p, img);
            else hipLaunchKernelGGL((mlp_gemm_x6s_kernel<EPI, false, 2, false>), g, b, 0, st, p, img);
        } else if (x6s_nontemporal()) {
            if (fullm) hipLaunchKernelGGL((mlp_gemm_x6s_kernel<EPI, true, 4, true>), g, b, 0, st, p, img);
            else hipLaunchKernelGGL((mlp_gemm_x6s_kernel<EPI, false, 4, true>), g, b, 0, st, p, img);
        } else {
            if (fullm) hipLaunchKernelGGL((mlp_gemm_x6s_kernel<EPI, true, 4, false>), g, b, 0, st, p, img);
            else hipLaunchKernelGGL((mlp_gemm_x6s_kernel<EPI, false, 4, false>), g, b, 0, st, p, img);
        }
        return true;
    } else {
        return false;
    }
}

int out_fwd_nt() {  // tuning knob: RSLRL_OUT_FWD_NT=0|1
    static const int v = [] {
        const char* e = std::getenv("RSLRL_OUT_FWD_NT");
        return (e && std::atoi(e) == 1) ? 1 : 0;
    }();
    return v;
}

int cu_count() {  // compute units of the current device (cached per device)
    static int cache[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cache[dev] <= 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cache[dev] = n;
    }
    return cache[dev];
}

int out_fwd_occupancy() {  // tuning knob: RSLRL_OUT_FWD_OCC=2|4 (default 4)
    static const int v = [] {
        const char* e = std::getenv("RSLRL_OUT_FWD_OCC");
        return (e && std::atoi(e) == 2) ? 2 : 4;
    }();
    return v;
}

// ---- Output-layer backward on the VALU (RSLRL_LINEAR_DGRAD_ELU_WGRAD; x6 image of W^T as input).  With a
// 4-16 wide reduction this op is a stream over H (read) and dZ_prev (written) with ~24 FMAs per element: MFMA
// tiles buy nothing here and their epilogue needed 256 registers (one workgroup per CU, hundreds of bytes of
// scratch per lane).  Per 128-row tile (workgroup of 4 waves, 32 rows each; lane l owns columns 4l..4l+3):
//   z[c] = sum_o dZ[row][o] W[o][c] (fp32 FMA chain, o ascending; W rebuilt exactly from the image's three
//   bf16 planes), dZ_prev = z * ELU'(H), column sums of dZ_prev, dW[o][c] += dZ[row][o] H[row][c], and
//   db_out[o] = sum of dZ[row][o] -- the same per-tile partial layouts as the MFMA kernel (tile-major).
// dZ rows are wave-uniform (scalar loads); four rows of H are in flight per wave.
constexpr int kOutBwdThreads = 256;

// per-tile partial row of the output-layer backward: dW [Nred][N], db [Nred], zero pad to a multiple of 4 floats
__host__ __device__ inline int64_t dgrad_wgrad_tile_floats(int nred, int n) {
    return (static_cast<int64_t>(nred) * n + nred + 3) / 4 * 4;
}

// CPL columns per lane (4: a wave spans a 256-column row; 2: two waves share a row, so W and the dW
// accumulators take 2 NR registers each instead of 4 NR -- NR >= 12 needed 178+ registers at CPL 4)
// LDS of one out_bwd body: red [RG][NR + 1][kBN] floats (per-row-group dW rows, then column sums), dzt4 [kBM][NR / 4]
// float4s (the tile's dZ rows), dzsum [RG][NR] floats
template <int NR, int CPL>
struct OutBwdLds {
    static constexpr int WPR = kBN / (kWave * CPL);          // waves per row
    static constexpr int RG = (kOutBwdThreads / kWave) / WPR;  // row groups per workgroup
    static constexpr int kRed = RG * (NR + 1) * kBN * 4;
    static constexpr int kDzt = kBM * (NR / 4) * 16;
    static constexpr int kBytes = kRed + kDzt + RG * NR * 4;
};

template <int NR, int CPL>
__device__ __forceinline__ void out_bwd_valu_body(const GemmParams& p, const uint4* __restrict__ bimg, char* smem) {
    using LD = OutBwdLds<NR, CPL>;
    constexpr int WPR = LD::WPR;
    constexpr int RG = LD::RG;
    constexpr int RPW = kBM / RG;                      // rows per wave
    using vec = typename std::conditional<CPL == 4, f32x4, f32x2>::type;
    auto red = reinterpret_cast<float (*)[NR + 1][kBN]>(smem);
    auto dzt4 = reinterpret_cast<float4 (*)[NR / 4]>(smem + LD::kRed);
    auto dzsum = reinterpret_cast<float (*)[NR]>(smem + LD::kRed + LD::kDzt);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int rg = wave / WPR;
    const int c0 = CPL * (lane + kWave * (wave % WPR));
    const bool col_ok = c0 < p.N;  // N % 4 == 0
    // W[o][c0 + e] from the image of W^T: chunk 0, row n = c0 + e, k = o; 16-byte half ph holds k = 8 lh + j
    float w[NR][CPL];
#pragma unroll
    for (int e = 0; e < CPL; ++e) {
        const int n = c0 + e;
#pragma unroll
        for (int lh = 0; lh < (NR + 7) / 8; ++lh) {
            const int ph = lh ^ ((n >> 3) & 1);
            uint4 q[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                q[pl] = col_ok ? bimg[(pl * kX6PlaneB + n * kX6RowB + 16 * ph) / 16] : make_uint4(0, 0, 0, 0);
            const uint32_t* u0 = reinterpret_cast<const uint32_t*>(&q[0]);
            const uint32_t* u1 = reinterpret_cast<const uint32_t*>(&q[1]);
            const uint32_t* u2 = reinterpret_cast<const uint32_t*>(&q[2]);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int o = 8 * lh + j;
                if (o >= NR) break;
                auto f = [j](const uint32_t* u) {
                    const uint32_t x = u[j >> 1];
                    return __uint_as_float((j & 1) ? (x & 0xffff0000u) : (x << 16));
                };
                w[o][e] = (f(u0) + f(u1)) + f(u2);  // exact: the planes were split from this fp32 value
            }
        }
    }
    float wacc[NR][CPL], cs[CPL], dzs[NR];
#pragma unroll
    for (int e = 0; e < CPL; ++e) cs[e] = 0.f;
#pragma unroll
    for (int o = 0; o < NR; ++o) {
        dzs[o] = 0.f;
#pragma unroll
        for (int e = 0; e < CPL; ++e) wacc[o][e] = 0.f;
    }
    float amx = 0.f;
    // the tile's dZ rows (128 x NR floats) staged once in LDS: a per-row uniform global load is a vector load
    // the waves would wait on (the compiler cannot prove dZ read-only for the scalar cache)
    // (p.K = Nred, the row stride of dZ: NR = Nred rounded up to 4, the missing rows staged as zeros -- a 1-wide
    // value head reads its [M, 1] gradient as it is, no zero-padded copy)
    {
        const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kBM;
        if (p.K == NR) {
            for (int i = threadIdx.x; i < kBM * NR / 4; i += kOutBwdThreads) {
                const int r = i / (NR / 4), q = i % (NR / 4);
                dzt4[r][q] = t0 + r < p.M ? *reinterpret_cast<const float4*>(p.a + (t0 + r) * p.K + 4 * q)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        } else {
            float* dzt = reinterpret_cast<float*>(dzt4);
            for (int i = threadIdx.x; i < kBM * NR; i += kOutBwdThreads) {
                const int r = i / NR, o = i % NR;
                dzt[i] = (t0 + r < p.M && o < p.K) ? p.a[(t0 + r) * p.K + o] : 0.f;
            }
        }
        __syncthreads();
    }
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * kBM + rg * RPW;
    const int64_t rows = p.M - row0 < RPW ? (p.M - row0 > 0 ? p.M - row0 : 0) : RPW;
#ifndef RSLRL_OUTBWD_U
#define RSLRL_OUTBWD_U 4  // (8: 188.4 us, 16: 223 us, 4: 185.5 us -- the actor's 393,216 rows, scripts/outbwd_u_ab.sh)
#endif
    constexpr int U = RSLRL_OUTBWD_U;  // rows of H in flight per wave
    for (int r0 = 0; r0 < rows; r0 += U) {
        vec hv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t row = row0 + (r0 + u < rows ? r0 + u : rows - 1);
            hv[u] = col_ok ? *reinterpret_cast<const vec*>(p.h + row * p.N + c0) : vec{};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (r0 + u >= rows) break;  // wave-uniform
            const int64_t row = row0 + r0 + u;
            float d[NR];
#pragma unroll
            for (int o4 = 0; o4 < NR / 4; ++o4) {  // LDS broadcast (every lane reads the same 16 bytes)
                const float4 t = dzt4[rg * RPW + r0 + u][o4];
                d[4 * o4] = t.x;
                d[4 * o4 + 1] = t.y;
                d[4 * o4 + 2] = t.z;
                d[4 * o4 + 3] = t.w;
            }
            vec out;
#pragma unroll
            for (int e = 0; e < CPL; ++e) {
                const float hh = hv[u][e];
                float z = 0.f;
#pragma unroll
                for (int o = 0; o < NR; ++o) z = fmaf(d[o], w[o][e], z);
                const float v = hh > 0.f ? z : z * (hh + 1.f);  // ELU'(x) = 1 if h > 0 else h + 1
                out[e] = v;
                cs[e] += v;
                amx = fmaxf(amx, fabsf(v));
#pragma unroll
                for (int o = 0; o < NR; ++o) wacc[o][e] = fmaf(d[o], hh, wacc[o][e]);
            }
            if (wave % WPR == 0)
#pragma unroll
                for (int o = 0; o < NR; ++o) dzs[o] += d[o];
            if (col_ok) __builtin_nontemporal_store(out, reinterpret_cast<vec*>(p.c + row * p.N + c0));
        }
    }
    // per-tile partials, the row groups added in order
#pragma unroll
    for (int o = 0; o <= NR; ++o)
#pragma unroll
        for (int e = 0; e < CPL; ++e) red[rg][o][c0 + e] = o < NR ? wacc[o][e] : cs[e];
    if (lane == 0 && wave % WPR == 0)
#pragma unroll
        for (int o = 0; o < NR; ++o) dzsum[rg][o] = dzs[o];
    __syncthreads();
    const int nred = p.K;
    const int64_t tile_floats = dgrad_wgrad_tile_floats(nred, p.N);
    float* wp = p.wpart + static_cast<int64_t>(blockIdx.x) * tile_floats;
    for (int idx = threadIdx.x; idx < (NR + 1) * kBN; idx += kOutBwdThreads) {
        const int o = idx / kBN, c = idx % kBN;
        if (c >= p.N) continue;
        float v = red[0][o][c];
#pragma unroll
        for (int g = 1; g < RG; ++g) v += red[g][o][c];
        if (o < nred) wp[static_cast<int64_t>(o) * p.N + c] = v;
        else if (o == NR && p.colsum) p.colsum[static_cast<int64_t>(blockIdx.x) * p.N + c] = v;
    }
    if (threadIdx.x < nred) {
        float v = dzsum[0][threadIdx.x];
#pragma unroll
        for (int g = 1; g < RG; ++g) v += dzsum[g][threadIdx.x];
        wp[static_cast<int64_t>(nred) * p.N + threadIdx.x] = v;
    }
    // the row's pad to a 16-byte multiple (the fold reads float4 columns): zeros
    const int pad = static_cast<int>(tile_floats - (static_cast<int64_t>(nred) * p.N + nred));
    if (threadIdx.x < pad) wp[static_cast<int64_t>(nred) * p.N + nred + threadIdx.x] = 0.f;
    amax_publish<kOutBwdThreads>(p.amax_out, p.amax_ws, amx);
}

template <int NR, int CPL>
__global__ __launch_bounds__(kOutBwdThreads, NR >= 16 ? 3 : 4) void out_bwd_valu_kernel(GemmParams p, const uint4* __restrict__ bimg) {
    __shared__ __attribute__((aligned(16))) char smem[OutBwdLds<NR, CPL>::kBytes];
    out_bwd_valu_body<NR, CPL>(p, bimg, smem);
}

// The actor's and the critic's output-layer backward in one launch (blockIdx.y; e.g. Nred 12 and 1), one body each
// over one LDS area: at 98,304 rows each fills three quarters of the workgroup slots.
template <int NR0, int CPL0, int NR1, int CPL1>
__global__ __launch_bounds__(kOutBwdThreads, 4) void out_bwd_valu_pair_kernel(GemmPair b) {
    constexpr int kBytes = OutBwdLds<NR0, CPL0>::kBytes > OutBwdLds<NR1, CPL1>::kBytes ? OutBwdLds<NR0, CPL0>::kBytes
                                                                                       : OutBwdLds<NR1, CPL1>::kBytes;
    __shared__ __attribute__((aligned(16))) char smem[kBytes];
    if (blockIdx.y == 0) {
        asm volatile("; out bwd pair: problem 0" ::: "memory");
        out_bwd_valu_body<NR0, CPL0>(b.p[0], b.img[0], smem);
    } else {
        asm volatile("; out bwd pair: problem 1" ::: "memory");
        out_bwd_valu_body<NR1, CPL1>(b.p[1], b.img[1], smem);
    }
}

int out_bwd_mode() {  // tuning knob: RSLRL_OUT_BWD=mfma selects the MFMA kernel (default: VALU)
    static const int v = [] {
        const char* e = std::getenv("RSLRL_OUT_BWD");
        return (e && std::string(e) == "mfma") ? 1 : 0;
    }();
    return v;
}

// bimage == nullptr: exact f32 MFMA main loop on p.bw; otherwise the split main loop on the image (PL = 3: x6
// bf16 planes, layout-0 image; PL = 2: h3 fp16 planes, layout-2 image, A scaled from *p.a_amax).
template <int EPI, int PL = 3>
int launch(const GemmParams& p, const void* bimage, hipStream_t st) {
    const int64_t tiles = ceil_div(p.M, kBM);
    if (tiles > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
    const dim3 g(static_cast<unsigned>(tiles)), b(kThreads);
    if (bimage) {
        const uint4* img = static_cast<const uint4*>(bimage);
        // a short reduction (the dgrad of the 12- / 1-wide output layer: one chunk) is bound by the
        // epilogue's h loads, which want the registers of the 2-waves-per-SIMD allocation
        const bool short_k = EPI != kEpiBias && EPI != kEpiBiasElu && p.K <= 2 * kKC;
        const bool fullm = p.M % kBM == 0 && p.K % kKC == 0;
        if constexpr (EPI == kEpiEluGradWgrad) {  // K = Nred in {4, 8, 12, 16}
            if constexpr (PL != 3) {
                return RSLRL_E_UNSUPPORTED;
            } else if (out_bwd_mode() == 0) {
                auto go = [&](auto nr) {
                    constexpr int NR = decltype(nr)::value;
                    constexpr int CPL = NR <= 4 ? 4 : 2;
                    hipLaunchKernelGGL((out_bwd_valu_kernel<NR, CPL>), g, dim3(kOutBwdThreads), 0, st, p, img);
                };
                switch ((p.K + 3) / 4 * 4) {  // Nred 1..16; a partial last group of 4 is staged with zeros
                    case 4: go(std::integral_constant<int, 4>{}); break;
                    case 8: go(std::integral_constant<int, 8>{}); break;
                    case 12: go(std::integral_constant<int, 12>{}); break;
                    default: go(std::integral_constant<int, 16>{}); break;
                }
            } else if (p.K & 3) {
                return RSLRL_E_UNSUPPORTED;  // the MFMA variant reads whole float4 rows of dZ
            } else {
                auto go = [&](auto nr) {
                    constexpr int NR = decltype(nr)::value;
                    if (fullm) hipLaunchKernelGGL((mlp_gemm_x6_kernel<EPI, true, 2, NR>), g, b, 0, st, p, img);
                    else hipLaunchKernelGGL((mlp_gemm_x6_kernel<EPI, false, 2, NR>), g, b, 0, st, p, img);
                };
                switch (p.K) {
                    case 4: go(std::integral_constant<int, 4>{}); break;
                    case 8: go(std::integral_constant<int, 8>{}); break;
                    case 12: go(std::integral_constant<int, 12>{}); break;
                    default: go(std::integral_constant<int, 16>{}); break;
                }
            }
        } else if constexpr (EPI == kEpiBiasEluOut) {
            auto go = [&](auto nr) {  // NR 1: VALU output layer (nout <= 4), 4: MFMA output layer
                constexpr int NR = decltype(nr)::value;
                if (out_fwd_occupancy() == 2) {
                    if (fullm) hipLaunchKernelGGL((mlp_gemm_x6_kernel<EPI, true, 2, NR, PL>), g, b, 0, st, p, img);
                    else hipLaunchKernelGGL((mlp_gemm_x6_kernel<EPI, false, 2, NR, PL>), g, b, 0, st, p, img);
                } else {
                    if (fullm) hipLaunchKernelGGL((mlp_gemm_x6_kernel<EPI, true, 4, NR, PL>), g, b, 0, st, p, img);
                    else hipLaunchKernelGGL((mlp_gemm_x6_kernel<EPI, false, 4, NR, PL>), g, b, 0, st, p, img);
                }
            };
            if (p.nout <= 4) go(std::integral_constant<int, 1>{});
            else go(std::integral_constant<int, 4>{});
        } else if (short_k) {
            if (fullm) hipLaunchKernelGGL((mlp_gemm_x6_kernel<EPI, true, 2, 4, PL>), g, b, 0, st, p, img);
            else hipLaunchKernelGGL((mlp_gemm_x6_kernel<EPI, false, 2, 4, PL>), g, b, 0, st, p, img);
        } else if (k48_deep<EPI>(p, fullm, PL)) {
            if constexpr (PL == 3 && (EPI == kEpiBias || EPI == kEpiBiasElu))
                hipLaunchKernelGGL((mlp_gemm_x6_kernel<EPI, true, 4, 4, PL, 3>), g, b, 0, st, p, img);
        } else if (PL != 3 || !launch_x6s<EPI>(p, img, fullm, g, st)) {
            if (fullm) hipLaunchKernelGGL((mlp_gemm_x6_kernel<EPI, true, 4, 4, PL>), g, b, 0, st, p, img);
            else hipLaunchKernelGGL((mlp_gemm_x6_kernel<EPI, false, 4, 4, PL>), g, b, 0, st, p, img);
        }
    } else if constexpr (EPI == kEpiEluGradWgrad || EPI == kEpiBiasEluOut) {
        return RSLRL_E_UNSUPPORTED;  // x6 path only
    } else if (EPI == kEpiEluGrad && dgrad_occupancy() == 2) {
        hipLaunchKernelGGL((mlp_gemm_kernel<EPI, 2>), g, b, 0, st, p);
    } else {
        hipLaunchKernelGGL((mlp_gemm_kernel<EPI, 4>), g, b, 0, st, p);
    }
    return launch_status();
}

}  // namespace
}  // namespace rslrl

using namespace rslrl;

extern "C" int64_t rslrl_linear_tiles(int64_t M) { return ceil_div(M, kBM); }

extern "C" size_t rslrl_linear_bimage_bytes(int32_t depth) {
    return depth < 1 ? 0 : static_cast<size_t>(ceil_div(static_cast<int64_t>(depth), kKC)) * kX6ChunkB;
}

extern "C" size_t rslrl_linear_bimage_h3_bytes(int32_t depth) {
    return depth < 1 ? 0 : static_cast<size_t>(h3_image_scales_offset(depth)) + kBN * sizeof(float);
}

extern "C" int rslrl_linear_prepare_bimages(const rslrl_bimage_desc_t* descs, int32_t n, rslrl_stream_t stream) {
    if (!descs || n < 1 || n > kMaxImages) return RSLRL_E_INVALID_ARGUMENT;
    BImageBatch batch{};
    int max_chunks = 0;
    int max_threads = 0;
    for (int i = 0; i < n; ++i) {
        const rslrl_bimage_desc_t& d = descs[i];
        if (!d.src || !d.image || d.rows < 1 || d.rows > kBN || d.depth < 1 || d.depth > (1 << 24))
            return RSLRL_E_INVALID_ARGUMENT;
        if (reinterpret_cast<uintptr_t>(d.image) & 15) return RSLRL_E_MISALIGNED;
        if (d.layout == RSLRL_BIMAGE_LAYOUT_OUT) {
            if (d.rows > kMaxOutWidth || d.depth > kBN || d.transposed) return RSLRL_E_INVALID_ARGUMENT;
            max_threads = std::max(max_threads, kOutImageThreads);
        } else if (d.layout == RSLRL_BIMAGE_LAYOUT_H3) {
            if (d.depth > kBN) return RSLRL_E_INVALID_ARGUMENT;
            max_threads = std::max(max_threads, kBN * 32);
        } else if (d.layout == RSLRL_BIMAGE_LAYOUT_GEMM) {
            max_chunks = std::max(max_chunks, static_cast<int>(ceil_div(static_cast<int64_t>(d.depth), kKC)));
        } else {
            return RSLRL_E_INVALID_ARGUMENT;
        }
        batch.d[i] = d;
    }
    max_threads = std::max(max_threads, max_chunks * kBN * 2);
    const dim3 grid(static_cast<unsigned>(ceil_div(max_threads, kBlock)), static_cast<unsigned>(n));
    hipLaunchKernelGGL(bimage_kernel, grid, dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream), batch);
    return launch_status();
}

extern "C" int rslrl_linear_prepare_bimage(const float* src, int32_t rows, int32_t depth, int32_t transposed,
                                           void* image, rslrl_stream_t stream) {
    const rslrl_bimage_desc_t d{src, image, rows, depth, transposed ? 1 : 0, RSLRL_BIMAGE_LAYOUT_GEMM};
    return rslrl_linear_prepare_bimages(&d, 1, stream);
}

extern "C" int rslrl_linear_fwd(const float* x, int64_t M, int32_t K, const float* weight, int32_t N,
                                const float* bias, int32_t activation, float* y, const void* bimage,
                                rslrl_stream_t stream) {
    if (M < 0 || K < 1 || N < 1 || N > kBN || (K & 3) || K > INT32_MAX / 2) return RSLRL_E_INVALID_ARGUMENT;
    if (M == 0) return RSLRL_OK;
    if (!x || (!weight && !bimage) || !bias || !y) return RSLRL_E_INVALID_ARGUMENT;
    if (!aligned16(x) || (!bimage && !aligned16(weight)) || (bimage && !aligned16(bimage))) return RSLRL_E_MISALIGNED;
    if (activation != 0 && activation != 1) return RSLRL_E_UNSUPPORTED;
    GemmParams p{x, weight, bias, nullptr, y, nullptr, M, K, N, 0, nullptr};
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    return activation ? launch<kEpiBiasElu>(p, bimage, st) : launch<kEpiBias>(p, bimage, st);
}

extern "C" int rslrl_linear_dgrad_elu(const float* dz, int64_t M, int32_t Nred, const float* weight_t, int32_t K,
                                      const float* h, float* dz_prev, float* colsum_partials, const void* bimage,
                                      rslrl_stream_t stream) {
    if (M < 0 || Nred < 1 || K < 1 || K > kBN || (Nred & 3)) return RSLRL_E_INVALID_ARGUMENT;
    if (M == 0) return RSLRL_OK;
    if (!dz || (!weight_t && !bimage) || !h || !dz_prev || !colsum_partials) return RSLRL_E_INVALID_ARGUMENT;
    if (!aligned16(dz) || (!bimage && !aligned16(weight_t)) || (bimage && !aligned16(bimage))) return RSLRL_E_MISALIGNED;
    // GEMM view: A = dZ [M, Nred], Bw = W^T [K, Nred] -> C = dZ W [M, K]
    GemmParams p{dz, weight_t, nullptr, h, dz_prev, colsum_partials, M, Nred, K, ceil_div(M, kBM), nullptr};
    return launch<kEpiEluGrad>(p, bimage, reinterpret_cast<hipStream_t>(stream));
}

extern "C" size_t rslrl_linear_dgrad_wgrad_partial_bytes(int64_t M, int32_t Nred, int32_t K) {
    if (M < 1 || Nred < 1 || K < 1) return 0;
    return static_cast<size_t>(ceil_div(M, kBM)) * static_cast<size_t>(dgrad_wgrad_tile_floats(Nred, K)) * sizeof(float);
}

extern "C" int rslrl_linear_dgrad_elu_wgrad(const float* dz, int64_t M, int32_t Nred, int32_t K, const float* h,
                                            float* dz_prev, float* colsum_partials, const void* bimage,
                                            float* wgrad_partials, rslrl_stream_t stream) {
    if (M < 0 || Nred < 1 || Nred > kMaxWgradRows || K < 1 || K > kBN) return RSLRL_E_INVALID_ARGUMENT;
    if (M == 0) return RSLRL_OK;
    if (!dz || !h || !dz_prev || !colsum_partials || !bimage || !wgrad_partials) return RSLRL_E_INVALID_ARGUMENT;
    if (!aligned16(dz) || !aligned16(bimage)) return RSLRL_E_MISALIGNED;
    GemmParams p{dz, nullptr, nullptr, h, dz_prev, colsum_partials, M, Nred, K, ceil_div(M, kBM), wgrad_partials};
    return launch<kEpiEluGradWgrad>(p, bimage, reinterpret_cast<hipStream_t>(stream));
}

extern "C" size_t rslrl_linear_out_image_bytes(void) { return static_cast<size_t>(kOutImageUnits) * 16; }

extern "C" int rslrl_linear_fwd_out(const float* x, int64_t M, int32_t K, const float* bias, int32_t N,
                                    const void* bimage, float* h_out, const float* out_bias, int32_t Nout,
                                    const void* out_image, float* y, rslrl_stream_t stream) {
    if (M < 0 || K < 1 || N < 1 || N > kBN || (K & 3) || (N & 3) || K > INT32_MAX / 2) return RSLRL_E_INVALID_ARGUMENT;
    if (Nout < 1 || Nout > kMaxOutWidth) return RSLRL_E_INVALID_ARGUMENT;
    if (M == 0) return RSLRL_OK;
    if (!x || !bias || !bimage || !out_bias || !out_image || !y) return RSLRL_E_INVALID_ARGUMENT;
    if (!aligned16(x) || !aligned16(bias) || !aligned16(bimage) || !aligned16(out_image) || (h_out && !aligned16(h_out)))
        return RSLRL_E_MISALIGNED;
    GemmParams p{x, nullptr, bias, nullptr, h_out, nullptr, M, K, N, 0, nullptr,
                 static_cast<const uint4*>(out_image), out_bias, y, Nout, out_fwd_nt()};
    return launch<kEpiBiasEluOut>(p, bimage, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int rslrl_column_sum_fold(float* partials, int64_t tiles, int32_t N, float* out,
                                     rslrl_stream_t stream) {
    if (tiles < 1 || tiles > INT32_MAX || N < 1 || !partials || !out) return RSLRL_E_INVALID_ARGUMENT;
    const int per = static_cast<int>(ceil_div(tiles, kFoldSlices));
    const int slices = static_cast<int>(ceil_div(tiles, per));
    const unsigned cg = static_cast<unsigned>(ceil_div(N, kFoldCols));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(colsum_slice_kernel, dim3(cg, static_cast<unsigned>(slices)), dim3(kBlock), 0, st, partials,
                       static_cast<int>(tiles), N, per);
    hipLaunchKernelGGL(colsum_fold_kernel, dim3(cg), dim3(kBlock), 0, st, partials, slices, N, per, out);
    return launch_status();
}

extern "C" size_t rslrl_amax_workspace_bytes(void) { return 1024; }

namespace {
// RSLRL_H3_DEEP = bit mask over ops (1 << RSLRL_LINEAR_*) taking the look-ahead main loop; read per call
// (A/B measurements in one process)
int h3_deep(int op) {
    const char* e = std::getenv("RSLRL_H3_DEEP");
    const int mask = e ? std::atoi(e) : kH3DeepDefault;
    return (mask >> op) & 1;
}
}  // namespace

// One entry point for every fused linear op in either split arithmetic, with the h3 operand scales
// (include/rslrl_amd.h rslrl_linear_args_t).
extern "C" int rslrl_linear_gemm(const rslrl_linear_args_t* a, rslrl_stream_t stream) {
    if (!a) return RSLRL_E_INVALID_ARGUMENT;
    const int op = a->op;
    const bool h3 = a->arith == RSLRL_ARITH_H3;
    if (!h3 && a->arith != RSLRL_ARITH_X6) return RSLRL_E_INVALID_ARGUMENT;
    // K % 4 == 0, except the output-layer backward's reduction width (Nred 1..16, dZ rows read as they are)
    if (a->M < 0 || a->K < 1 || a->N < 1 || a->N > kBN || ((a->K & 3) && op != RSLRL_LINEAR_DGRAD_ELU_WGRAD) ||
        a->K > INT32_MAX / 2)
        return RSLRL_E_INVALID_ARGUMENT;
    if (a->M == 0) return RSLRL_OK;
    if (!a->a || !a->bimage || (h3 && !a->a_amax)) return RSLRL_E_INVALID_ARGUMENT;
    if (a->amax_out && !a->amax_workspace) return RSLRL_E_INVALID_ARGUMENT;
    if (!aligned16(a->a) || !aligned16(a->bimage)) return RSLRL_E_MISALIGNED;
    if (a->amax_out && op == RSLRL_LINEAR_FWD_OUT) return RSLRL_E_UNSUPPORTED;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    GemmParams p{};
    p.a = a->a;
    p.M = a->M;
    p.K = a->K;
    p.N = a->N;
    p.a_amax = a->a_amax;
    p.amax_out = a->amax_out;
    p.amax_ws = static_cast<unsigned*>(a->amax_workspace);
    p.deep = h3_deep(op);
    switch (op) {
        case RSLRL_LINEAR_FWD:
        case RSLRL_LINEAR_FWD_ELU:
            if (!a->bias || !a->c) return RSLRL_E_INVALID_ARGUMENT;
            p.bias = a->bias;
            p.c = a->c;
            if (op == RSLRL_LINEAR_FWD_ELU)
                return h3 ? launch<kEpiBiasElu, 2>(p, a->bimage, st) : launch<kEpiBiasElu, 3>(p, a->bimage, st);
            return h3 ? launch<kEpiBias, 2>(p, a->bimage, st) : launch<kEpiBias, 3>(p, a->bimage, st);
        case RSLRL_LINEAR_DGRAD_ELU:
            if (!a->h || !a->c) return RSLRL_E_INVALID_ARGUMENT;  // colsum_partials optional
            p.h = a->h;
            p.c = a->c;
            p.colsum = a->colsum_partials;
            p.ctiles = ceil_div(a->M, kBM);
            return h3 ? launch<kEpiEluGrad, 2>(p, a->bimage, st) : launch<kEpiEluGrad, 3>(p, a->bimage, st);
        case RSLRL_LINEAR_DGRAD_ELU_WGRAD:
            if (h3) return RSLRL_E_UNSUPPORTED;
            if (a->K > kMaxWgradRows || !a->h || !a->c || !a->wgrad_partials)  // colsum_partials optional
                return RSLRL_E_INVALID_ARGUMENT;
            p.h = a->h;
            p.c = a->c;
            p.colsum = a->colsum_partials;
            p.ctiles = ceil_div(a->M, kBM);
            p.wpart = a->wgrad_partials;
            return launch<kEpiEluGradWgrad, 3>(p, a->bimage, st);
        case RSLRL_LINEAR_FWD_OUT:
            if ((a->N & 3) || a->nout < 1 || a->nout > kMaxOutWidth || !a->bias || !a->out_bias || !a->out_image ||
                !a->y)
                return RSLRL_E_INVALID_ARGUMENT;
            if (!aligned16(a->bias) || !aligned16(a->out_image) || (a->c && !aligned16(a->c))) return RSLRL_E_MISALIGNED;
            p.bias = a->bias;
            p.c = a->c;
            p.oimg = static_cast<const uint4*>(a->out_image);
            p.obias = a->out_bias;
            p.y = a->y;
            p.nout = a->nout;
            p.nt = out_fwd_nt();
            return h3 ? launch<kEpiBiasEluOut, 2>(p, a->bimage, st) : launch<kEpiBiasEluOut, 3>(p, a->bimage, st);
        default:
            return RSLRL_E_INVALID_ARGUMENT;
    }
}

namespace {
// validated GemmParams of a forward op (rslrl_linear_gemm's checks for RSLRL_LINEAR_FWD[_ELU])
int fwd_params(const rslrl_linear_args_t* a, GemmParams& p) {
    const bool h3 = a->arith == RSLRL_ARITH_H3;
    if (!h3 && a->arith != RSLRL_ARITH_X6) return RSLRL_E_INVALID_ARGUMENT;
    if (a->M < 0 || a->K < 1 || a->N < 1 || a->N > kBN || (a->K & 3) || a->K > INT32_MAX / 2)
        return RSLRL_E_INVALID_ARGUMENT;
    if (!a->a || !a->bimage || (h3 && !a->a_amax) || !a->bias || !a->c) return RSLRL_E_INVALID_ARGUMENT;
    if (a->amax_out && !a->amax_workspace) return RSLRL_E_INVALID_ARGUMENT;
    if (!aligned16(a->a) || !aligned16(a->bimage)) return RSLRL_E_MISALIGNED;
    p = GemmParams{};
    p.a = a->a;
    p.M = a->M;
    p.K = a->K;
    p.N = a->N;
    p.a_amax = a->a_amax;
    p.amax_out = a->amax_out;
    p.amax_ws = static_cast<unsigned*>(a->amax_workspace);
    p.deep = h3_deep(a->op);
    p.bias = a->bias;
    p.c = a->c;
    return RSLRL_OK;
}

// ---- "w4": the same x6 GEMM with 4 waves per workgroup side by side (1 x 4), each 128 x 64 = 4 x 2 MFMA tiles, on
// the 128 x 256 tile: a B fragment feeds 4 MFMAs and an A fragment 2 (0.375 ds_read_b128 per MFMA instead of 0.5),
// two workgroups per CU at <= 256 registers (2 waves per SIMD).  Full tiles, x6, K = 256, no column sums or amax
// (the paired update's hidden forward and input gradient); RSLRL_W4 selects it (A/B).
constexpr int kThreadsW4 = 256;
#ifndef RSLRL_W4_DEPTH
#define RSLRL_W4_DEPTH 2
#endif
constexpr int kW4Depth = RSLRL_W4_DEPTH;  // A look-ahead (chunks): the 256-register budget has room for 2

template <int EPI>
__device__ __forceinline__ void mlp_gemm_x6_w4_body(const GemmParams& p, const uint4* __restrict__ bimg, char* lds_b0,
                                                    char* lds_b1) {
    constexpr int BM = kBM, PL = 3, I = 4;
    constexpr int planeA = BM * kX6RowB;
    using Frag = typename Arith<PL>::frag;
    char* lds[2];
    lds[0] = lds_b0;
    lds[1] = lds_b1;
    const int lane = threadIdx.x & 63;
    const int wn = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // cols wn * 64
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * BM;
    f32x16 acc[I][2];
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
    auto compute = [&](const char* a_lds, const char* b_lds) {
        Frag bf[2][PL];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < PL; ++q) bf[j][q] = read_frag<Frag>(b_lds + q * kX6PlaneB, wn * 64 + j * 32 + l32, h);
#pragma unroll
        for (int i = 0; i < I; ++i) {
            Frag af[PL];
#pragma unroll
            for (int q = 0; q < PL; ++q) af[q] = read_frag<Frag>(a_lds + q * planeA, i * 32 + l32, h);
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = Arith<PL>::mfma(af, bf[j], acc[i][j]);
        }
    };
    deep_pipeline<BM, PL, 16, kW4Depth, decltype(compute)&, NoHook, kThreadsW4>(p, row0, bimg, lds, 1.f, compute);
    if constexpr (kStagedEpi) {  // after deep_pipeline's final barrier no wave reads the LDS buffers any more
        epilogue_tiles_staged<EPI, I, 2>(p, acc, row0, wn * 64, reinterpret_cast<float*>(lds_b0) + wn * 1024);
    } else {
        float colpart[2];
        float amx = 0.f;
        epilogue_tiles<EPI, I, 2>(p, acc, row0, wn * 64, true, colpart, amx);
    }
}

template <int EPI>
__global__ __launch_bounds__(kThreadsW4, 2) void mlp_gemm_x6_w4_pair_kernel(GemmPair b) {
    __shared__ __attribute__((aligned(16))) char lds_b0[x6_buf_bytes<EPI, 3>()];
    __shared__ __attribute__((aligned(16))) char lds_b1[x6_buf_bytes<EPI, 3>()];
    mlp_gemm_x6_w4_body<EPI>(b.p[blockIdx.y], b.img[blockIdx.y], lds_b0, lds_b1);
}

// ---- "w8": 256 x 256 tiles, 8 waves as 2 (M) x 4 (N) of the w4 wave tile (128 x 64), one workgroup per CU at <= 256
// registers.  Each B-image chunk is staged once per 256 rows instead of once per 128: the image (384 KiB per tile, from
// L2) is the kernels' largest stream -- at 128-row tiles 2.36 GB per input-gradient pair launch against 2.4 GB of HBM
// traffic, 2.4 M of the launch's 6.3 M vector-memory instructions (SQ counters, profiles/r4_mlp_pmc_base.json).
constexpr int kBMW8 = 256;
#ifndef RSLRL_W8_DEPTH
#define RSLRL_W8_DEPTH 2
#endif
constexpr int kW8Depth = RSLRL_W8_DEPTH;  // A look-ahead (chunks)

template <int EPI>
__device__ __forceinline__ void mlp_gemm_x6_w8_body(const GemmParams& p, const uint4* __restrict__ bimg, char* lds_b0,
                                                    char* lds_b1) {
    constexpr int BM = kBMW8, PL = 3, I = 4;
    constexpr int planeA = BM * kX6RowB;
    using Frag = typename Arith<PL>::frag;
    char* lds[2];
    lds[0] = lds_b0;
    lds[1] = lds_b1;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 2;  // rows wm * 128
    const int wn = wave & 3;   // cols wn * 64
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * BM;
    f32x16 acc[I][2];
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
    auto compute = [&](const char* a_lds, const char* b_lds) {
        Frag bf[2][PL];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < PL; ++q) bf[j][q] = read_frag<Frag>(b_lds + q * kX6PlaneB, wn * 64 + j * 32 + l32, h);
#pragma unroll
        for (int i = 0; i < I; ++i) {
            Frag af[PL];
#pragma unroll
            for (int q = 0; q < PL; ++q) af[q] = read_frag<Frag>(a_lds + q * planeA, wm * 128 + i * 32 + l32, h);
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = Arith<PL>::mfma(af, bf[j], acc[i][j]);
        }
    };
    deep_pipeline<BM, PL, 16, kW8Depth, decltype(compute)&, NoHook, kThreads>(p, row0, bimg, lds, 1.f, compute);
    if constexpr (kStagedEpi) {
        epilogue_tiles_staged<EPI, I, 2>(p, acc, row0 + wm * 128, wn * 64, reinterpret_cast<float*>(lds_b0) + wave * 1024);
    } else {
        float colpart[2];
        float amx = 0.f;
        epilogue_tiles<EPI, I, 2>(p, acc, row0 + wm * 128, wn * 64, true, colpart, amx);
    }
}

template <int EPI>
__global__ __launch_bounds__(kThreads, 2) void mlp_gemm_x6_w8_pair_kernel(GemmPair b) {
    constexpr int bytes = 3 * kBMW8 * kX6RowB + 3 * kX6PlaneB;
    __shared__ __attribute__((aligned(16))) char lds_b0[bytes];
    __shared__ __attribute__((aligned(16))) char lds_b1[bytes];
    mlp_gemm_x6_w8_body<EPI>(b.p[blockIdx.y], b.img[blockIdx.y], lds_b0, lds_b1);
}

// RSLRL_W4 (read per call: A/B in one process): 1 = every eligible launch, 0 = none; unset = the input gradient at
// >= 2048 tiles per problem (measured, scripts/w4_probe.py: dgrad pair at 393,216 rows 669 -> 642 us; the hidden
// forward 607 -> 617 us and both equal within noise at 98,304 rows)
bool w4_enabled(int epi, int64_t tiles) {
    const char* e = std::getenv("RSLRL_W4");
    if (e && e[0] == '1') return true;
    if (e && e[0] == '0') return false;
    return epi == kEpiEluGrad && tiles >= 2048;
}

// RSLRL_W8 (read per call): 1 = the 256-row tiles for every eligible launch (M % 256 == 0), 0 = none (default)
bool w8_enabled(int epi, int64_t M) {
    (void)epi;
    const char* e = std::getenv("RSLRL_W8");
    return e && e[0] == '1' && M % kBMW8 == 0;
}

template <int EPI, int PL>
int launch_pair(const GemmPair& b, bool fullm, hipStream_t st) {
    const int64_t tiles = ceil_div(b.p[0].M, kBM);
    if (tiles > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
    const dim3 g(static_cast<unsigned>(tiles), 2), blk(kThreads);
    if constexpr (PL == 3 && (EPI == kEpiBias || EPI == kEpiBiasElu)) {
        if (k48_deep<EPI>(b.p[0], fullm, PL)) {  // both problems share the shape and the op
            hipLaunchKernelGGL((mlp_gemm_x6_pair_kernel<EPI, true, PL, 3>), g, blk, 0, st, b);
            return launch_status();
        }
    }
    if constexpr (PL == 3 && (EPI == kEpiBiasElu || EPI == kEpiEluGrad)) {
        const bool plain = b.p[0].colsum == nullptr && b.p[1].colsum == nullptr && b.p[0].amax_out == nullptr &&
                           b.p[1].amax_out == nullptr;
        if (w8_enabled(EPI, b.p[0].M) && plain && b.p[0].K == 16 * kKC && b.p[0].N == kBN && b.p[0].deep) {
            hipLaunchKernelGGL((mlp_gemm_x6_w8_pair_kernel<EPI>), dim3(static_cast<unsigned>(b.p[0].M / kBMW8), 2),
                               dim3(kThreads), 0, st, b);
            return launch_status();
        }
        if (w4_enabled(EPI, tiles) && fullm && plain && b.p[0].K == 16 * kKC && b.p[0].N == kBN && b.p[0].deep) {
            hipLaunchKernelGGL((mlp_gemm_x6_w4_pair_kernel<EPI>), g, dim3(kThreadsW4), 0, st, b);
            return launch_status();
        }
    }
    if constexpr (EPI == kEpiEluGrad) {  // the input gradient stages its first H block like the single launch
        if (fullm) hipLaunchKernelGGL((mlp_gemm_x6_pair_kernel<EPI, true, PL, 0, true>), g, blk, 0, st, b);
        else hipLaunchKernelGGL((mlp_gemm_x6_pair_kernel<EPI, false, PL, 0, true>), g, blk, 0, st, b);
        return launch_status();
    }
    if (fullm) hipLaunchKernelGGL((mlp_gemm_x6_pair_kernel<EPI, true, PL>), g, blk, 0, st, b);
    else hipLaunchKernelGGL((mlp_gemm_x6_pair_kernel<EPI, false, PL>), g, blk, 0, st, b);
    return launch_status();
}

// validated GemmParams of a fused output-layer forward (rslrl_linear_gemm's checks for RSLRL_LINEAR_FWD_OUT)
int out_params(const rslrl_linear_args_t* a, GemmParams& p) {
    const bool h3 = a->arith == RSLRL_ARITH_H3;
    if (!h3 && a->arith != RSLRL_ARITH_X6) return RSLRL_E_INVALID_ARGUMENT;
    if (a->M < 0 || a->K < 1 || a->N < 1 || a->N > kBN || (a->K & 3) || (a->N & 3) || a->K > INT32_MAX / 2)
        return RSLRL_E_INVALID_ARGUMENT;
    if (!a->a || !a->bimage || (h3 && !a->a_amax)) return RSLRL_E_INVALID_ARGUMENT;
    if (a->nout < 1 || a->nout > kMaxOutWidth || !a->bias || !a->out_bias || !a->out_image || !a->y)
        return RSLRL_E_INVALID_ARGUMENT;
    if (a->amax_out) return RSLRL_E_UNSUPPORTED;
    if (!aligned16(a->a) || !aligned16(a->bimage) || !aligned16(a->bias) || !aligned16(a->out_image) ||
        (a->c && !aligned16(a->c)))
        return RSLRL_E_MISALIGNED;
    p = GemmParams{};
    p.a = a->a;
    p.M = a->M;
    p.K = a->K;
    p.N = a->N;
    p.a_amax = a->a_amax;
    p.deep = h3_deep(RSLRL_LINEAR_FWD_OUT);
    p.bias = a->bias;
    p.c = a->c;
    p.oimg = static_cast<const uint4*>(a->out_image);
    p.obias = a->out_bias;
    p.y = a->y;
    p.nout = a->nout;
    p.nt = out_fwd_nt();
    return RSLRL_OK;
}

// (MINW 2: both epilogues in one kernel do not fit 128 registers without spills; the pair is only taken when its
// tiles are at most one per CU, where the occupancy limit costs nothing)
template <bool FULL, int NR0>
void launch_out_pair(const GemmPair& b, int nr1, dim3 g, hipStream_t st) {
    if (nr1 == 1) hipLaunchKernelGGL((mlp_gemm_x6_out_pair_kernel<FULL, 2, NR0, 1, 3>), g, dim3(kThreads), 0, st, b);
    else hipLaunchKernelGGL((mlp_gemm_x6_out_pair_kernel<FULL, 2, NR0, 4, 3>), g, dim3(kThreads), 0, st, b);
}

// validated GemmParams of a fused output-layer backward (rslrl_linear_gemm's checks for RSLRL_LINEAR_DGRAD_ELU_WGRAD)
int dgrad_wgrad_params(const rslrl_linear_args_t* a, GemmParams& p) {
    if (a->arith != RSLRL_ARITH_X6) return RSLRL_E_UNSUPPORTED;
    if (a->M < 0 || a->K < 1 || a->K > kMaxWgradRows || a->N < 1 || a->N > kBN) return RSLRL_E_INVALID_ARGUMENT;
    if (!a->a || !a->bimage || !a->h || !a->c || !a->wgrad_partials) return RSLRL_E_INVALID_ARGUMENT;
    if (a->amax_out && !a->amax_workspace) return RSLRL_E_INVALID_ARGUMENT;
    if (!aligned16(a->a) || !aligned16(a->bimage)) return RSLRL_E_MISALIGNED;
    p = GemmParams{};
    p.a = a->a;
    p.M = a->M;
    p.K = a->K;
    p.N = a->N;
    p.amax_out = a->amax_out;
    p.amax_ws = static_cast<unsigned*>(a->amax_workspace);
    p.h = a->h;
    p.c = a->c;
    p.colsum = a->colsum_partials;
    p.ctiles = ceil_div(a->M, kBM);
    p.wpart = a->wgrad_partials;
    return RSLRL_OK;
}

template <int NR0, int NR1>
void launch_out_bwd_pair(const GemmPair& b, dim3 g, hipStream_t st) {
    constexpr int C0 = NR0 <= 4 ? 4 : 2, C1 = NR1 <= 4 ? 4 : 2;
    hipLaunchKernelGGL((out_bwd_valu_pair_kernel<NR0, C0, NR1, C1>), g, dim3(kOutBwdThreads), 0, st, b);
}

// (one of the two reductions <= 4 wide -- the value head -- the other any of 4 / 8 / 12 / 16)
bool out_bwd_pair_dispatch(const GemmPair& b, int nr0, int nr1, dim3 g, hipStream_t st) {
    auto other = [&](int nr, auto small_first) {
        constexpr bool F = decltype(small_first)::value;
        switch (nr) {
            case 4: launch_out_bwd_pair<4, 4>(b, g, st); return true;
            case 8: F ? launch_out_bwd_pair<4, 8>(b, g, st) : launch_out_bwd_pair<8, 4>(b, g, st); return true;
            case 12: F ? launch_out_bwd_pair<4, 12>(b, g, st) : launch_out_bwd_pair<12, 4>(b, g, st); return true;
            case 16: F ? launch_out_bwd_pair<4, 16>(b, g, st) : launch_out_bwd_pair<16, 4>(b, g, st); return true;
            default: return false;
        }
    };
    if (nr1 == 4) return other(nr0, std::false_type{});
    if (nr0 == 4) return other(nr1, std::true_type{});
    return false;
}

// validated GemmParams of an input-gradient op (rslrl_linear_gemm's checks for RSLRL_LINEAR_DGRAD_ELU)
int dgrad_params(const rslrl_linear_args_t* a, GemmParams& p) {
    const bool h3 = a->arith == RSLRL_ARITH_H3;
    if (!h3 && a->arith != RSLRL_ARITH_X6) return RSLRL_E_INVALID_ARGUMENT;
    if (a->M < 0 || a->K < 1 || a->N < 1 || a->N > kBN || (a->K & 3) || a->K > INT32_MAX / 2)
        return RSLRL_E_INVALID_ARGUMENT;
    if (!a->a || !a->bimage || (h3 && !a->a_amax) || !a->h || !a->c) return RSLRL_E_INVALID_ARGUMENT;
    if (a->amax_out && !a->amax_workspace) return RSLRL_E_INVALID_ARGUMENT;
    if (!aligned16(a->a) || !aligned16(a->bimage)) return RSLRL_E_MISALIGNED;
    p = GemmParams{};
    p.a = a->a;
    p.M = a->M;
    p.K = a->K;
    p.N = a->N;
    p.a_amax = a->a_amax;
    p.amax_out = a->amax_out;
    p.amax_ws = static_cast<unsigned*>(a->amax_workspace);
    p.deep = h3_deep(RSLRL_LINEAR_DGRAD_ELU);
    p.h = a->h;
    p.c = a->c;
    p.colsum = a->colsum_partials;
    p.ctiles = ceil_div(a->M, kBM);
    return RSLRL_OK;
}
}  // namespace

// The critic's last hidden layer, value head, value-loss gradient and value-head backward in one launch
// (include/rslrl_amd.h).  Unsupported shapes return RSLRL_E_UNSUPPORTED before anything is launched (the caller
// then runs the separate launches).
extern "C" int rslrl_value_head_fwd_bwd(const rslrl_linear_args_t* a, const rslrl_value_head_args_t* v,
                                        rslrl_stream_t stream) {
    if (!a || !v || a->op != RSLRL_LINEAR_FWD_OUT) return RSLRL_E_INVALID_ARGUMENT;
    GemmParams p;
    const int rc = out_params(a, p);
    if (rc) return rc;
    if (a->arith != RSLRL_ARITH_X6 || a->nout != 1 || a->N != kBN || a->K != 16 * kKC || a->M % kBM != 0 || !p.deep)
        return RSLRL_E_UNSUPPORTED;
    if (!a->c || !v->target_values || !v->returns || !v->out_weight || !v->wgrad_partials)
        return RSLRL_E_INVALID_ARGUMENT;
    if (!aligned16(v->out_weight)) return RSLRL_E_MISALIGNED;
    p.vh_tv = v->target_values;
    p.vh_ret = v->returns;
    p.vh_w = v->out_weight;
    p.vh_clip = v->clip_param;
    p.vh_g = v->value_loss_coef / static_cast<float>(a->M);  // the loss kernel's g_value (ppo_loss.hip)
    p.vh_clipped = v->use_clipped_value_loss ? 1 : 0;
    p.wpart = v->wgrad_partials;
    p.colsum = v->colsum_partials;
    if (a->M == 0) return RSLRL_OK;
    const int64_t tiles = ceil_div(a->M, kBM);
    if (tiles > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
    if (value_head_stream_enabled() && !v->colsum_partials) {  // opt-in: the streaming main loop (mlp_fwd_stream.hip)
        const ValueHeadStreamArgs s{p.a, a->bimage, p.bias, v->out_weight, p.obias, v->target_values, v->returns,
                                    a->c, p.y, v->wgrad_partials, p.vh_clip, p.vh_g, p.vh_clipped, a->M};
        return value_head_stream(s, reinterpret_cast<hipStream_t>(stream));
    }
    hipLaunchKernelGGL(mlp_gemm_x6_value_head_kernel, dim3(static_cast<unsigned>(tiles)), dim3(kThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), p, static_cast<const uint4*>(a->bimage));
    return launch_status();
}

extern "C" int64_t rslrl_value_head_partial_rows(int64_t M, int32_t with_colsum) {
    if (M <= 0) return 0;
    // the same dispatch as rslrl_value_head_fwd_bwd: the streaming form never takes colsum_partials
    return value_head_stream_enabled() && !with_colsum ? value_head_stream_rows(M) : ceil_div(M, kBM);
}

// The actor's last hidden layer, output layer, the PPO loss and the output layer's backward in one launch
// (include/rslrl_amd.h).  Unsupported shapes return RSLRL_E_UNSUPPORTED before anything is launched.
extern "C" size_t rslrl_actor_head_workspace_bytes(int64_t M) {
    const int64_t tiles = ceil_div(M > 0 ? M : 0, kBM);
    const int64_t groups = ceil_div(tiles, kFoldGroup);  // >= the groups of 128 a larger grid folds in
    return 1024 + sizeof(double) * static_cast<size_t>(kActCols * (tiles + groups));
}

extern "C" int rslrl_actor_head_fwd_bwd(const rslrl_linear_args_t* a, const rslrl_actor_head_args_t* h,
                                        void* workspace, size_t workspace_bytes, rslrl_stream_t stream) {
    if (!a || !h || a->op != RSLRL_LINEAR_FWD_OUT) return RSLRL_E_INVALID_ARGUMENT;
    GemmParams p;
    const int rc = out_params(a, p);
    if (rc) return rc;
    const int64_t tiles = ceil_div(a->M, kBM);
    if (a->arith != RSLRL_ARITH_X6 || a->nout != kActA || h->num_actions != kActA || a->N != kBN ||
        a->K != 16 * kKC || a->M % kBM != 0 || a->M < 1 || !p.deep || tiles > int64_t{2 * kFoldGroup} * kFoldGroup)
        return RSLRL_E_UNSUPPORTED;
    if (!a->c || !h->actions || !h->old_log_prob || !h->advantages || !h->values || !h->target_values ||
        !h->returns || !h->old_mu || !h->old_sigma || !h->sigma || !h->out_weight_t_image || !h->wgrad_partials ||
        !h->grad_sigma || !h->stats || !workspace)
        return RSLRL_E_INVALID_ARGUMENT;
    if (!aligned16(a->c) || !aligned16(h->out_weight_t_image) || !aligned16(workspace)) return RSLRL_E_MISALIGNED;
    if (workspace_bytes < rslrl_actor_head_workspace_bytes(a->M)) return RSLRL_E_WORKSPACE_TOO_SMALL;
    ActorParams ap{};
    ap.actions = h->actions;
    ap.old_mu = h->old_mu;
    ap.old_sigma = h->old_sigma;
    ap.sigma = h->sigma;
    ap.old_logp = h->old_log_prob;
    ap.adv = h->advantages;
    ap.values = h->values;
    ap.target_values = h->target_values;
    ap.returns = h->returns;
    ap.w_t_img = static_cast<const uint4*>(h->out_weight_t_image);
    ap.wpart = h->wgrad_partials;
    ap.grad_sigma = h->grad_sigma;
    ap.stats = h->stats;
    ap.grad_mu = h->grad_mu;
    ap.tickets = static_cast<unsigned*>(workspace);
    ap.partials = reinterpret_cast<double*>(static_cast<char*>(workspace) + 1024);
    // the loss kernel's scalars (rslrl_ppo_loss_fwd_bwd)
    const float Bf = static_cast<float>(a->M);
    ap.clip = h->clip_param;
    ap.ratio_lo = static_cast<float>(1.0 - static_cast<double>(h->clip_param));
    ap.ratio_hi = static_cast<float>(1.0 + static_cast<double>(h->clip_param));
    ap.g_surr = 1.0f / Bf;
    ap.g_ent = -h->entropy_coef / Bf;
    ap.value_loss_coef = h->value_loss_coef;
    ap.entropy_coef = h->entropy_coef;
    ap.clipped_value = h->use_clipped_value_loss ? 1 : 0;
    ap.compute_kl = h->compute_kl ? 1 : 0;
    {  // RSLRL_KL_FAST=0 disables the per-action-constant KL (as in the loss kernel)
        const char* e = std::getenv("RSLRL_KL_FAST");
        ap.kl_fast = (e && e[0] == '0') ? 0 : 1;
    }
    if (tiles > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
    hipLaunchKernelGGL(mlp_gemm_x6_actor_head_kernel, dim3(static_cast<unsigned>(tiles)), dim3(kThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), p, static_cast<const uint4*>(a->bimage), ap);
    return launch_status();
}

// Two forward problems of one shape (op, arithmetic, M, K, N) in one launch -- e.g. the actor's and the
// critic's layer l in the rollout.  Each keeps its own operands, bias, output, amax and amax workspace.
extern "C" int rslrl_linear_gemm_pair(const rslrl_linear_args_t* a0, const rslrl_linear_args_t* a1,
                                      rslrl_stream_t stream) {
    if (!a0 || !a1) return RSLRL_E_INVALID_ARGUMENT;
    const int op = a0->op;
    if (a1->op != op || (op != RSLRL_LINEAR_FWD && op != RSLRL_LINEAR_FWD_ELU && op != RSLRL_LINEAR_DGRAD_ELU &&
                         op != RSLRL_LINEAR_FWD_OUT && op != RSLRL_LINEAR_DGRAD_ELU_WGRAD))
        return RSLRL_E_UNSUPPORTED;
    if (op == RSLRL_LINEAR_DGRAD_ELU_WGRAD) {  // reduction widths (K = Nred) may differ; VALU kernels only
        if (a0->M != a1->M || a0->N != a1->N) return RSLRL_E_INVALID_ARGUMENT;
        GemmPair b{};
        int rc = RSLRL_OK;
        for (int i = 0; i < 2 && rc == RSLRL_OK; ++i) {
            rc = dgrad_wgrad_params(i ? a1 : a0, b.p[i]);
            b.img[i] = static_cast<const uint4*>((i ? a1 : a0)->bimage);
        }
        if (rc == RSLRL_E_UNSUPPORTED || out_bwd_mode() != 0) {
            rc = rslrl_linear_gemm(a0, stream);
            return rc ? rc : rslrl_linear_gemm(a1, stream);
        }
        if (rc) return rc;
        if (a0->M == 0) return RSLRL_OK;
        const int64_t tiles = ceil_div(a0->M, kBM);
        if (tiles > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        if (!out_bwd_pair_dispatch(b, (a0->K + 3) / 4 * 4, (a1->K + 3) / 4 * 4, dim3(static_cast<unsigned>(tiles), 2),
                                   st)) {
            rc = rslrl_linear_gemm(a0, stream);
            return rc ? rc : rslrl_linear_gemm(a1, stream);
        }
        return launch_status();
    }
    if (op == RSLRL_LINEAR_FWD_OUT) {  // output widths may differ; x6 at the default occupancy, else two launches
        if (a0->arith != a1->arith || a0->M != a1->M || a0->K != a1->K || a0->N != a1->N) return RSLRL_E_INVALID_ARGUMENT;
        if (a0->arith != RSLRL_ARITH_X6 || x6_shape() == 16 || 2 * ceil_div(a0->M, kBM) > cu_count()) {
            const int rc = rslrl_linear_gemm(a0, stream);
            return rc ? rc : rslrl_linear_gemm(a1, stream);
        }
        GemmPair b{};
        for (int i = 0; i < 2; ++i) {
            const int rc = out_params(i ? a1 : a0, b.p[i]);
            if (rc) return rc;
            b.img[i] = static_cast<const uint4*>((i ? a1 : a0)->bimage);
        }
        if (a0->M == 0) return RSLRL_OK;
        const int64_t tiles = ceil_div(a0->M, kBM);
        if (tiles > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
        const dim3 g(static_cast<unsigned>(tiles), 2);
        const bool fullm = a0->M % kBM == 0 && a0->K % kKC == 0;
        const int nr0 = a0->nout <= 4 ? 1 : 4, nr1 = a1->nout <= 4 ? 1 : 4;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        if (fullm) {
            if (nr0 == 1) launch_out_pair<true, 1>(b, nr1, g, st);
            else launch_out_pair<true, 4>(b, nr1, g, st);
        } else {
            if (nr0 == 1) launch_out_pair<false, 1>(b, nr1, g, st);
            else launch_out_pair<false, 4>(b, nr1, g, st);
        }
        return launch_status();
    }
    if (a0->arith != a1->arith || a0->M != a1->M || a0->K != a1->K || a0->N != a1->N) return RSLRL_E_INVALID_ARGUMENT;
    if (a0->amax_out && a1->amax_out && a0->amax_workspace == a1->amax_workspace) return RSLRL_E_INVALID_ARGUMENT;
    const bool h3 = a0->arith == RSLRL_ARITH_H3;
    if (!h3 && x6_shape() == 16) {  // the opt-in 16x16x32 x6 forward has no pair kernel: two launches
        const int rc = rslrl_linear_gemm(a0, stream);
        return rc ? rc : rslrl_linear_gemm(a1, stream);
    }
    GemmPair b{};
    for (int i = 0; i < 2; ++i) {
        const int rc = op == RSLRL_LINEAR_DGRAD_ELU ? dgrad_params(i ? a1 : a0, b.p[i]) : fwd_params(i ? a1 : a0, b.p[i]);
        if (rc) return rc;
        b.img[i] = static_cast<const uint4*>((i ? a1 : a0)->bimage);
    }
    if (a0->M == 0) return RSLRL_OK;
    const bool fullm = a0->M % kBM == 0 && a0->K % kKC == 0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (op == RSLRL_LINEAR_DGRAD_ELU)
        return h3 ? launch_pair<kEpiEluGrad, 2>(b, fullm, st) : launch_pair<kEpiEluGrad, 3>(b, fullm, st);
    // streaming only where it measured faster (profiles/r5_fs_ab.json, medians of two processes each): M >= 196,608
    // (393,216: 688-695 vs 706-708 us; 196,608: 307 vs 325-327) and M <= 16,384 (37 vs 40 us; one tile per
    // workgroup); 65,536 and 98,304 rows stay tiled (106-108 vs 105-106, 155-157 vs 151-152)
    const int64_t ftiles = a0->M / kBM;
    const bool stream_m = ftiles >= 1536 || ftiles <= 128 || fwd_stream_forced();
    if (op == RSLRL_LINEAR_FWD_ELU && !h3 && fwd_stream_enabled() && stream_m &&
        (a0->K == kBN || (a0->K == 48 && fwd_stream48())) && a0->N == kBN && a0->M % kBM == 0 && !a0->amax_out &&
        !a1->amax_out) {
        // the square hidden layers: the streaming forward (mlp_fwd_stream.hip, same bits); the 48-wide first layer only
        // on request (RSLRL_FWD_STREAM=48): HBM-bound, it measured 222 vs 190-201 us on the tiled kernel's two
        // workgroups per CU (profiles/r5_fs_ab.json)
        const FwdStreamProblem fp[2] = {{b.p[0].a, b.img[0], b.p[0].bias, b.p[0].c},
                                        {b.p[1].a, b.img[1], b.p[1].bias, b.p[1].c}};
        return fwd_stream_pair(fp, 2, a0->M, a0->K, st);
    }
    if (op == RSLRL_LINEAR_FWD_ELU)
        return h3 ? launch_pair<kEpiBiasElu, 2>(b, fullm, st) : launch_pair<kEpiBiasElu, 3>(b, fullm, st);
    return h3 ? launch_pair<kEpiBias, 2>(b, fullm, st) : launch_pair<kEpiBias, 3>(b, fullm, st);
}
