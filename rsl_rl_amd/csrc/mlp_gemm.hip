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

#include <cstdlib>

#include "common.h"

namespace rslrl {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int kBM = 128;
constexpr int kBN = 256;
constexpr int kKC = 16;
constexpr int kPad = 2;
constexpr int kLd = kKC + kPad;  // LDS row stride (floats)
constexpr int kThreads = 512;

enum Epilogue { kEpiBias = 0, kEpiBiasElu = 1, kEpiEluGrad = 2 };

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

    // ---- epilogue: C/D map of the 32x32 tile: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).
    // Sub-tiles (i, j) are processed in order b = 2 i + j; for the ELU' epilogue the 16 h values of
    // sub-tile b + 1 are loaded before sub-tile b is finished, so no h load waits alone.
    float colpart[2] = {0.f, 0.f};
    const bool full = (row0 + kBM <= p.M) && (p.N == kBN);  // wave-uniform: no per-element bounds checks
    float hcur[16], hnext[16];
    auto load_h = [&](int b, float (&dst)[16]) {
        const int i = b >> 1, j = b & 1;
        const int col = wn * 64 + j * 32 + l32;
        const int64_t rbase = row0 + wm * 64 + i * 32 + 4 * h;
        const float* hp = p.h + rbase * p.N + col;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int roff = (r & 3) + 8 * (r >> 2);
            dst[r] = (full || (rbase + roff < p.M && col < p.N)) ? hp[static_cast<int64_t>(roff) * p.N] : 0.f;
        }
    };
    if constexpr (EPI == kEpiEluGrad) load_h(0, hcur);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int i = b >> 1, j = b & 1;
        if constexpr (EPI == kEpiEluGrad) {
            if (b + 1 < 4) load_h(b + 1, hnext);
        }
        const int col = wn * 64 + j * 32 + l32;
        const bool col_ok = col < p.N;
        float bias = 0.f;
        if constexpr (EPI != kEpiEluGrad) bias = col_ok ? p.bias[col] : 0.f;
        const int64_t rbase = row0 + wm * 64 + i * 32 + 4 * h;
        float* cp = p.c + rbase * p.N + col;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int roff = (r & 3) + 8 * (r >> 2);
            if (full || (rbase + roff < p.M && col_ok)) {
                float v = acc[i][j][r];
                if constexpr (EPI == kEpiBias) {
                    v = v + bias;
                } else if constexpr (EPI == kEpiBiasElu) {
                    v = v + bias;
                    v = v > 0.f ? v : expm1f(v);  // torch ELU, alpha = 1
                } else {
                    const float hv = hcur[r];  // ELU'(z) = 1 if z > 0 else hv + 1
                    v = hv > 0.f ? v : v * (hv + 1.f);
                    colpart[j] += v;
                }
                cp[static_cast<int64_t>(roff) * p.N] = v;
            }
        }
        if constexpr (EPI == kEpiEluGrad) {
#pragma unroll
            for (int r = 0; r < 16; ++r) hcur[r] = hnext[r];
        }
    }
    if constexpr (EPI == kEpiEluGrad) {
        // column sums over the tile's 128 rows: lanes l and l+32 hold the two row halves, the two wm waves
        // the two 64-row halves; fixed combine order -> deterministic
        __shared__ float colred[2][kBN];
        __syncthreads();  // the LDS tiles are no longer read
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float s = colpart[j] + __shfl_xor(colpart[j], 32, 64);
            if (h == 0) colred[wm][wn * 64 + j * 32 + l32] = s;
        }
        __syncthreads();
        // column-major partials [N][tiles]: the fold then reads each column contiguously
        for (int col = threadIdx.x; col < p.N && col < kBN; col += kThreads)
            p.colsum[static_cast<int64_t>(col) * gridDim.x + blockIdx.x] = colred[0][col] + colred[1][col];
    }
}

// Bias gradient: out[col] = sum over tiles of part[col][tiles] -- one workgroup per column, lanes stride
// over the tiles (coalesced), fp64 fold in a fixed order.
__global__ __launch_bounds__(kBlock) void colsum_fold_kernel(const float* __restrict__ part, int tiles,
                                                             float* __restrict__ out) {
    __shared__ double scratch[kBlock / kWave];
    const float* col = part + static_cast<int64_t>(blockIdx.x) * tiles;
    double s = 0.0;
    for (int t = threadIdx.x; t < tiles; t += kBlock) s += static_cast<double>(col[t]);
    s = block_sum(s, scratch);
    if (threadIdx.x == 0) out[blockIdx.x] = static_cast<float>(s);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int dgrad_occupancy() {  // tuning knob: RSLRL_DGRAD_OCC=2|4 (default 4)
    static const int v = [] {
        const char* e = std::getenv("RSLRL_DGRAD_OCC");
        return (e && std::atoi(e) == 2) ? 2 : 4;
    }();
    return v;
}

template <int EPI>
int launch(const GemmParams& p, hipStream_t st) {
    const int64_t tiles = ceil_div(p.M, kBM);
    if (tiles > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
    const dim3 g(static_cast<unsigned>(tiles)), b(kThreads);
    if (EPI == kEpiEluGrad && dgrad_occupancy() == 2)
        hipLaunchKernelGGL((mlp_gemm_kernel<EPI, 2>), g, b, 0, st, p);
    else
        hipLaunchKernelGGL((mlp_gemm_kernel<EPI, 4>), g, b, 0, st, p);
    return launch_status();
}

}  // namespace
}  // namespace rslrl

using namespace rslrl;

extern "C" int64_t rslrl_linear_tiles(int64_t M) { return ceil_div(M, kBM); }

extern "C" int rslrl_linear_fwd(const float* x, int64_t M, int32_t K, const float* weight, int32_t N,
                                const float* bias, int32_t activation, float* y, rslrl_stream_t stream) {
    if (M < 0 || K < 1 || N < 1 || N > kBN || (K & 3) || K > INT32_MAX / 2) return RSLRL_E_INVALID_ARGUMENT;
    if (M == 0) return RSLRL_OK;
    if (!x || !weight || !bias || !y) return RSLRL_E_INVALID_ARGUMENT;
    if (!aligned16(x) || !aligned16(weight)) return RSLRL_E_MISALIGNED;
    if (activation != 0 && activation != 1) return RSLRL_E_UNSUPPORTED;
    GemmParams p{x, weight, bias, nullptr, y, nullptr, M, K, N};
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    return activation ? launch<kEpiBiasElu>(p, st) : launch<kEpiBias>(p, st);
}

extern "C" int rslrl_linear_dgrad_elu(const float* dz, int64_t M, int32_t Nred, const float* weight_t, int32_t K,
                                      const float* h, float* dz_prev, float* colsum_partials,
                                      rslrl_stream_t stream) {
    if (M < 0 || Nred < 1 || K < 1 || K > kBN || (Nred & 3)) return RSLRL_E_INVALID_ARGUMENT;
    if (M == 0) return RSLRL_OK;
    if (!dz || !weight_t || !h || !dz_prev || !colsum_partials) return RSLRL_E_INVALID_ARGUMENT;
    if (!aligned16(dz) || !aligned16(weight_t)) return RSLRL_E_MISALIGNED;
    // GEMM view: A = dZ [M, Nred], Bw = W^T [K, Nred] -> C = dZ W [M, K]
    GemmParams p{dz, weight_t, nullptr, h, dz_prev, colsum_partials, M, Nred, K};
    return launch<kEpiEluGrad>(p, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int rslrl_column_sum_fold(const float* partials, int64_t tiles, int32_t N, float* out,
                                     rslrl_stream_t stream) {
    if (tiles < 1 || tiles > INT32_MAX || N < 1 || !partials || !out) return RSLRL_E_INVALID_ARGUMENT;
    hipLaunchKernelGGL(colsum_fold_kernel, dim3(static_cast<unsigned>(N)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), partials, static_cast<int>(tiles), out);
    return launch_status();
}
