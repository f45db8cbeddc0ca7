// Weight gradient of the actor/critic MLP layers on the split-bf16 ("x6") MFMA path:
//   dW[n][k] = sum_m dZ[m][n] X[m][k]        dZ [M, N] (layer output grad), X [M, K] (layer input)
// the autograd backward of nn.Linear's weight (rsl_rl/networks/mlp.py:106-114 layers; the reference runs
// it as one cuBLAS GEMM per layer).  M is the mini-batch (393216 rows at C3); N, K <= 256.
//
// Split-K over M: workgroup s reduces rows [s * rows_per, (s + 1) * rows_per) into a full TN x 256 tile
// of partial sums ([S][N][K] fp32), fold_kernel adds the S partials in a fixed order in fp64 ->
// deterministic.  Both operands are consumed along their row index m, which is the MFMA reduction
// index, so each is staged in its natural [m][col] layout (coalesced float4 loads, split into three bf16
// planes while staged) and read back column-wise with ds_read_b64_tr_b16 (MI355X_MICROARCH.md §LDS;
// cdna_hip_programming.md T10): lane 4q+p of each 16-lane group addresses row q, columns 4p..4p+3 of a
// 4-row block and receives its own column's 4 rows -- exactly a 32x32x16 operand fragment half.
//
// LDS image per buffer and operand: 3 planes x [16 m][COLS bf16]; on 512-B rows the 16-B chunks of row m
// are XOR-permuted by 4 (m & 3), which makes the transposed reads (4 rows x 64 B per 32-lane half) and
// the staging stores (ds_write_b64, 128 contiguous bytes per 16 lanes) bank-conflict free; on 128-B rows
// (TN = 64) rows 2, 3 (mod 4) swap their 64-B halves, which separates the banks of the four rows a 32-lane
// transposed read spans; 64-B rows (TN = 32) need no permutation.
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "x6_split.h"

namespace rslrl {
namespace {

constexpr int kThreadsW = 512;
constexpr int kMC = 16;  // rows of m per chunk (one MFMA k step)
constexpr int kTK = 256;
#ifndef RSLRL_WGRAD_DEPTH
#define RSLRL_WGRAD_DEPTH 2
#endif
constexpr int kWgradDepth = RSLRL_WGRAD_DEPTH;  // chunks of look-ahead in registers (full tiles): 2 or 4

using s16x4 = __attribute__((ext_vector_type(4))) short;

struct WgradParams {
    const float* dz;  // [M, N]
    const float* x;   // [M, K]
    float* part;      // [S, N, K]
    int64_t M;
    int64_t rows_per;  // multiple of kMC
    int N;
    int K;
    const float* dz_amax;  // h3 (PL = 2): max |dz|, max |x| -> the operands' power-of-two scales
    const float* x_amax;
};

template <int COLS>
__device__ __forceinline__ int swz(int m, int col) {  // byte offset of (m, col), col % 4 == 0, within a plane
    constexpr int rowb = COLS * 2;
    if constexpr (rowb >= 512) return rowb * m + 16 * ((col >> 3) ^ (4 * (m & 3))) + 8 * ((col >> 2) & 1);
    if constexpr (rowb == 128) return rowb * m + 16 * ((col >> 3) ^ (4 * ((m >> 1) & 1))) + 8 * ((col >> 2) & 1);
    return rowb * m + 2 * col;
}

// stage one operand chunk: rows m0.. m0+15 (global rows < m_end valid), columns < ncols valid
// MASKC (full tiles whose operand has fewer than COLS columns, e.g. the first layer's 48 inputs on 64-row tiles):
// columns >= ncols load a clamped in-row address unconditionally and are zeroed by a select, so the load stream
// keeps no control flow (the look-ahead's waitcnt counting needs that)
template <int COLS, bool FULL, bool MASKC = false>
__device__ __forceinline__ void load_tile(const float* __restrict__ src, int ld, int64_t m0, int64_t m_end,
                                          int ncols, float4 (&v)[(kMC * COLS / 4 + kThreadsW - 1) / kThreadsW]) {
    constexpr int units = kMC * COLS / 4;
    constexpr int per = (units + kThreadsW - 1) / kThreadsW;
#pragma unroll
    for (int i = 0; i < per; ++i) {
        const int u = threadIdx.x + kThreadsW * i;
        const int m = u / (COLS / 4);
        const int c = 4 * (u % (COLS / 4));
        const int64_t row = m0 + m;
        if constexpr (FULL && MASKC) {
            const bool ok = c < ncols;
            const float4 t = *reinterpret_cast<const float4*>(src + row * ld + (ok ? c : 0));
            v[i] = ((units % kThreadsW == 0 || u < units) && ok) ? t : make_float4(0.f, 0.f, 0.f, 0.f);
        } else if constexpr (FULL) {
            v[i] = (units % kThreadsW == 0 || u < units)
                       ? *reinterpret_cast<const float4*>(src + row * ld + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
            const bool ok = (units % kThreadsW == 0 || u < units) && row < m_end && c < ncols;
            const float4 t = *reinterpret_cast<const float4*>(src + (ok ? row * ld + c : 0));
            v[i] = ok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
}

template <int COLS, int PL>
__device__ __forceinline__ void store_tile(const float4 (&v)[(kMC * COLS / 4 + kThreadsW - 1) / kThreadsW],
                                           char* __restrict__ img, float sc) {
    constexpr int units = kMC * COLS / 4;
    constexpr int per = (units + kThreadsW - 1) / kThreadsW;
    constexpr int plane = kMC * COLS * 2;
#pragma unroll
    for (int i = 0; i < per; ++i) {
        const int u = threadIdx.x + kThreadsW * i;
        if (units % kThreadsW == 0 || u < units) {
            const int m = u / (COLS / 4);
            const int c = 4 * (u % (COLS / 4));
            uint2 w[PL];
            float4 x = v[i];
            if constexpr (PL == 2) x = make_float4(x.x * sc, x.y * sc, x.z * sc, x.w * sc);
            Arith<PL>::split(x, w);
            const int off = swz<COLS>(m, c);
#pragma unroll
            for (int q = 0; q < PL; ++q) *reinterpret_cast<uint2*>(img + q * plane + off) = w[q];
        }
    }
}

// 32x32x16 operand fragment of columns [cb, cb + 32) (all 16 rows) of one plane, via two transposed reads
template <int COLS, typename F = bf16x8>
__device__ __forceinline__ F read_frag_tr(const char* __restrict__ plane, int cb) {
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4;
    const int q = (lane >> 2) & 3;
    const int p = lane & 3;
    const int col = cb + 16 * (g & 1) + 4 * p;
    const int m = 8 * (g >> 1) + q;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(plane + swz<COLS>(m, col)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(plane + swz<COLS>(m + 4, col)));
    const __attribute__((ext_vector_type(8))) short v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(F, v);
}

// TN = rows of dW per workgroup (256: waves 2 (n) x 4 (k), wave tile 128 x 64; 64: waves 2 x 4, 32 x 64;
// 32: waves 1 x 8, 32 x 32)
// CS: also the column sums of one operand -- the bias gradient of the layer (1: of dz, the TN-row side, TN = 256;
// 2: of x, the 256-column side) -- accumulated in fp32 from the staged registers (every thread's float4 units
// share their 4 columns), folded over the 8 threads of a column quad through LDS in a fixed order and written
// after the tile as the slice's extra partial row: part[s] = [dW (N x K) | colsum (N or K)].
template <int TN, bool FULL, int PL = 3, bool MASKN = false, int CS = 0>
__device__ __forceinline__ void wgrad_x6_body(const WgradParams& p) {
    static_assert(CS != 1 || TN == kTK, "column sums of the dz side need 256-row tiles");
    using Frag = typename Arith<PL>::frag;
    constexpr int WN = TN == 32 ? 1 : 2;
    constexpr int WK = 8 / WN;
    constexpr int I = TN / WN / 32;
    constexpr int J = kTK / WK / 32;
    constexpr int planeA = kMC * TN * 2;
    constexpr int planeB = kMC * kTK * 2;
    constexpr int bufBytes = PL * planeA + PL * planeB;
    constexpr int perA = (kMC * TN / 4 + kThreadsW - 1) / kThreadsW;
    constexpr int perB = (kMC * kTK / 4 + kThreadsW - 1) / kThreadsW;
    __shared__ __attribute__((aligned(16))) char lds[2][bufBytes];

    const int wave = threadIdx.x >> 6;
    const int wn = wave / WK;
    const int wk = wave % WK;
    const int64_t m_begin = static_cast<int64_t>(blockIdx.x) * p.rows_per;
    const int64_t m_end = m_begin + p.rows_per < p.M ? m_begin + p.rows_per : p.M;
    const int nchunks = static_cast<int>((m_end - m_begin + kMC - 1) / kMC);
    const float sa = PL == 2 ? h3_scale(*p.dz_amax) : 1.f;
    const float sb = PL == 2 ? h3_scale(*p.x_amax) : 1.f;

    f32x16 acc[I][J];
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j) acc[i][j] = f32x16{};
    float4 csum = make_float4(0.f, 0.f, 0.f, 0.f);  // CS: this thread's 4 columns
    // sum the staged chunk of the CS operand (raw values, before any h3 scaling)
    auto accum_a = [&](const float4 (&v)[perA]) {
        if constexpr (CS == 1) {
#pragma unroll
            for (int i = 0; i < perA; ++i) { csum.x += v[i].x; csum.y += v[i].y; csum.z += v[i].z; csum.w += v[i].w; }
        }
    };
    auto accum_b = [&](const float4 (&v)[perB]) {
        if constexpr (CS == 2) {
#pragma unroll
            for (int i = 0; i < perB; ++i) { csum.x += v[i].x; csum.y += v[i].y; csum.z += v[i].z; csum.w += v[i].w; }
        }
    };

    auto compute = [&](const char* a_img) {
        const char* b_img = a_img + PL * planeA;
        Frag bf[J][PL];
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int q = 0; q < PL; ++q) bf[j][q] = read_frag_tr<kTK, Frag>(b_img + q * planeB, wk * (J * 32) + j * 32);
#pragma unroll
        for (int i = 0; i < I; ++i) {
            Frag af[PL];
#pragma unroll
            for (int q = 0; q < PL; ++q) af[q] = read_frag_tr<TN, Frag>(a_img + q * planeA, wn * (I * 32) + i * 32);
#pragma unroll
            for (int j = 0; j < J; ++j) acc[i][j] = Arith<PL>::mfma(af, bf[j], acc[i][j]);
        }
    };

    if constexpr (FULL) {
        // Look-ahead pipeline: chunk c + 1 is split into LDS at the end of chunk c from registers loaded kWgradDepth
        // chunks earlier, so kWgradDepth chunks (2 x 32 KiB per workgroup at TN = 256) stay in flight across
        // the chunk barriers -- a one-chunk look-ahead behind __syncthreads (whose release fence waits
        // vmcnt(0)) left ~32 KiB per CU in flight, about half of what the HBM latency asks for.
        constexpr int D = kWgradDepth;
        float4 ra[D][perA], rb[D][perB];
        {
            float4 va[perA], vb[perB];
            load_tile<TN, true, MASKN>(p.dz, p.N, m_begin, m_end, p.N, va);
            load_tile<kTK, true>(p.x, p.K, m_begin, m_end, p.K, vb);
            accum_a(va);
            accum_b(vb);
            store_tile<TN, PL>(va, lds[0], sa);
            store_tile<kTK, PL>(vb, lds[0] + PL * planeA, sb);
        }
        // every look-ahead load is issued, past the end clamped to the last chunk (data unused): with
        // conditional loads the waitcnt pass cannot count the younger slot's loads and waits vmcnt(0)
        auto chunk_row = [&](int c) { return m_begin + static_cast<int64_t>(c < nchunks ? c : nchunks - 1) * kMC; };
#pragma unroll
        for (int d = 1; d <= D; ++d) {
            load_tile<TN, true, MASKN>(p.dz, p.N, chunk_row(d), m_end, p.N, ra[d % D]);
            load_tile<kTK, true>(p.x, p.K, chunk_row(d), m_end, p.K, rb[d % D]);
        }
        __syncthreads();
        // chunk c (ring position u = c % D) followed by chunk c + 1: no branch between a slot's loads and their
        // use, so the waitcnt pass counts the younger slot's loads (vmcnt(4 per slot)) instead of draining
        auto step = [&](auto uc, int c) {
            constexpr int u = decltype(uc)::value;
            constexpr int s = (u + 1) % D;
            compute(lds[u & 1]);
            __builtin_amdgcn_sched_barrier(0);  // the splits below stay behind this chunk's MFMAs
            accum_a(ra[s]);  // chunk c + 1: every real chunk is stored (and summed) exactly once
            accum_b(rb[s]);
            store_tile<TN, PL>(ra[s], lds[(u + 1) & 1], sa);
            store_tile<kTK, PL>(rb[s], lds[(u + 1) & 1] + PL * planeA, sb);
            load_tile<TN, true, MASKN>(p.dz, p.N, chunk_row(c + 1 + D), m_end, p.N, ra[s]);
            load_tile<kTK, true>(p.x, p.K, chunk_row(c + 1 + D), m_end, p.K, rb[s]);
            // only the LDS writes must retire before the barrier (not the look-ahead loads)
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        };
        static_assert(D == 2 || D == 4, "the host guarantees a chunk count that is a multiple of D >= 2");
        int c0 = 0;
        for (; c0 + D < nchunks; c0 += D) {
            step(std::integral_constant<int, 0>{}, c0);
            step(std::integral_constant<int, 1>{}, c0 + 1);
            if constexpr (D == 4) {
                step(std::integral_constant<int, 2>{}, c0 + 2);
                step(std::integral_constant<int, 3>{}, c0 + 3);
            }
        }
        step(std::integral_constant<int, 0>{}, c0);
        if constexpr (D == 4) {
            step(std::integral_constant<int, 1>{}, c0 + 1);
            step(std::integral_constant<int, 2>{}, c0 + 2);
        }
        compute(lds[1]);
    } else {
    float4 va[perA], vb[perB];
    if (nchunks > 0) {
        load_tile<TN, FULL>(p.dz, p.N, m_begin, m_end, p.N, va);
        load_tile<kTK, FULL>(p.x, p.K, m_begin, m_end, p.K, vb);
        accum_a(va);
        accum_b(vb);
        store_tile<TN, PL>(va, lds[0], sa);
        store_tile<kTK, PL>(vb, lds[0] + PL * planeA, sb);
    }
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
        const int buf = c & 1;
        const bool more = c + 1 < nchunks;
        if (more) {
            const int64_t m0 = m_begin + static_cast<int64_t>(c + 1) * kMC;
            load_tile<TN, FULL>(p.dz, p.N, m0, m_end, p.N, va);
            load_tile<kTK, FULL>(p.x, p.K, m0, m_end, p.K, vb);
        }
        compute(lds[buf]);
        if (more) {
            accum_a(va);
            accum_b(vb);
            store_tile<TN, PL>(va, lds[buf ^ 1], sa);
            store_tile<kTK, PL>(vb, lds[buf ^ 1] + PL * planeA, sb);
        }
        __syncthreads();
    }
    }  // !FULL

    // partial tile -> part[s][n][k]; C/D map: col (k) = lane & 31, row (n) = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    const int lane = threadIdx.x & 63;
    const int l32 = lane & 31;
    const int h = lane >> 5;
    const float unscale = PL == 2 ? (1.f / sa) * (1.f / sb) : 1.f;  // exact: powers of two
    const int E = CS == 1 ? p.N : (CS == 2 ? p.K : 0);
    float* out = p.part + static_cast<int64_t>(blockIdx.x) * (static_cast<int64_t>(p.N) * p.K + E);
    if constexpr (CS != 0) {
        // threads t, t + 64, ..., t + 448 hold columns 4 (t & 63) .. + 3 of different rows: fixed-order fold
        float* red = reinterpret_cast<float*>(&lds[0][0]);  // [8][256]
        __syncthreads();  // the last chunk's fragments have been read
        reinterpret_cast<float4*>(red)[threadIdx.x] = csum;
        __syncthreads();
        if (threadIdx.x < 64) {
            float4 t = reinterpret_cast<const float4*>(red)[threadIdx.x];
#pragma unroll
            for (int g = 1; g < 8; ++g) {
                const float4 v = reinterpret_cast<const float4*>(red)[64 * g + threadIdx.x];
                t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
            }
            const int col = 4 * threadIdx.x;
            float* dst = out + static_cast<int64_t>(p.N) * p.K;
            if (col + 3 < E) {
                *reinterpret_cast<float4*>(dst + col) = t;
            } else {
                const float tv[4] = {t.x, t.y, t.z, t.w};
                for (int e = 0; e < 4; ++e)
                    if (col + e < E) dst[col + e] = tv[e];
            }
        }
    }
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int k = wk * (J * 32) + j * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = wn * (I * 32) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (n < p.N && k < p.K) out[n * p.K + k] = PL == 2 ? acc[i][j][r] * unscale : acc[i][j][r];
            }
        }
}

template <int TN, bool FULL, int PL = 3, bool MASKN = false, int CS = 0>
__global__ __launch_bounds__(kThreadsW, TN <= 64 ? 4 : 2) void wgrad_x6_kernel(WgradParams p) {  // <= 64: 2 per CU
    wgrad_x6_body<TN, FULL, PL, MASKN, CS>(p);
}

// Two weight gradients of one shape in one launch (blockIdx.y selects the problem) -- the actor's and the critic's
// layer l in the update's backward.  With both in one grid each problem takes half the slices (twice the rows per
// slice), so its partials (and their fold) are half as large at the same occupancy.
struct WgradPair {
    WgradParams p[2];
};

template <int TN, bool FULL, int PL = 3, bool MASKN = false, int CS = 0>
__global__ __launch_bounds__(kThreadsW, TN <= 64 ? 4 : 2) void wgrad_x6_pair_kernel(WgradPair b) {
    wgrad_x6_body<TN, FULL, PL, MASKN, CS>(b.p[blockIdx.y]);
}

// dW[e] = sum over s of part[s][e] (e < N * K), fp64, fixed order: thread (g, c) of a 256-thread block
// sums slices s = g (mod 4) of the float4 column group c (unrolled so several loads are in flight), then
// the four group sums are added in g order through LDS.  One block per 256 outputs.
// out[e] = sum of part[s][e] over the slices s of group blockIdx.y (per slices each) in a fixed order: four
// interleaved fp64 accumulator groups (s % 4), combined ((g0 + g1) + g2) + g3.  IN is float (partials) or
// double (stage-1 group sums); OUT is double (stage 1 of a two-stage fold) or float (final).
// Where a folded fp32 value e lands: e < out_len only; the leading t_rows x t_cols block transposed
// (e = r * t_cols + c -> out[c * t_rows + r]: the first layer's (x^T dz)^T weight gradient written as W's layout),
// the rest (the column sums) in place.  Identity: out_len = NK, t_rows = 0.
struct OutMap {
    int64_t out_len;
    int t_rows, t_cols;
};

__device__ __forceinline__ void store_mapped(float* __restrict__ out, int64_t e0, const float (&v)[4], OutMap m) {
    if (m.t_rows == 0 && e0 + 3 < m.out_len && !(reinterpret_cast<uintptr_t>(out + e0) & 15)) {
        *reinterpret_cast<float4*>(out + e0) = make_float4(v[0], v[1], v[2], v[3]);
        return;
    }
    const int64_t tn = static_cast<int64_t>(m.t_rows) * m.t_cols;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t e = e0 + k;
        if (e >= m.out_len) break;
        out[e < tn ? (e % m.t_cols) * m.t_rows + e / m.t_cols : e] = v[k];
    }
}

template <typename IN, typename OUT>
__global__ __launch_bounds__(kBlock) void fold_kernel(const IN* __restrict__ part, int S, int per, int NK,
                                                      OUT* __restrict__ out, OutMap omap) {
    __shared__ double red[4][64][4];
    const int g = threadIdx.x >> 6;
    const int c = threadIdx.x & 63;
    const int e0 = blockIdx.x * 256 + 4 * c;  // NK % 4 == 0 (K % 4 == 0)
    const int s0 = blockIdx.y * per;
    const int s1 = min(S, s0 + per);
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    if (e0 < NK) {
        const IN* src = part + e0;
#pragma unroll 8
        for (int s = s0 + g; s < s1; s += 4) {
            const IN* q = src + static_cast<int64_t>(s) * NK;
            if constexpr (sizeof(IN) == 4) {
                const float4 v = *reinterpret_cast<const float4*>(q);
                a[0] += v.x; a[1] += v.y; a[2] += v.z; a[3] += v.w;
            } else {
                const double2 v0 = reinterpret_cast<const double2*>(q)[0];
                const double2 v1 = reinterpret_cast<const double2*>(q)[1];
                a[0] += v0.x; a[1] += v0.y; a[2] += v1.x; a[3] += v1.y;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) red[g][c][k] = a[k];
    __syncthreads();
    if (g == 0 && e0 < NK) {
        double r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = ((red[0][c][k] + red[1][c][k]) + red[2][c][k]) + red[3][c][k];
        OUT* dst = out + static_cast<int64_t>(blockIdx.y) * NK + e0;
        if constexpr (sizeof(OUT) == 4) {  // the final stage (one group): mapped
            const float v[4] = {static_cast<float>(r[0]), static_cast<float>(r[1]), static_cast<float>(r[2]),
                                static_cast<float>(r[3])};
            store_mapped(out, e0, v, omap);
        } else {
            reinterpret_cast<double2*>(dst)[0] = make_double2(r[0], r[1]);
            reinterpret_cast<double2*>(dst)[1] = make_double2(r[2], r[3]);
        }
    }
}

// One-pass fold for wide partials (NK >= 64 * kWideMinBlocks, e.g. the 256 x 256 hidden-layer weight gradient:
// 256 slices x 65536 values): 64 columns per 256-thread block, the block's threads as 16 column quads x 16 slice
// phases.  Thread (phase p, quad q) adds slices p, p + 16, ... of its float4 in fp64 with up to 16 loads in
// flight (the one-quad-per-thread fold_kernel had 8 and one block per CU: 21 us for 67 MB), then the 16
// phases are added in phase order through LDS.  Deterministic: the order depends on S alone.
constexpr int kWideMinBlocks = 128;  // the first layer's 48 x 256 (+ bias) partials (193 blocks): 14.4 us in
                                     // two fold_kernel stages; one pass keeps 64 KiB per CU in flight
__global__ __launch_bounds__(kBlock) void fold_wide_kernel(const float* __restrict__ part, int S, int NK,
                                                           float* __restrict__ out, OutMap omap) {
    __shared__ double red[16][16][4];
    const int q = threadIdx.x & 15;
    const int ph = threadIdx.x >> 4;
    const int e0 = blockIdx.x * 64 + 4 * q;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    if (e0 < NK) {
        const float* src = part + e0;
        for (int s0 = ph; s0 < S; s0 += 16 * 16) {
            float4 v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int s = s0 + 16 * k;
                v[k] = s < S ? *reinterpret_cast<const float4*>(src + static_cast<int64_t>(s) * NK)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                a[0] += v[k].x; a[1] += v[k].y; a[2] += v[k].z; a[3] += v[k].w;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) red[ph][q][k] = a[k];
    __syncthreads();
    if (ph == 0 && e0 < NK) {
        double r[4] = {red[0][q][0], red[0][q][1], red[0][q][2], red[0][q][3]};
        for (int p2 = 1; p2 < 16; ++p2)
#pragma unroll
            for (int k = 0; k < 4; ++k) r[k] += red[p2][q][k];
        const float v[4] = {static_cast<float>(r[0]), static_cast<float>(r[1]), static_cast<float>(r[2]),
                            static_cast<float>(r[3])};
        store_mapped(out, e0, v, omap);
    }
}

// Several folds in one launch (rslrl_fold_partials_batch).  Job j spans CB = ceil(NK / 64) column blocks x G slice
// groups; block (cb, g) runs fold_wide's body over its group's slices (16 slice phases x 16 column quads, fp64,
// phase order).  G = 1 (many columns or <= 256 slices): the block writes its 64 outputs.  G > 1 (a narrow job with
// many slices, e.g. the value head's 3072 tile partials of 260 columns, which one pass would leave to 5 blocks): the
// groups' fp64 sums go to the workspace and the last-arriving group of the column block adds them in group order.
// Deterministic: the order depends on (S, G) alone.
constexpr int kMaxFoldJobs = 16;
#ifndef RSLRL_FOLD_UNROLL
#define RSLRL_FOLD_UNROLL 4
#endif
constexpr int kFoldUnroll = RSLRL_FOLD_UNROLL;  // slices loaded per round per thread (fold_batch_kernel)
constexpr int kFoldGroupSlices = 256;
struct FoldJobs {
    const float* part[kMaxFoldJobs];
    float* out[kMaxFoldJobs];
    OutMap omap[kMaxFoldJobs];
    int S[kMaxFoldJobs];
    int NK[kMaxFoldJobs];
    int G[kMaxFoldJobs];
    int64_t ws_off[kMaxFoldJobs];  // doubles
    int t_off[kMaxFoldJobs];       // tickets
    int first_block[kMaxFoldJobs + 1];
    int n;
    double* ws;
    unsigned* tickets;
};

int fold_batch_groups(int64_t S, int64_t NK) {
    const int64_t cb = ceil_div(NK, 64);
    if (S <= kFoldGroupSlices || cb >= 128) return 1;
    return static_cast<int>(std::min<int64_t>(ceil_div(S, kFoldGroupSlices), 16));
}

__global__ __launch_bounds__(kBlock) void fold_batch_kernel(FoldJobs jobs) {
    __shared__ double red[16][16][4];
    __shared__ int last_flag;
    int j = 0;
    while (j + 1 < jobs.n && static_cast<int>(blockIdx.x) >= jobs.first_block[j + 1]) ++j;  // wave-uniform
    const int NK = jobs.NK[j], S = jobs.S[j], G = jobs.G[j];
    const int CB = (NK + 63) / 64;
    const int li = static_cast<int>(blockIdx.x) - jobs.first_block[j];
    const int cb = li % CB, g = li / CB;
    const int per = (S + G - 1) / G;
    const int s_lo = g * per, s_hi = min(S, s_lo + per);
    const int q = threadIdx.x & 15;
    const int ph = threadIdx.x >> 4;
    const int e0 = cb * 64 + 4 * q;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    if (e0 < NK) {
        const float* src = jobs.part[j] + e0;
        // kFoldUnroll slices per round (the same slice order for any unroll: s_lo + ph, + 16, + 32, ...): 4 keeps the
        // kernel at 52 VGPRs, 8 workgroups per CU (16: 148 VGPRs, 3 per CU, 49.7 us per fold at the 16384-env share;
        // 8: 84 VGPRs, 36.2 us; 4: 35.1 us -- rocprof, profiles/r4_fold_unroll_ab.json)
        for (int s0 = s_lo + ph; s0 < s_hi; s0 += 16 * kFoldUnroll) {
            float4 v[kFoldUnroll];
#pragma unroll
            for (int k = 0; k < kFoldUnroll; ++k) {
                const int s = s0 + 16 * k;
                v[k] = s < s_hi ? *reinterpret_cast<const float4*>(src + static_cast<int64_t>(s) * NK)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int k = 0; k < kFoldUnroll; ++k) {
                a[0] += v[k].x; a[1] += v[k].y; a[2] += v[k].z; a[3] += v[k].w;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) red[ph][q][k] = a[k];
    __syncthreads();
    double r[4] = {0.0, 0.0, 0.0, 0.0};
    if (ph == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = red[0][q][k];
        for (int p2 = 1; p2 < 16; ++p2)
#pragma unroll
            for (int k = 0; k < 4; ++k) r[k] += red[p2][q][k];
    }
    if (G > 1) {
        double* wp = jobs.ws + jobs.ws_off[j];
        if (ph == 0 && e0 < NK) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                __hip_atomic_store(reinterpret_cast<unsigned long long*>(wp + static_cast<int64_t>(g) * NK + e0 + k),
                                   __double_as_longlong(r[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned* t = jobs.tickets + jobs.t_off[j] + cb;
            const unsigned k = __hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = k == static_cast<unsigned>(G) - 1;
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed for the next call
            }
            last_flag = last;
        }
        __syncthreads();
        if (!last_flag) return;
        if (ph == 0 && e0 < NK) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                double t = 0.0;
                for (int g2 = 0; g2 < G; ++g2)
                    t += __longlong_as_double(__hip_atomic_load(
                        reinterpret_cast<unsigned long long*>(wp + static_cast<int64_t>(g2) * NK + e0 + k),
                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                r[k] = t;
            }
        }
    }
    if (ph == 0 && e0 < NK) {
        const float v[4] = {static_cast<float>(r[0]), static_cast<float>(r[1]), static_cast<float>(r[2]),
                            static_cast<float>(r[3])};
        store_mapped(jobs.out[j], e0, v, jobs.omap[j]);
    }
}

// Two-stage fold when one pass would leave the chip idle (few columns, many slices -- e.g. the output
// layer's per-tile partials: 3072 slices x 3072 columns): stage 1 sums groups of kFoldPer slices into fp64
// [G][NK], stage 2 sums the G groups.  The order is fixed by (S, NK) alone: deterministic.
constexpr int kFoldPer = 64;

int64_t fold_groups(int64_t S, int64_t NK) {
    const int64_t cols = ceil_div(NK, 256);
    if (S <= kFoldPer || cols >= 256) return 1;
    return ceil_div(S, kFoldPer);
}

// one workgroup per CU for the 256-row tiles (98 KiB of LDS each); the 32 / 64-row tiles (<= 60 KiB) run two
// per CU, so twice as many slices keep 16 waves per CU in flight; at least 4 chunks per slice
int64_t wgrad_slices(int64_t M, int N) {
    const int64_t chunks = ceil_div(M, kMC);
    const int64_t max_slices = N <= 64 ? 512 : 256;
    return std::max<int64_t>(1, std::min<int64_t>(max_slices, chunks / 4));
}

int64_t wgrad_rows_per(int64_t M, int N) { return ceil_div(ceil_div(M, wgrad_slices(M, N)), kMC) * kMC; }

}  // namespace
}  // namespace rslrl

using namespace rslrl;

extern "C" size_t rslrl_fold_partials_workspace_bytes(int64_t S, int64_t NK) {
    if (S < 1 || NK < 1) return 0;
    const int64_t G = fold_groups(S, NK);
    return G > 1 ? static_cast<size_t>(G) * NK * sizeof(double) : 0;
}

// workspace: the [S][N][K] partials, then the fold's fp64 group sums
namespace rslrl {
namespace {
// extra values per partial row for a column-sum side (0 none, 1 dz: N, 2 x: K)
int64_t colsum_len(int side, int32_t N, int32_t K) { return side == 1 ? N : (side == 2 ? K : 0); }
}  // namespace
}  // namespace rslrl

extern "C" size_t rslrl_linear_wgrad_bias_workspace_bytes(int64_t M, int32_t N, int32_t K, int32_t bias_side) {
    if (M < 1 || N < 1 || K < 1 || bias_side < 0 || bias_side > 2) return 0;
    const int64_t S = ceil_div(M, wgrad_rows_per(M, N));
    const int64_t NKE = static_cast<int64_t>(N) * K + colsum_len(bias_side, N, K);
    return static_cast<size_t>(S) * NKE * sizeof(float) + rslrl_fold_partials_workspace_bytes(S, NKE);
}

extern "C" size_t rslrl_linear_wgrad_workspace_bytes(int64_t M, int32_t N, int32_t K) {
    return rslrl_linear_wgrad_bias_workspace_bytes(M, N, K, 0);
}

extern "C" int rslrl_fold_partials_ex(const float* partials, int64_t S, int64_t NK, float* out, int64_t out_len,
                                      int32_t t_rows, int32_t t_cols, void* workspace, size_t workspace_bytes,
                                      rslrl_stream_t stream) {
    if (!partials || !out || S < 1 || S > INT32_MAX || NK < 4 || NK > INT32_MAX || (NK & 3)) return RSLRL_E_INVALID_ARGUMENT;
    if (out_len < 1 || out_len > NK || t_rows < 0 || t_cols < 0 || (t_rows > 0) != (t_cols > 0) ||
        static_cast<int64_t>(t_rows) * t_cols > out_len)
        return RSLRL_E_INVALID_ARGUMENT;
    if (reinterpret_cast<uintptr_t>(partials) & 15) return RSLRL_E_MISALIGNED;  // (out: any 4-byte alignment)
    const OutMap omap{out_len, t_rows, t_cols};
    const OutMap ident{NK, 0, 0};
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (ceil_div(NK, 64) >= kWideMinBlocks) {
        hipLaunchKernelGGL(fold_wide_kernel, dim3(static_cast<unsigned>(ceil_div(NK, 64))), dim3(kBlock), 0, st,
                           partials, static_cast<int>(S), static_cast<int>(NK), out, omap);
        return launch_status();
    }
    const unsigned cols = static_cast<unsigned>(ceil_div(NK, 256));
    const int64_t G = fold_groups(S, NK);
    if (G == 1) {
        hipLaunchKernelGGL((fold_kernel<float, float>), dim3(cols), dim3(kBlock), 0, st, partials,
                           static_cast<int>(S), static_cast<int>(S), static_cast<int>(NK), out, omap);
        return launch_status();
    }
    if (!workspace) return RSLRL_E_INVALID_ARGUMENT;
    if (reinterpret_cast<uintptr_t>(workspace) & 15) return RSLRL_E_MISALIGNED;
    if (workspace_bytes < static_cast<size_t>(G) * NK * sizeof(double)) return RSLRL_E_WORKSPACE_TOO_SMALL;
    double* ws = static_cast<double*>(workspace);
    hipLaunchKernelGGL((fold_kernel<float, double>), dim3(cols, static_cast<unsigned>(G)), dim3(kBlock), 0, st,
                       partials, static_cast<int>(S), kFoldPer, static_cast<int>(NK), ws, ident);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL((fold_kernel<double, float>), dim3(cols), dim3(kBlock), 0, st, static_cast<const double*>(ws),
                       static_cast<int>(G), static_cast<int>(G), static_cast<int>(NK), out, omap);
    return launch_status();
}

extern "C" int rslrl_fold_partials(const float* partials, int64_t S, int64_t NK, float* out, void* workspace,
                                   size_t workspace_bytes, rslrl_stream_t stream) {
    return rslrl_fold_partials_ex(partials, S, NK, out, NK, 0, 0, workspace, workspace_bytes, stream);
}

namespace rslrl {
namespace {
// workspace of a batch: tickets (one per column block of every grouped job) first -- the region a zero-filled
// buffer keeps zero across calls -- then the grouped jobs' fp64 group sums
int64_t fold_batch_layout(const rslrl_fold_job_t* jobs, int32_t n, FoldJobs* fj) {
    int64_t tickets = 0, doubles = 0;
    for (int i = 0; i < n; ++i) {
        const int G = fold_batch_groups(jobs[i].S, jobs[i].NK);
        if (fj) {
            fj->G[i] = G;
            fj->t_off[i] = static_cast<int>(tickets);
        }
        if (G > 1) tickets += ceil_div(jobs[i].NK, 64);
    }
    const int64_t ticket_bytes = (tickets * 4 + 255) / 256 * 256;
    for (int i = 0; i < n; ++i) {
        const int G = fold_batch_groups(jobs[i].S, jobs[i].NK);
        if (fj) fj->ws_off[i] = ticket_bytes / 8 + doubles;
        if (G > 1) doubles += static_cast<int64_t>(G) * jobs[i].NK;
    }
    return ticket_bytes + doubles * 8;
}
}  // namespace
}  // namespace rslrl

extern "C" size_t rslrl_fold_partials_batch_workspace_bytes(const rslrl_fold_job_t* jobs, int32_t n) {
    if (!jobs || n < 1 || n > kMaxFoldJobs) return 0;
    return static_cast<size_t>(fold_batch_layout(jobs, n, nullptr));
}

extern "C" int rslrl_fold_partials_batch(const rslrl_fold_job_t* jobs, int32_t n, void* workspace,
                                         size_t workspace_bytes, rslrl_stream_t stream) {
    if (!jobs || n < 1 || n > kMaxFoldJobs) return RSLRL_E_INVALID_ARGUMENT;
    FoldJobs fj{};
    fj.n = n;
    int64_t blocks = 0;
    for (int i = 0; i < n; ++i) {
        const rslrl_fold_job_t& j = jobs[i];
        if (!j.partials || !j.out || j.S < 1 || j.S > INT32_MAX || j.NK < 4 || j.NK > INT32_MAX || (j.NK & 3))
            return RSLRL_E_INVALID_ARGUMENT;
        if (j.out_len < 1 || j.out_len > j.NK || j.t_rows < 0 || j.t_cols < 0 || (j.t_rows > 0) != (j.t_cols > 0) ||
            static_cast<int64_t>(j.t_rows) * j.t_cols > j.out_len)
            return RSLRL_E_INVALID_ARGUMENT;
        if (reinterpret_cast<uintptr_t>(j.partials) & 15) return RSLRL_E_MISALIGNED;
    }
    const int64_t need = fold_batch_layout(jobs, n, &fj);
    if (need > 256) {  // some job is grouped: the workspace holds its tickets (zero) and group sums
        if (!workspace) return RSLRL_E_INVALID_ARGUMENT;
        if (workspace_bytes < static_cast<size_t>(need)) return RSLRL_E_WORKSPACE_TOO_SMALL;
        if (reinterpret_cast<uintptr_t>(workspace) & 255) return RSLRL_E_MISALIGNED;
    }
    fj.tickets = static_cast<unsigned*>(workspace);
    fj.ws = static_cast<double*>(workspace);
    for (int i = 0; i < n; ++i) {
        const rslrl_fold_job_t& j = jobs[i];
        fj.part[i] = j.partials;
        fj.out[i] = j.out;
        fj.omap[i] = OutMap{j.out_len, j.t_rows, j.t_cols};
        fj.S[i] = static_cast<int>(j.S);
        fj.NK[i] = static_cast<int>(j.NK);
        fj.first_block[i] = static_cast<int>(blocks);
        blocks += ceil_div(j.NK, 64) * fj.G[i];
        if (blocks > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
    }
    fj.first_block[n] = static_cast<int>(blocks);
    hipLaunchKernelGGL(fold_batch_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), fj);
    return launch_status();
}

extern "C" int rslrl_linear_wgrad_bias(const float* dz, const float* dz_amax, const float* x, const float* x_amax,
                                       int64_t M, int32_t N, int32_t K, int32_t arith, int32_t bias_side, float* dw_db,
                                       void* workspace, size_t workspace_bytes, rslrl_stream_t stream) {
    if (M < 1 || N < 1 || K < 1 || N > 256 || K > kTK || (N & 3) || (K & 3)) return RSLRL_E_INVALID_ARGUMENT;
    if (bias_side < 0 || bias_side > 2 || (bias_side == 1 && N <= 64)) return RSLRL_E_INVALID_ARGUMENT;
    if (!dz || !x || !dw_db || !workspace) return RSLRL_E_INVALID_ARGUMENT;
    const bool h3 = arith == RSLRL_ARITH_H3;
    if (!h3 && arith != RSLRL_ARITH_X6) return RSLRL_E_INVALID_ARGUMENT;
    if (h3 && (!dz_amax || !x_amax)) return RSLRL_E_INVALID_ARGUMENT;
    if ((reinterpret_cast<uintptr_t>(dz) | reinterpret_cast<uintptr_t>(x)) & 15) return RSLRL_E_MISALIGNED;
    const int64_t rows_per = wgrad_rows_per(M, N);
    const int64_t S = ceil_div(M, rows_per);
    const int64_t NKE = static_cast<int64_t>(N) * K + colsum_len(bias_side, N, K);
    const size_t part_bytes = static_cast<size_t>(S) * NKE * sizeof(float);  // 16-byte multiple (N, K % 4)
    if (workspace_bytes < rslrl_linear_wgrad_bias_workspace_bytes(M, N, K, bias_side)) return RSLRL_E_WORKSPACE_TOO_SMALL;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    WgradParams p{dz, x, static_cast<float*>(workspace), M, rows_per, N, K, dz_amax, x_amax};
    // full tiles: whole chunks, an even count of them >= 2 (the look-ahead loop), K == kTK (and N <= TN, per branch)
    bool full = (M % rows_per == 0) && K == kTK && (rows_per / kMC) % kWgradDepth == 0;
    const dim3 g(static_cast<unsigned>(S)), b(kThreadsW);
    auto go = [&](auto tn, auto pl, auto cs) {
        constexpr int TN = decltype(tn)::value, PL = decltype(pl)::value, CS = decltype(cs)::value;
        if constexpr (CS == 1 && TN != kTK) {
            return;  // excluded above (N > 64 selects 256-row tiles)
        } else {
            if (full && N == TN) hipLaunchKernelGGL((wgrad_x6_kernel<TN, true, PL, false, CS>), g, b, 0, st, p);
            else if (full && N < TN) hipLaunchKernelGGL((wgrad_x6_kernel<TN, true, PL, true, CS>), g, b, 0, st, p);
            else hipLaunchKernelGGL((wgrad_x6_kernel<TN, false, PL, false, CS>), g, b, 0, st, p);
        }
    };
    auto by_side = [&](auto tn, auto pl) {
        using C0 = std::integral_constant<int, 0>;
        using C1 = std::integral_constant<int, 1>;
        using C2 = std::integral_constant<int, 2>;
        if (bias_side == 1) go(tn, pl, C1{});
        else if (bias_side == 2) go(tn, pl, C2{});
        else go(tn, pl, C0{});
    };
    using I32 = std::integral_constant<int, 32>;
    using I64 = std::integral_constant<int, 64>;
    using I256 = std::integral_constant<int, 256>;
    using P2 = std::integral_constant<int, 2>;
    using P3 = std::integral_constant<int, 3>;
    if (N <= 32) h3 ? by_side(I32{}, P2{}) : by_side(I32{}, P3{});
    else if (N <= 64) h3 ? by_side(I64{}, P2{}) : by_side(I64{}, P3{});
    else h3 ? by_side(I256{}, P2{}) : by_side(I256{}, P3{});
    int rc = launch_status();
    if (rc) return rc;
    return rslrl_fold_partials(static_cast<const float*>(workspace), S, NKE, dw_db,
                               static_cast<char*>(workspace) + part_bytes, workspace_bytes - part_bytes, stream);
}

extern "C" int rslrl_linear_wgrad_ex(const float* dz, const float* dz_amax, const float* x, const float* x_amax,
                                     int64_t M, int32_t N, int32_t K, int32_t arith, float* dw, void* workspace,
                                     size_t workspace_bytes, rslrl_stream_t stream) {
    return rslrl_linear_wgrad_bias(dz, dz_amax, x, x_amax, M, N, K, arith, 0, dw, workspace, workspace_bytes, stream);
}

extern "C" int rslrl_linear_wgrad(const float* dz, const float* x, int64_t M, int32_t N, int32_t K, float* dw,
                                  void* workspace, size_t workspace_bytes, rslrl_stream_t stream) {
    return rslrl_linear_wgrad_ex(dz, nullptr, x, nullptr, M, N, K, RSLRL_ARITH_X6, dw, workspace, workspace_bytes,
                                 stream);
}

// ---- two weight gradients of one shape in one launch (the actor's and the critic's layer l)
namespace rslrl {
namespace {
int64_t wgrad_pair_rows_per(int64_t M, int N) {
    const int64_t S = std::max<int64_t>(1, wgrad_slices(M, N) / 2);
    return ceil_div(ceil_div(M, S), kMC) * kMC;
}
}  // namespace
}  // namespace rslrl

extern "C" size_t rslrl_linear_wgrad_bias_pair_workspace_bytes(int64_t M, int32_t N, int32_t K, int32_t bias_side) {
    if (M < 1 || N < 1 || K < 1 || bias_side < 0 || bias_side > 2) return 0;
    const int64_t S = ceil_div(M, wgrad_pair_rows_per(M, N));
    const int64_t NKE = static_cast<int64_t>(N) * K + colsum_len(bias_side, N, K);
    return static_cast<size_t>(S) * NKE * sizeof(float) + rslrl_fold_partials_workspace_bytes(S, NKE);
}

extern "C" int64_t rslrl_linear_wgrad_bias_pair_slices(int64_t M, int32_t N) {
    return M < 1 || N < 1 ? 0 : ceil_div(M, wgrad_pair_rows_per(M, N));
}

extern "C" int rslrl_linear_wgrad_bias_pair(const rslrl_wgrad_problem_t* a0, const rslrl_wgrad_problem_t* a1,
                                            int64_t M, int32_t N, int32_t K, int32_t arith, int32_t bias_side,
                                            int32_t flags, rslrl_stream_t stream) {
    if (flags & ~RSLRL_WGRAD_NO_FOLD) return RSLRL_E_INVALID_ARGUMENT;
    if (!a0 || !a1) return RSLRL_E_INVALID_ARGUMENT;
    if (M < 1 || N < 1 || K < 1 || N > 256 || K > kTK || (N & 3) || (K & 3)) return RSLRL_E_INVALID_ARGUMENT;
    if (bias_side < 0 || bias_side > 2 || (bias_side == 1 && N <= 64)) return RSLRL_E_INVALID_ARGUMENT;
    const bool h3 = arith == RSLRL_ARITH_H3;
    if (!h3 && arith != RSLRL_ARITH_X6) return RSLRL_E_INVALID_ARGUMENT;
    const rslrl_wgrad_problem_t* a[2] = {a0, a1};
    const size_t need = rslrl_linear_wgrad_bias_pair_workspace_bytes(M, N, K, bias_side);
    for (int i = 0; i < 2; ++i) {
        if (!a[i]->dz || !a[i]->x || !a[i]->dw_db || !a[i]->workspace) return RSLRL_E_INVALID_ARGUMENT;
        if (h3 && (!a[i]->dz_amax || !a[i]->x_amax)) return RSLRL_E_INVALID_ARGUMENT;
        if ((reinterpret_cast<uintptr_t>(a[i]->dz) | reinterpret_cast<uintptr_t>(a[i]->x)) & 15) return RSLRL_E_MISALIGNED;
        if (a[i]->workspace_bytes < need) return RSLRL_E_WORKSPACE_TOO_SMALL;
    }
    const int64_t rows_per = wgrad_pair_rows_per(M, N);
    const int64_t S = ceil_div(M, rows_per);
    const int64_t NKE = static_cast<int64_t>(N) * K + colsum_len(bias_side, N, K);
    const size_t part_bytes = static_cast<size_t>(S) * NKE * sizeof(float);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    WgradPair b{};
    for (int i = 0; i < 2; ++i)
        b.p[i] = WgradParams{a[i]->dz, a[i]->x, static_cast<float*>(a[i]->workspace), M, rows_per, N, K, a[i]->dz_amax,
                             a[i]->x_amax};
    const bool full = (M % rows_per == 0) && K == kTK && (rows_per / kMC) % kWgradDepth == 0;
    const dim3 g(static_cast<unsigned>(S), 2), blk(kThreadsW);
    auto go = [&](auto tn, auto pl, auto cs) {
        constexpr int TN = decltype(tn)::value, PL = decltype(pl)::value, CS = decltype(cs)::value;
        if constexpr (CS == 1 && TN != kTK) {
            return;
        } else {
            if (full && N == TN) hipLaunchKernelGGL((wgrad_x6_pair_kernel<TN, true, PL, false, CS>), g, blk, 0, st, b);
            else if (full && N < TN) hipLaunchKernelGGL((wgrad_x6_pair_kernel<TN, true, PL, true, CS>), g, blk, 0, st, b);
            else hipLaunchKernelGGL((wgrad_x6_pair_kernel<TN, false, PL, false, CS>), g, blk, 0, st, b);
        }
    };
    auto by_side = [&](auto tn, auto pl) {
        using C0 = std::integral_constant<int, 0>;
        using C1 = std::integral_constant<int, 1>;
        using C2 = std::integral_constant<int, 2>;
        if (bias_side == 1) go(tn, pl, C1{});
        else if (bias_side == 2) go(tn, pl, C2{});
        else go(tn, pl, C0{});
    };
    using I32 = std::integral_constant<int, 32>;
    using I64 = std::integral_constant<int, 64>;
    using I256 = std::integral_constant<int, 256>;
    using P2 = std::integral_constant<int, 2>;
    using P3 = std::integral_constant<int, 3>;
    if (N <= 32) h3 ? by_side(I32{}, P2{}) : by_side(I32{}, P3{});
    else if (N <= 64) h3 ? by_side(I64{}, P2{}) : by_side(I64{}, P3{});
    else h3 ? by_side(I256{}, P2{}) : by_side(I256{}, P3{});
    int rc = launch_status();
    if (rc || (flags & RSLRL_WGRAD_NO_FOLD)) return rc;
    for (int i = 0; i < 2; ++i) {
        const bool tr = a[i]->transpose_out != 0;
        rc = rslrl_fold_partials_ex(static_cast<const float*>(a[i]->workspace), S, NKE, a[i]->dw_db, NKE, tr ? N : 0,
                                    tr ? K : 0, static_cast<char*>(a[i]->workspace) + part_bytes,
                                    a[i]->workspace_bytes - part_bytes, stream);
        if (rc) return rc;
    }
    return RSLRL_OK;
}
