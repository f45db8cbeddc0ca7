// Hidden-layer forward H = ELU(X W^T + b) of a square 256-wide layer (rsl_rl/networks/mlp.py:106-114: Linear(256, 256)
// + ELU, the update's forward ppo.py:246-253 and the rollout's policy.act / evaluate ppo.py:155-156) on the x6 split-bf16
// MFMA path, for the actor's and the critic's layer in one launch -- a streaming main loop that keeps the matrix pipe fed
// across tiles (round 5).
//
// The tiled kernel (mlp_gemm.hip deep_pipeline) stages each 16-deep k-chunk of A and B through LDS with a barrier per
// chunk: 16 barriers per 128-row tile, two workgroups per CU contending for the pipes (PMC: MFMA pipe 0.58 busy).
// Here one workgroup per CU (8 waves, 2 per SIMD) runs a slice of consecutive 128-row tiles:
//  * wave w owns output columns [32 w, 32 w + 32) of all 128 rows (4 MFMA blocks, 64 accumulator registers);
//  * B fragments (the W^T x6 image, 384 KiB, L2-resident) go straight from global memory into registers one chunk
//    ahead -- no LDS, no barrier for B;
//  * A (X split into three bf16 planes) streams through two LDS buffers of one K quarter each (4 chunks x 128 rows:
//    48 KiB): while the waves run the MFMAs of quarter s from one buffer, each thread splits its share of quarter s + 1
//    (loaded into registers one quarter earlier) into the other buffer -- one barrier per quarter (4 per tile), the
//    split's VALU and LDS writes beside the MFMAs instead of in a phase of their own;
//  * epilogue per tile: + b, ELU (epilogue_tiles_impl's expression: the same bits), nontemporal 4-byte stores whose
//    64 lanes cover two whole 128-byte rows.
// The accumulation order of every output is the tiled kernel's (chunks 0..15, the six products of mfma_x6 in order):
// H is bit-identical to RSLRL_LINEAR_FWD_ELU's x6 kernel.
//
// LDS image of a quarter buffer plane: [4 chunks][128 row slots][32 bytes], row m of chunk c in slot m ^ f(c),
// f(c) = (c & 3) | 4 (c & 1), 16-byte halves swapped when (m >> 3) & 1 (mlp_bwd_fused.hip's plane layout with 128
// rows): conflict-free for the ds_read_b128 row fragments and the split's ds_write_b64 (16 lanes = one row of 4 chunks).
#include "common.h"
#include "fwd_stream.h"
#include "x6_split.h"

namespace rslrl {
namespace {

constexpr int kFsT = 128;                  // rows per tile
constexpr int kFsW = 256;                  // K = N = 256
constexpr int kFsThreads = 512;            // 8 waves
constexpr int kFsQChunks = 4;              // chunks per K quarter
constexpr int kFsChunkB = kFsT * 32;       // one chunk of one plane: 4 KiB
constexpr int kFsPlaneB = kFsQChunks * kFsChunkB;  // 16 KiB
constexpr int kFsBufB = 3 * kFsPlaneB;     // 48 KiB per quarter buffer
constexpr int kFsMaxSlices = 128;          // per problem: a pair fills the 256 CUs with one workgroup each
constexpr int kFsImgPlaneU = kFsW * 32 / 16;  // 16-byte units of one plane of one image chunk (bimage layout 0)
constexpr int kFsImgChunkU = 3 * kFsImgPlaneU;
constexpr uint32_t kFsRsrcFlags = 0x00020000;
#ifndef RSLRL_FS_LA
#define RSLRL_FS_LA 1
#endif
constexpr bool kFsLA = RSLRL_FS_LA != 0;  // A fragments one MFMA block ahead (A/B: 688-693 vs 697-721 us, r5_fs_ab.json)

struct FsProblem {
    const float* x;     // [M, 256]
    const uint4* img;   // x6 image of W (layout 0, 16 chunks)
    const float* bias;  // [256]
    float* h;           // [M, 256]
};

struct FsArgs {
    FsProblem p[2];
    int tiles;      // M / 128
    int tiles_per;  // tiles per slice
};

__host__ __device__ constexpr int fs_f(int c) { return (c & 3) | ((c & 1) << 2); }

// byte offset of (row m, column col % 4 == 0 of the quarter) in a plane of a quarter buffer
__device__ __forceinline__ int fs_off(int m, int col) {
    const int c = col >> 4;
    return c * kFsChunkB + (m ^ fs_f(c)) * 32 + 16 * (((col >> 3) & 1) ^ ((m >> 3) & 1)) + 8 * ((col >> 2) & 1);
}

__device__ __forceinline__ bf16x8 fs_read16(int addr) {
    typedef __attribute__((address_space(3))) uint4 lds_u4;
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const lds_u4*>(addr));
}

// the tile's X columns [64 q, 64 q + 64): 4 float4 per thread, row (t >> 4) + 32 j, columns 64 q + 4 (t & 15) .. + 3
__device__ __forceinline__ void fs_load_x(__amdgpu_buffer_rsrc_t r, int q, float4 (&v)[4]) {
    const int off = ((threadIdx.x >> 4) * kFsW + 4 * (threadIdx.x & 15)) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        v[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, j * 32 * kFsW * 4 + q * 256, 2));
}

// unit j of the thread's share: split into the three planes of a quarter buffer
__device__ __forceinline__ void fs_store_x1(const float4& v, int j, char* __restrict__ buf) {
    uint2 w[3];
    split4(v, w[0], w[1], w[2]);
    const int off = fs_off((threadIdx.x >> 4) + 32 * j, 4 * (threadIdx.x & 15));
#pragma unroll
    for (int q = 0; q < 3; ++q) *reinterpret_cast<uint2*>(buf + q * kFsPlaneB + off) = w[q];
}

__device__ __forceinline__ void fs_store_x(const float4 (&v)[4], char* __restrict__ buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) fs_store_x1(v[j], j, buf);
}

__device__ __forceinline__ float fs_elu_neg(float v) {  // mlp_gemm.hip elu_neg: the same expression
    float t = __fmaf_rn(v, 2.7557319e-6f, 2.4801587e-5f);
    t = __fmaf_rn(v, t, 1.9841270e-4f);
    t = __fmaf_rn(v, t, 1.3888889e-3f);
    t = __fmaf_rn(v, t, 8.3333333e-3f);
    t = __fmaf_rn(v, t, 4.1666667e-2f);
    t = __fmaf_rn(v, t, 1.6666667e-1f);
    t = __fmaf_rn(v, t, 0.5f);
    t = __fmaf_rn(v, t, 1.0f);
    const float poly = v * t;
    const float e = __expf(v) - 1.0f;
    return v > -0.5f ? poly : e;
}

__global__ __launch_bounds__(kFsThreads, 1) void fwd_stream_kernel(FsArgs args) {
    __shared__ __attribute__((aligned(16))) char lds[2 * kFsBufB];
    const FsProblem& P = args.p[blockIdx.y];
    const int t_begin = blockIdx.x * args.tiles_per;
    const int t_end = min(args.tiles, t_begin + args.tiles_per);
    if (t_begin >= t_end) return;

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);  // static priority for the second-dispatched half (MI355X_MICROARCH)
    const int h = lane >> 5;
    const int l32 = lane & 31;

    // A fragment lane addresses: fs_off(32 i + l32, 16 c + 8 h) = la[c] + i * 1 KiB (+ plane, + buffer)
    const int lbase = static_cast<int>(reinterpret_cast<uintptr_t>(lds));
    int la[2][4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        la[0][c] = lbase + fs_off(l32, 16 * c + 8 * h);
        la[1][c] = la[0][c] + kFsBufB;
    }
    // B fragments: image row 32 w + l32 (output column), half h, swizzled as the image stores it
    const int brow = 32 * wave + l32;
    const int boff = (brow * 2 + (h ^ ((brow >> 3) & 1))) * 16;
    const __amdgpu_buffer_rsrc_t rimg = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint4*>(P.img), 0, static_cast<uint32_t>(16 * kFsImgChunkU * 16), kFsRsrcFlags);
    auto bload = [&](int c, int q) {
        return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rimg, boff, (c * kFsImgChunkU + q * kFsImgPlaneU) * 16, 0));
    };
    const float bias = P.bias[32 * wave + l32];

    auto tile_rsrc = [&](int tile) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(P.x + static_cast<int64_t>(tile) * kFsT * kFsW), 0,
                                                 static_cast<uint32_t>(kFsT * kFsW * 4), kFsRsrcFlags);
    };

    // prologue: quarter 0 split into buffer 0, quarter 1 in registers
    float4 xr[4];
    fs_load_x(tile_rsrc(t_begin), 0, xr);
    fs_store_x(xr, lds);
    fs_load_x(tile_rsrc(t_begin), 1, xr);
    __syncthreads();

    uint4 bq[2][3];
#pragma unroll
    for (int q = 0; q < 3; ++q) bq[0][q] = bload(0, q);

    // epilogue part e (0..15) of a finished tile's accumulators: values 4 (e & 3) .. + 3 of row block e >> 2 -> + b,
    // ELU, nontemporal stores (lane: column 32 w + l32, rows 32 i + 4 h + (r & 3) + 8 (r >> 2))
    auto epi_part = [&](const f32x16 (&acc)[4], int tile, int e) {
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
            P.h + static_cast<int64_t>(tile) * kFsT * kFsW + 32 * wave, 0, static_cast<uint32_t>(kFsT * kFsW * 4),
            kFsRsrcFlags);
        const int i = e >> 2;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int r = 4 * (e & 3) + k;
            float v = acc[i][r] + bias;
            const float n = fs_elu_neg(fminf(v, 0.f));
            v = v > 0.f ? v : n;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rc, ((4 * h + (r & 3)) * kFsW + l32) * 4,
                                                  (32 * i + 8 * (r >> 2)) * kFsW * 4, 2 /* nt */);
        }
    };

    // One tile into acc; the previous tile's epilogue (prev, when has_prev) spread over the first quarter's 16 MFMA
    // blocks, 4 values after each, beside the MFMAs.  Two accumulator sets alternate by tile parity.
    auto run_tile = [&](int tile, f32x16 (&acc)[4], const f32x16 (&prev)[4], bool has_prev) {
        const bool more = tile + 1 < t_end;
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) {  // quarter s = 4 (tile - t_begin) + kq lives in buffer kq & 1
            const int buf = kq & 1;
            bf16x8 an[3];
            if constexpr (kFsLA) {
                an[0] = fs_read16(la[buf][0]);
                an[1] = fs_read16(la[buf][0] + kFsPlaneB);
                an[2] = fs_read16(la[buf][0] + 2 * kFsPlaneB);
            }
#pragma unroll
            for (int c = 0; c < kFsQChunks; ++c) {
                const int gc = 4 * kq + c;  // chunk of the tile
                // the image chunk after this one (the next tile's chunk 0 after chunk 15)
#pragma unroll
                for (int q = 0; q < 3; ++q) bq[(c + 1) & 1][q] = bload((gc + 1) & 15, q);
                bf16x8 bf[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) bf[q] = __builtin_bit_cast(bf16x8, bq[c & 1][q]);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    bf16x8 af[3];
                    if constexpr (kFsLA) {
                        // the fragments of block (c, i) were read during the previous block; read the next one's now
                        // (not across the quarter's barrier: block (0, 0) is read at the quarter's start)
#pragma unroll
                        for (int q = 0; q < 3; ++q) af[q] = an[q];
                        if (4 * c + i + 1 < 16) {
                            const int cn = (4 * c + i + 1) >> 2, in = (4 * c + i + 1) & 3;
                            const int a1 = la[buf][cn] + in * 1024;
                            an[0] = fs_read16(a1);
                            an[1] = fs_read16(a1 + kFsPlaneB);
                            an[2] = fs_read16(a1 + 2 * kFsPlaneB);
                        }
                    } else {
                        const int a0 = la[buf][c] + i * 1024;
                        af[0] = fs_read16(a0);
                        af[1] = fs_read16(a0 + kFsPlaneB);
                        af[2] = fs_read16(a0 + 2 * kFsPlaneB);
                    }
                    // chunk 0 starts from zero accumulators: the same bits as accumulating onto zeros
                    acc[i] = mfma_x6(af, bf, gc == 0 ? f32x16{} : acc[i]);
                    if (kq == 0 && has_prev) epi_part(prev, tile - 1, 4 * c + i);
                    // quarter s + 1 into the other buffer, one unit after each of chunk 1's MFMA blocks (the buffer
                    // was last read in quarter s - 1 and every wave passed the barrier after it)
                    if (c == 1 && (kq < 3 || more)) fs_store_x1(xr[i], i, lds + (buf ^ 1) * kFsBufB);
                    __builtin_amdgcn_sched_barrier(0);
                }
                // quarter s + 2 into the registers after chunk 3's B load.  Loads return in issue order: a B fragment
                // issued after them waits for them, so they go out where the next such wait is two chunks away.
                if (c == 3 && (kq < 2 || more)) {
                    fs_load_x(tile_rsrc(kq < 2 ? tile : tile + 1), (kq + 2) & 3, xr);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            __syncthreads();  // the other buffer holds quarter s + 1; this one may be overwritten
        }
    };

    f32x16 acc0[4], acc1[4];
    int tile = t_begin;
    for (; tile + 1 < t_end; tile += 2) {
        run_tile(tile, acc0, acc1, tile > t_begin);
        run_tile(tile + 1, acc1, acc0, true);
    }
    if (tile < t_end) {  // an odd tile count: the last tile in acc0, after acc1's tile (if any)
        run_tile(tile, acc0, acc1, tile > t_begin);
#pragma unroll
        for (int e = 0; e < 16; ++e) epi_part(acc0, tile, e);
    } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) epi_part(acc1, tile - 1, e);
    }
}

int64_t fs_tiles_per(int64_t tiles) { return ceil_div(tiles, std::min<int64_t>(kFsMaxSlices, tiles)); }

}  // namespace

bool fwd_stream_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("RSLRL_FWD_STREAM");
        return !(e && e[0] == '0');
    }();
    return on;
}

int fwd_stream_pair(const FwdStreamProblem* p, int n, int64_t M, hipStream_t st) {
    if (n < 1 || n > 2 || M <= 0 || M % kFsT || M / kFsT > INT32_MAX) return RSLRL_E_UNSUPPORTED;
    FsArgs args{};
    for (int i = 0; i < n; ++i) {
        const uintptr_t bits = reinterpret_cast<uintptr_t>(p[i].x) | reinterpret_cast<uintptr_t>(p[i].img);
        if (!p[i].x || !p[i].img || !p[i].bias || !p[i].h) return RSLRL_E_INVALID_ARGUMENT;
        if (bits & 15) return RSLRL_E_MISALIGNED;
        args.p[i] = FsProblem{p[i].x, static_cast<const uint4*>(p[i].img), p[i].bias, p[i].h};
    }
    const int64_t tiles = M / kFsT;
    const int64_t per = fs_tiles_per(tiles);
    args.tiles = static_cast<int>(tiles);
    args.tiles_per = static_cast<int>(per);
    const dim3 grid(static_cast<unsigned>(ceil_div(tiles, per)), static_cast<unsigned>(n));
    hipLaunchKernelGGL(fwd_stream_kernel, grid, dim3(kFsThreads), 0, st, args);
    return launch_status();
}

}  // namespace rslrl
