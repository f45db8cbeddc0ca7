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
#include <cstring>

#include "common.h"
#include "fwd_stream.h"
#include "ppo_loss_common.h"
#include "x6_split.h"

namespace rslrl {
namespace {

constexpr int kFsT = 128;                  // rows per tile
constexpr int kFsN = 256;                  // output width
constexpr int kFsThreads = 512;            // 8 waves
constexpr int kFsChunkB = kFsT * 32;       // one chunk of one plane of a stage buffer: 4 KiB
constexpr int kFsMaxSlices = 128;          // per problem: a pair fills the 256 CUs with one workgroup each
constexpr int kFsImgPlaneU = kFsN * 32 / 16;  // 16-byte units of one plane of one image chunk (bimage layout 0)
constexpr int kFsImgChunkU = 3 * kFsImgPlaneU;
constexpr uint32_t kFsRsrcFlags = 0x00020000;
#ifndef RSLRL_FS_LA
#define RSLRL_FS_LA 1
#endif
constexpr bool kFsLA = RSLRL_FS_LA != 0;  // A fragments one MFMA block ahead (A/B: 688-693 vs 697-721 us, r5_fs_ab.json)

// K = 256: four stages (K quarters) of 4 chunks per tile; K = 48 (the first layer): one stage of 3 chunks per tile
template <int K>
struct FsCfg {
    static constexpr int kChunks = K / 16;                   // chunks of the tile
    static constexpr int kStages = K == 256 ? 4 : 1;         // stages per tile
    static constexpr int kNch = kChunks / kStages;           // chunks per stage
    static constexpr int kCols = 16 * kNch;                  // columns of X per stage
    static constexpr int kPlaneB = kNch * kFsChunkB;         // one plane of a stage buffer
    static constexpr int kBufB = 3 * kPlaneB;                // 48 KiB (K = 256) / 36 KiB (K = 48)
    static constexpr int kUnitsRow = kCols / 4;              // 16-byte units of a row's stage columns
    static constexpr int kUpt = kFsT * kUnitsRow / kFsThreads;  // units per thread per stage: 4 / 3
    static_assert(K == 256 || K == 48, "streaming forward: K = 256 or 48");
    static_assert(kNch >= 2 && kUpt <= 4 && kFsT * kUnitsRow % kFsThreads == 0, "stage shape");
};

struct FsProblem {
    const float* x;     // [M, K]
    const uint4* img;   // x6 image of W (layout 0, K / 16 chunks)
    const float* bias;  // [256]
    float* h;           // [M, 256]
};

struct FsArgs {
    FsProblem p[2];
    int tiles;      // M / 128
    int tiles_per;  // tiles per slice
};

__host__ __device__ constexpr int fs_f(int c) { return (c & 3) | ((c & 1) << 2); }

// byte offset of (row m, column col % 4 == 0 of the stage) in a plane of a stage buffer
__device__ __forceinline__ int fs_off(int m, int col) {
    const int c = col >> 4;
    return c * kFsChunkB + (m ^ fs_f(c)) * 32 + 16 * (((col >> 3) & 1) ^ ((m >> 3) & 1)) + 8 * ((col >> 2) & 1);
}

__device__ __forceinline__ bf16x8 fs_read16(int addr) {
    typedef __attribute__((address_space(3))) uint4 lds_u4;
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const lds_u4*>(addr));
}

// stage q of the tile's X: unit u = t + 512 j (j < kUpt) is row u / kUnitsRow, columns kCols q + 4 (u % kUnitsRow)
template <int K>
__device__ __forceinline__ void fs_load_x(__amdgpu_buffer_rsrc_t r, int q, float4 (&v)[4]) {
    using C = FsCfg<K>;
#pragma unroll
    for (int j = 0; j < C::kUpt; ++j) {
        const int u = threadIdx.x + kFsThreads * j;
        const int off = ((u / C::kUnitsRow) * K + 4 * (u % C::kUnitsRow)) * 4;
        v[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, q * C::kCols * 4, 2));
    }
}

// unit j of the thread's share of a stage: split into the three planes of a stage buffer
template <int K>
__device__ __forceinline__ void fs_store_x1(const float4& v, int j, char* __restrict__ buf) {
    using C = FsCfg<K>;
    uint2 w[3];
    split4(v, w[0], w[1], w[2]);
    const int u = threadIdx.x + kFsThreads * j;
    const int off = fs_off(u / C::kUnitsRow, 4 * (u % C::kUnitsRow));
#pragma unroll
    for (int q = 0; q < 3; ++q) *reinterpret_cast<uint2*>(buf + q * C::kPlaneB + off) = w[q];
}

__device__ __forceinline__ float fs_elu_neg(float v) {  // mlp_gemm.hip elu_neg: the same expression
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

template <int K>
__global__ __launch_bounds__(kFsThreads, 1) void fwd_stream_kernel(FsArgs args) {
    using C = FsCfg<K>;
    __shared__ __attribute__((aligned(16))) char lds[2 * C::kBufB];
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
    int la[2][C::kNch];
#pragma unroll
    for (int c = 0; c < C::kNch; ++c) {
        la[0][c] = lbase + fs_off(l32, 16 * c + 8 * h);
        la[1][c] = la[0][c] + C::kBufB;
    }
    // B fragments: image row 32 w + l32 (output column), half h, swizzled as the image stores it
    const int brow = 32 * wave + l32;
    const int boff = (brow * 2 + (h ^ ((brow >> 3) & 1))) * 16;
    const __amdgpu_buffer_rsrc_t rimg = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint4*>(P.img), 0, static_cast<uint32_t>(C::kChunks * kFsImgChunkU * 16), kFsRsrcFlags);
    auto bload = [&](int c, int q) {
        return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rimg, boff, (c * kFsImgChunkU + q * kFsImgPlaneU) * 16, 0));
    };
    const float bias = P.bias[32 * wave + l32];

    auto tile_rsrc = [&](int tile) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(P.x + static_cast<int64_t>(tile) * kFsT * K), 0,
                                                 static_cast<uint32_t>(kFsT * K * 4), kFsRsrcFlags);
    };

    // prologue: stage 0 split into buffer 0, stage 1 (the next tile's stage 0 when a tile is one stage) in registers
    float4 xr[4];
    fs_load_x<K>(tile_rsrc(t_begin), 0, xr);
#pragma unroll
    for (int j = 0; j < C::kUpt; ++j) fs_store_x1<K>(xr[j], j, lds);
    if (C::kStages > 1) fs_load_x<K>(tile_rsrc(t_begin), 1, xr);
    else if (t_begin + 1 < t_end) fs_load_x<K>(tile_rsrc(t_begin + 1), 0, xr);
    __syncthreads();

    uint4 bq[2][3];
#pragma unroll
    for (int q = 0; q < 3; ++q) bq[0][q] = bload(0, q);

    // epilogue part e (0..15) of a finished tile's accumulators: values 4 (e & 3) .. + 3 of row block e >> 2 -> + b,
    // ELU, nontemporal stores (lane: column 32 w + l32, rows 32 i + 4 h + (r & 3) + 8 (r >> 2))
    auto epi_part = [&](const f32x16 (&acc)[4], int tile, int e) {
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
            P.h + static_cast<int64_t>(tile) * kFsT * kFsN + 32 * wave, 0, static_cast<uint32_t>(kFsT * kFsN * 4),
            kFsRsrcFlags);
        const int i = e >> 2;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int r = 4 * (e & 3) + k;
            float v = acc[i][r] + bias;
            const float n = fs_elu_neg(fminf(v, 0.f));
            v = v > 0.f ? v : n;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rc, ((4 * h + (r & 3)) * kFsN + l32) * 4,
                                                  (32 * i + 8 * (r >> 2)) * kFsN * 4, 2 /* nt */);
        }
    };

    // One tile into acc; the previous tile's epilogue (prev, when has_prev) spread over the first stage's MFMA blocks,
    // one part after each (the rest after the stage's last block), beside the MFMAs.  Two accumulator sets alternate by
    // tile parity.  Stage s = kStages (tile - t_begin) + kq lives in buffer s & 1.
    // par: the tile's parity from t_begin (a literal at each call: the buffers' indices fold into immediates)
    auto run_tile = [&](int tile, f32x16 (&acc)[4], const f32x16 (&prev)[4], bool has_prev, int par) {
        const bool more = tile + 1 < t_end;
#pragma unroll
        for (int kq = 0; kq < C::kStages; ++kq) {
            const int buf = (C::kStages % 2 == 0) ? (kq & 1) : (par ^ (kq & 1));
            bf16x8 an[3];
            if constexpr (kFsLA) {
                an[0] = fs_read16(la[buf][0]);
                an[1] = fs_read16(la[buf][0] + C::kPlaneB);
                an[2] = fs_read16(la[buf][0] + 2 * C::kPlaneB);
            }
            const bool next_stage = kq + 1 < C::kStages || more;   // a stage follows this one
#pragma unroll
            for (int c = 0; c < C::kNch; ++c) {
                const int gc = C::kNch * kq + c;  // chunk of the tile
                // the image chunk after this one (the next tile's chunk 0 after the last)
                // ring slot of this chunk: chunks alternate over the whole slice (a tile of 3 chunks flips it)
                const int slot = (par * C::kChunks + gc) & 1;
#pragma unroll
                for (int q = 0; q < 3; ++q) bq[slot ^ 1][q] = bload((gc + 1) % C::kChunks, q);
                bf16x8 bf[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) bf[q] = __builtin_bit_cast(bf16x8, bq[slot][q]);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int blk = 4 * c + i;  // block of the stage
                    bf16x8 af[3];
                    if constexpr (kFsLA) {
                        // the fragments of block (c, i) were read during the previous block; read the next one's now
                        // (not across the stage's barrier: block (0, 0) is read at the stage's start)
#pragma unroll
                        for (int q = 0; q < 3; ++q) af[q] = an[q];
                        if (blk + 1 < 4 * C::kNch) {
                            const int a1 = la[buf][(blk + 1) >> 2] + ((blk + 1) & 3) * 1024;
                            an[0] = fs_read16(a1);
                            an[1] = fs_read16(a1 + C::kPlaneB);
                            an[2] = fs_read16(a1 + 2 * C::kPlaneB);
                        }
                    } else {
                        const int a0 = la[buf][c] + i * 1024;
                        af[0] = fs_read16(a0);
                        af[1] = fs_read16(a0 + C::kPlaneB);
                        af[2] = fs_read16(a0 + 2 * C::kPlaneB);
                    }
                    // chunk 0 starts from zero accumulators: the same bits as accumulating onto zeros
                    acc[i] = mfma_x6(af, bf, gc == 0 ? f32x16{} : acc[i]);
                    if (kq == 0 && has_prev) {
                        if (blk < 16) epi_part(prev, tile - 1, blk);
                        if (blk == 4 * C::kNch - 1) {
#pragma unroll
                            for (int e = 4 * C::kNch; e < 16; ++e) epi_part(prev, tile - 1, e);
                        }
                    }
                    // stage s + 1 into the other buffer, one unit after each of chunk 1's MFMA blocks (that buffer was
                    // last read in stage s - 1 and every wave passed the barrier after it)
                    if (c == 1 && i < C::kUpt && next_stage) fs_store_x1<K>(xr[i], i, lds + (buf ^ 1) * C::kBufB);
                    __builtin_amdgcn_sched_barrier(0);
                }
                // stage s + 2 into the registers after the last chunk's B load.  Loads return in issue order: a B
                // fragment issued after them waits for them, so they go out where the next such wait is a chunk away.
                if (c == C::kNch - 1) {
                    if (C::kStages > 1) {
                        if (kq < C::kStages - 2 || more) {
                            const int s2 = kq + 2;
                            fs_load_x<K>(tile_rsrc(s2 < C::kStages ? tile : tile + 1), s2 % C::kStages, xr);
                        }
                    } else if (tile + 2 < t_end) {
                        fs_load_x<K>(tile_rsrc(tile + 2), 0, xr);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            __syncthreads();  // the other buffer holds stage s + 1; this one may be overwritten
        }
    };

    f32x16 acc0[4], acc1[4];
    int tile = t_begin;
    for (; tile + 1 < t_end; tile += 2) {
        run_tile(tile, acc0, acc1, tile > t_begin, 0);
        run_tile(tile + 1, acc1, acc0, true, 1);
    }
    if (tile < t_end) {  // an odd tile count: the last tile in acc0, after acc1's tile (if any)
        run_tile(tile, acc0, acc1, tile > t_begin, 0);
#pragma unroll
        for (int e = 0; e < 16; ++e) epi_part(acc0, tile, e);
    } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) epi_part(acc1, tile - 1, e);
    }
}


// ---- The critic's head on the streaming main loop (round 5; RSLRL_VALUE_HEAD_STREAM=0 keeps the tiled head) --------
// rslrl_value_head_fwd_bwd's computation -- H = ELU(X W^T + b) of the last hidden layer, V = H w_v + b_v, dV = d(value
// loss)/dV (value_loss_grad: the loss kernel's expression), dZ = (dV w_v) * ELU'(H) and the head's [dW | db] -- with
// the main loop of fwd_stream_kernel<256> on C^T accumulators (lane: row 32 i + l32, columns 8 g + 4 h + k of the
// wave's 32; the tiled value head's orientation and MFMA order, so H has its bits).  V sums each wave's 32 columns
// (16 per lane in one fma chain, then the other lane half) and the 8 waves in order: a different association than the
// tiled head's 4 x 64 columns (fp32 reassociation; V, dV and dZ agree to rounding).  The [dW | db] partials are one
// row per slice (rows = rslrl_value_head_stream_rows(M)), accumulated in registers across the slice's tiles.
struct VhArgs {
    const float* x;      // [M, 256] the critic's last hidden input
    const uint4* img;    // x6 image of W (layout 0)
    const float* bias;   // [256]
    const float* wv;     // [256] value weights
    float bv;            // value bias (read by the host from nothing: passed as a device pointer below)
    const float* bvp;    // [1] value bias (device)
    const float* tv;     // [M] target values
    const float* ret;    // [M] returns
    float* dz;           // [M, 256]
    float* y;            // [M] values
    float* wpart;        // [slices][kVhP]
    float clip, g;
    int clipped;
    int tiles, tiles_per;
};
constexpr int kVhP = 260;  // [dW (256) | db | pad 3]

__global__ __launch_bounds__(kFsThreads, 1) void value_head_stream_kernel(VhArgs a) {
    using C = FsCfg<256>;
    __shared__ __attribute__((aligned(16))) char lds[2 * C::kBufB];
    __shared__ float red[8 * kFsT];   // per wave: its 32 columns' share of V, per row
    __shared__ float dvl[kFsT];       // dV per row
    __shared__ float dbred[kFsT / 64];
    const int t_begin = blockIdx.x * a.tiles_per;
    const int t_end = min(a.tiles, t_begin + a.tiles_per);
    if (t_begin >= t_end) return;

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    const int h = lane >> 5;
    const int l32 = lane & 31;

    const int lbase = static_cast<int>(reinterpret_cast<uintptr_t>(lds));
    int la[2][C::kNch];
#pragma unroll
    for (int c = 0; c < C::kNch; ++c) {
        la[0][c] = lbase + fs_off(l32, 16 * c + 8 * h);
        la[1][c] = la[0][c] + C::kBufB;
    }
    const int brow = 32 * wave + l32;
    const int boff = (brow * 2 + (h ^ ((brow >> 3) & 1))) * 16;
    const __amdgpu_buffer_rsrc_t rimg = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint4*>(a.img), 0, static_cast<uint32_t>(C::kChunks * kFsImgChunkU * 16), kFsRsrcFlags);
    auto bload = [&](int c, int q) {
        return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rimg, boff, (c * kFsImgChunkU + q * kFsImgPlaneU) * 16, 0));
    };
    // this lane's 16 columns 32 w + 8 g + 4 h + k (r = 4 g + k): bias and value weights, fixed for the slice
    float bcol[16], wcol[16];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const float4 b4 = *reinterpret_cast<const float4*>(a.bias + 32 * wave + 8 * g + 4 * h);
        const float4 w4 = *reinterpret_cast<const float4*>(a.wv + 32 * wave + 8 * g + 4 * h);
        bcol[4 * g] = b4.x; bcol[4 * g + 1] = b4.y; bcol[4 * g + 2] = b4.z; bcol[4 * g + 3] = b4.w;
        wcol[4 * g] = w4.x; wcol[4 * g + 1] = w4.y; wcol[4 * g + 2] = w4.z; wcol[4 * g + 3] = w4.w;
    }
    const float bv = *a.bvp;
    auto tile_rsrc = [&](int tile) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x + static_cast<int64_t>(tile) * kFsT * 256), 0,
                                                 static_cast<uint32_t>(kFsT * 256 * 4), kFsRsrcFlags);
    };

    float4 xr[4];
    fs_load_x<256>(tile_rsrc(t_begin), 0, xr);
#pragma unroll
    for (int j = 0; j < C::kUpt; ++j) fs_store_x1<256>(xr[j], j, lds);
    fs_load_x<256>(tile_rsrc(t_begin), 1, xr);
    __syncthreads();

    uint4 bq[2][3];
#pragma unroll
    for (int q = 0; q < 3; ++q) bq[0][q] = bload(0, q);

    float wacc[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) wacc[r] = 0.f;
    float dbacc = 0.f;  // threads < 128: this row position's dV over the slice's tiles

    for (int tile = t_begin; tile < t_end; ++tile) {
        const bool more = tile + 1 < t_end;
        const int64_t row0 = static_cast<int64_t>(tile) * kFsT;
        f32x16 acc[4];
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) {
            const int buf = kq & 1;
            bf16x8 an[3];
            an[0] = fs_read16(la[buf][0]);
            an[1] = fs_read16(la[buf][0] + C::kPlaneB);
            an[2] = fs_read16(la[buf][0] + 2 * C::kPlaneB);
#pragma unroll
            for (int c = 0; c < C::kNch; ++c) {
                const int gc = C::kNch * kq + c;
                const int slot = gc & 1;
#pragma unroll
                for (int q = 0; q < 3; ++q) bq[slot ^ 1][q] = bload((gc + 1) % C::kChunks, q);
                bf16x8 bf[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) bf[q] = __builtin_bit_cast(bf16x8, bq[slot][q]);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int blk = 4 * c + i;
                    bf16x8 af[3];
#pragma unroll
                    for (int q = 0; q < 3; ++q) af[q] = an[q];
                    if (blk + 1 < 4 * C::kNch) {
                        const int a1 = la[buf][(blk + 1) >> 2] + ((blk + 1) & 3) * 1024;
                        an[0] = fs_read16(a1);
                        an[1] = fs_read16(a1 + C::kPlaneB);
                        an[2] = fs_read16(a1 + 2 * C::kPlaneB);
                    }
                    // C^T: the weight fragment is the A operand (rows = output columns)
                    acc[i] = mfma_x6(bf, af, gc == 0 ? f32x16{} : acc[i]);
                    if (c == 1 && i < C::kUpt && (kq < 3 || more)) fs_store_x1<256>(xr[i], i, lds + (buf ^ 1) * C::kBufB);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (c == C::kNch - 1) {
                    if (kq < 2 || more) fs_load_x<256>(tile_rsrc(kq < 2 ? tile : tile + 1), (kq + 2) & 3, xr);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            __syncthreads();
        }
        // ---- the head's epilogue (the next tile's first quarter is in buffer 0 already)
        float tvr = 0.f, retr = 0.f;
        if (threadIdx.x < kFsT) {
            tvr = a.tv[row0 + threadIdx.x];
            retr = a.ret[row0 + threadIdx.x];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float oval = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float tt = acc[i][r] + bcol[r];
                const float n = fs_elu_neg(fminf(tt, 0.f));
                const float hv = tt > 0.f ? tt : n;
                acc[i][r] = hv;
                oval = fmaf(hv, wcol[r], oval);
            }
            const float tsum = oval + __shfl_xor(oval, 32, 64);
            if (h == 0) red[wave * kFsT + 32 * i + l32] = tsum;
        }
        __syncthreads();
        if (threadIdx.x < kFsT) {
            const int rl = threadIdx.x;
            float V = red[rl];
#pragma unroll
            for (int w = 1; w < 8; ++w) V += red[w * kFsT + rl];
            V += bv;
            a.y[row0 + rl] = V;
            const float dV = value_loss_grad(V, tvr, retr, a.clipped, a.clip, a.g);
            dvl[rl] = dV;
            dbacc += dV;
        }
        __syncthreads();
        float* dzt = a.dz + row0 * 256 + 32 * wave + 4 * h;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float dv = dvl[32 * i + l32];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                float o[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int r = 4 * g + k;
                    const float hh = acc[i][r];
                    const float z = __fmaf_rn(dv, wcol[r], 0.f);  // out_bwd_valu_body's fma chain of one term
                    o[k] = hh > 0.f ? z : z * (hh + 1.f);          // ELU'(x) = 1 if h > 0 else h + 1
                    wacc[r] = fmaf(dv, hh, wacc[r]);
                }
                // plain (write-back) stores: the four 32-byte pieces of a row's line from this wave's 4 g steps merge
                // in L2 (nontemporal ones reach HBM as partial-line writes: 571 vs 418 us measured)
                const f32x4 ov = {o[0], o[1], o[2], o[3]};
                *reinterpret_cast<f32x4*>(dzt + (32 * i + l32) * 256 + 8 * g) = ov;
            }
        }
        // dvl / red are rewritten only after the next tile's four quarter barriers (a one-barrier form in which every
        // lane finishes V / dV of its own rows measured slower: 347-353 vs 340-342 us, the 16-fold redundant tail)
    }
    // ---- the slice's partial row: dW over the 32 row lanes (fixed butterfly), db over the 128 row positions
    float* wp = a.wpart + static_cast<int64_t>(blockIdx.x) * kVhP;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        float v = wacc[r];
#pragma unroll
        for (int off = 1; off < 32; off <<= 1) v += __shfl_xor(v, off, 64);
        wacc[r] = v;
    }
    if (l32 == 0) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(wp + 32 * wave + 8 * g + 4 * h) =
                make_float4(wacc[4 * g], wacc[4 * g + 1], wacc[4 * g + 2], wacc[4 * g + 3]);
    }
    if (threadIdx.x < kFsT) {
        float v = dbacc;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
        if (lane == 0) dbred[wave] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        wp[256] = dbred[0] + dbred[1];
        wp[257] = 0.f;
        wp[258] = 0.f;
        wp[259] = 0.f;
    }
}

int64_t fs_tiles_per(int64_t tiles) { return ceil_div(tiles, std::min<int64_t>(kFsMaxSlices, tiles)); }

}  // namespace

bool fwd_stream_forced() {  // RSLRL_FWD_STREAM=1 or 48: every eligible M (tests, A/B)
    static const bool on = [] {
        const char* e = std::getenv("RSLRL_FWD_STREAM");
        return e && (std::strcmp(e, "1") == 0 || std::strcmp(e, "48") == 0);
    }();
    return on;
}

bool fwd_stream48() {
    static const bool on = [] {
        const char* e = std::getenv("RSLRL_FWD_STREAM");
        return e && std::strcmp(e, "48") == 0;
    }();
    return on;
}

bool fwd_stream_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("RSLRL_FWD_STREAM");
        return !(e && e[0] == '0');
    }();
    return on;
}

int fwd_stream_pair(const FwdStreamProblem* p, int n, int64_t M, int K, hipStream_t st) {
    if (n < 1 || n > 2 || M <= 0 || M % kFsT || M / kFsT > INT32_MAX || (K != 256 && K != 48))
        return RSLRL_E_UNSUPPORTED;
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
    if (K == 256) hipLaunchKernelGGL(fwd_stream_kernel<256>, grid, dim3(kFsThreads), 0, st, args);
    else hipLaunchKernelGGL(fwd_stream_kernel<48>, grid, dim3(kFsThreads), 0, st, args);
    return launch_status();
}


int value_head_stream(const ValueHeadStreamArgs& v, hipStream_t st) {
    if (v.M <= 0 || v.M % kFsT || v.M / kFsT > INT32_MAX) return RSLRL_E_UNSUPPORTED;
    const uintptr_t bits = reinterpret_cast<uintptr_t>(v.x) | reinterpret_cast<uintptr_t>(v.img) |
                           reinterpret_cast<uintptr_t>(v.bias) | reinterpret_cast<uintptr_t>(v.wv) |
                           reinterpret_cast<uintptr_t>(v.dz) | reinterpret_cast<uintptr_t>(v.wpart);
    if (bits & 15) return RSLRL_E_MISALIGNED;
    const int64_t tiles = v.M / kFsT;
    const int64_t per = ceil_div(tiles, std::min<int64_t>(2 * kFsMaxSlices, tiles));
    VhArgs a{};
    a.x = v.x;
    a.img = static_cast<const uint4*>(v.img);
    a.bias = v.bias;
    a.wv = v.wv;
    a.bvp = v.bv;
    a.tv = v.tv;
    a.ret = v.ret;
    a.dz = v.dz;
    a.y = v.y;
    a.wpart = v.wpart;
    a.clip = v.clip;
    a.g = v.g;
    a.clipped = v.clipped;
    a.tiles = static_cast<int>(tiles);
    a.tiles_per = static_cast<int>(per);
    hipLaunchKernelGGL(value_head_stream_kernel, dim3(static_cast<unsigned>(ceil_div(tiles, per))), dim3(kFsThreads), 0,
                       st, a);
    return launch_status();
}

int64_t value_head_stream_rows(int64_t M) {
    if (M <= 0 || M % kFsT) return 0;
    const int64_t tiles = M / kFsT;
    const int64_t per = ceil_div(tiles, std::min<int64_t>(2 * kFsMaxSlices, tiles));
    return ceil_div(tiles, per);
}

bool value_head_stream_enabled() {  // default since round 5's bench A/B; RSLRL_VALUE_HEAD_STREAM=0 keeps the tiled head
    static const bool on = [] {
        const char* e = std::getenv("RSLRL_VALUE_HEAD_STREAM");
        return !(e && e[0] == '0');
    }();
    return on;
}
}  // namespace rslrl
