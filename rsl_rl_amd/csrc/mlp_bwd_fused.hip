// Backward of a square hidden layer (Linear(256, 256) + ELU of rsl_rl/networks/mlp.py:106-114, reached from
// ppo.py:367's loss.backward()) in ONE pass over the mini-batch rows, on the x6 split-bf16 MFMA path:
//   input gradient   dZp = (dZ W) * ELU'(H)            (rslrl_linear_gemm RSLRL_LINEAR_DGRAD_ELU: the same bits)
//   weight gradient  dW  = dZ^T H,  bias gradient db = sum_m dZ[m]   (rslrl_linear_wgrad_bias, bias_side 1)
// where dZ [M, 256] is the gradient at this layer's pre-activation and H [M, 256] this layer's input (the previous
// layer's ELU output).  The separate kernels read dZ and H twice (input gradient, then weight gradient: 1.6 GB per
// actor + critic pair at 393,216 rows); here every 64-row tile of dZ and H is read from HBM once and feeds both GEMMs.
//
// One workgroup per CU (8 waves, 256 registers per lane, all 160 KiB of LDS) runs a slice of consecutive 64-row
// tiles and keeps the slice's whole 256 x 256 weight gradient in registers (wave w: columns k in [32w, 32w + 32),
// 8 MFMA blocks of 32 x 32 = 128 accumulator registers); the slice's [dW | db] partial row is folded in fp64 in a
// fixed order afterwards (rslrl_fold_partials_batch, as the weight-gradient kernel's).  Per tile:
//  1. the dZ tile sits in LDS as three bf16 planes (96 KiB, split once) for the whole tile;
//  2. input gradient: wave w computes the output columns [32w, 32w + 32) of all 64 rows (2 MFMA blocks) over the
//     16 k-chunks -- A fragments (dZ rows) from the resident planes, B fragments (the W^T image, L2-resident) straight
//     from global memory one chunk ahead: no LDS writes and no barrier inside the main loop;
//  3. epilogue: H read in the accumulator layout from the wave's own 8 KiB region of a 64 KiB LDS stage (each wave
//     DMAs exactly the H columns it needs, so the epilogue waits for its own loads only: no workgroup barrier between
//     the two GEMMs, and waves that finish the main loop early run their epilogue beside the others' MFMAs), ELU',
//     dZp stored (nontemporal); the next tile's H is DMA'd into the region right after;
//  4. weight gradient: dW[n][k] += sum over the tile's rows of dZ[m][n] H[m][k] -- A = dZ^T from the resident planes
//     by ds_read_b64_tr_b16, B = H straight from the epilogue's registers: the accumulator layout holds, per lane,
//     column k at rows (r & 3) + 8 (r >> 2) + 4 (lane >> 5), so each 16-deep MFMA step takes the reduction rows in
//     the permuted order pi(8 h + t) = 16 s + 4 h + (t & 3) + 8 (t >> 2) -- the same order for the dZ^T fragments
//     (the transposed reads address exactly those rows), i.e. the same sum over the tile's rows;
//  5. meanwhile the next tile's dZ is loaded into registers (split into the planes after a barrier: 2 per tile).
// The column sums of dZ (db) accumulate in fp32 from the staged registers (every thread owns four fixed columns) and
// fold over the 8 waves in wave order at the end.  Deterministic: the summation order depends on M alone.
//
// LDS image of a dZ plane: [16 chunks of 16 columns][64 row slots][32 bytes] (the input gradient's 16-deep k-chunks),
// row m of chunk c in slot m ^ f(c), f(c) = (c & 3) | 4 (c & 1), its two 16-byte halves swapped when (m >> 3) & 1.
// Bank-conflict free for all three accesses: the input gradient's ds_read_b128 row fragments (one chunk per
// instruction: the half swap separates the rows that share a bank quad), the weight gradient's transposed reads
// (4 rows of two adjacent chunks per 32-lane group: bit 2 of f puts the odd chunk's rows on the other 32 banks) and
// the staging stores (ds_write_b64, 16 lanes = one row of 4 chunks: f's low bits give each chunk its own 8 banks).
// Every chunk offset (and the 8-row / 32-row steps) lands in the instructions' immediate offsets: a handful of
// address registers for the whole tile.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "x6_split.h"

namespace rslrl {
namespace {

constexpr int kHbT = 64;                        // rows per tile
constexpr int kHbW = 256;                       // the layer's width (N = K = 256)
constexpr int kHbThreads = 512;                 // 8 waves
constexpr int kHbPlane = kHbT * kHbW * 2;       // one bf16 plane of the dZ tile: 32 KiB
constexpr int kHbDzBytes = 3 * kHbPlane;        // 96 KiB
constexpr int kHbHBytes = kHbT * kHbW * 4;      // the H stage: 64 KiB
constexpr int kHbLds = kHbDzBytes + kHbHBytes;  // 160 KiB: the whole LDS of a CU
constexpr int kHbChunks = kHbW / 16;            // k-chunks of the input gradient
constexpr int kHbImgPlaneU = kHbW * 32 / 16;    // 16-byte units of one plane of one image chunk (bimage layout 0)
constexpr int kHbImgChunkU = 3 * kHbImgPlaneU;
constexpr int kHbPartFloats = kHbW * kHbW + kHbW;  // a slice's partial row: [dW (256 x 256) | db (256)]
constexpr int kHbMaxSlices = 128;               // per problem: a pair fills the 256 CUs with one workgroup each
#ifndef RSLRL_HB_BDEPTH
#define RSLRL_HB_BDEPTH 1
#endif
constexpr int kHbBDepth = RSLRL_HB_BDEPTH;      // image chunks loaded ahead of the input gradient's MFMAs

using s16x4 = __attribute__((ext_vector_type(4))) short;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

struct HbProblem {
    const float* dz;   // [M, 256]
    const float* h;    // [M, 256]
    const uint4* img;  // x6 image of W^T (layout 0, 16 chunks)
    float* dz_prev;    // [M, 256]
    float* part;       // [S][kHbPartFloats]
};

struct HbArgs {
    HbProblem p[2];
    int tiles;      // M / 64
    int tiles_per;  // tiles per slice
};

constexpr int kHbChunkB = kHbT * 32;  // one chunk of one plane: 2 KiB

__host__ __device__ constexpr int hb_f(int c) { return (c & 3) | ((c & 1) << 2); }

// byte offset of (row m, column col % 4 == 0) in a plane
__device__ __forceinline__ int hb_dz_off(int m, int col) {
    const int c = col >> 4;
    return c * kHbChunkB + (m ^ hb_f(c)) * 32 + 16 * (((col >> 3) & 1) ^ ((m >> 3) & 1)) + 8 * ((col >> 2) & 1);
}

constexpr uint32_t kHbRsrcFlags = 0x00020000;
constexpr uint32_t kHbTileBytes = kHbT * kHbW * 4;  // 64 KiB: one tile of dZ or H

// a buffer resource over the tile's rows of an [M, 256] fp32 array: wave-uniform base, every offset in the
// instructions' voffset / soffset / immediate fields (no 64-bit address registers)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t hb_tile_rsrc(const float* base, int64_t row0) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base + row0 * kHbW), 0, kHbTileBytes, kHbRsrcFlags);
}

// the tile's dZ (8 float4 per thread: row (t >> 6) + 8 i, columns 4 (t & 63) .. + 3); nontemporal like the H DMA:
// dZ and H are read once, so they should not push the W^T image out of L2 (PMC: reads 1.14x -> 1.00x algorithmic)
template <int I0 = 0, int I1 = 8>
__device__ __forceinline__ void hb_load_dz(__amdgpu_buffer_rsrc_t r, float4 (&v)[8]) {
    const int off = ((threadIdx.x >> 6) * kHbW + 4 * (threadIdx.x & 63)) * 4;
#pragma unroll
    for (int i = I0; i < I1; ++i)
        v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, i * 8 * kHbW * 4, 2));
}

__device__ __forceinline__ void hb_store_dz(const float4 (&v)[8], char* __restrict__ lds, float4& csum) {
    const int col = 4 * (threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int m = (threadIdx.x >> 6) + 8 * i;
        csum.x += v[i].x;
        csum.y += v[i].y;
        csum.z += v[i].z;
        csum.w += v[i].w;
        uint2 w[3];
        split4(v[i], w[0], w[1], w[2]);
        const int off = hb_dz_off(m, col);
#pragma unroll
        for (int q = 0; q < 3; ++q) *reinterpret_cast<uint2*>(lds + q * kHbPlane + off) = w[q];
    }
}

// H stage: wave w owns the 8 KiB region [64 row slots][32 columns] of its columns [32 w, 32 w + 32) -- the only H
// the wave's epilogue reads, so no other wave's DMA is waited for.  Row r sits in slot r ^ ((r >> 2) & 1): rows r and
// r + 4 (the two lane halves of one accumulator-layout read) land on opposite 32-bank halves.
constexpr int kHbHRegion = kHbT * 32 * 4;  // 8 KiB
__device__ __forceinline__ int hb_hslot(int r) { return r ^ ((r >> 2) & 1); }

// the tile's H columns of this wave into its region: instruction i fills slots 8 i .. 8 i + 7 (lane l: slot 8 i + l / 8,
// 16 bytes of column quad l % 8)
__device__ __forceinline__ void hb_dma_h(__amdgpu_buffer_rsrc_t r, char* stage) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int off = (hb_hslot(lane >> 3) * kHbW + 32 * wave + 4 * (lane & 7)) * 4;  // slot ^ row differ in bit 0 only
#pragma unroll
    for (int i = 0; i < 8; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void*)(stage + wave * kHbHRegion + i * 1024), 16, off,
            i * 8 * kHbW * 4, 0, 2);
}

// one 4-row transposed read (ds_read_b64_tr_b16) at byte address addr of the LDS
__device__ __forceinline__ s16x4 hb_tr(int addr) {
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(reinterpret_cast<lds_s16x4*>(addr));
}

__device__ __forceinline__ bf16x8 hb_cat(s16x4 lo, s16x4 hi) {
    const __attribute__((ext_vector_type(8))) short v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 hb_read16(int addr) {
    typedef __attribute__((address_space(3))) uint4 lds_u4;
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const lds_u4*>(addr));
}

#ifdef RSLRL_HB_STAMPS
// diagnostic build only (never the shipped library): per workgroup, tile and wave, s_memtime at 7 phase points ->
// g_hb_stamps[((wg * tiles_per + tile) * 8 + wave) * 8 + k]; the values go to this buffer alone (scripts/hb_stamps.py)
__device__ uint64_t* g_hb_stamps;
#define HB_STAMP(k)                                                                                          \
    do {                                                                                                     \
        if (g_hb_stamps && (threadIdx.x & 63) == 0)                                                          \
            g_hb_stamps[((static_cast<int64_t>(blockIdx.y * gridDim.x + blockIdx.x) * args.tiles_per + (t - t_begin)) * 8 + \
                         (threadIdx.x >> 6)) * 8 + (k)] = __builtin_amdgcn_s_memtime();                     \
    } while (0)
#else
#define HB_STAMP(k) \
    do {            \
    } while (0)
#endif

// BD: image chunks loaded ahead of the input gradient's MFMAs; LA: the LDS fragments of the next MFMA block read
// ahead of the current block's MFMAs (1) or just before their own (0).  RSLRL_HB_VARIANT="BD,LA" picks an instance
// per call (A/B in one process); default kHbBDepth, 1.
template <int BD, int LA, int PRIO = 0>
__global__ __launch_bounds__(kHbThreads, 2) void hidden_bwd_kernel(HbArgs args) {
    __shared__ __attribute__((aligned(16))) char lds[kHbLds];
    char* const dzl = lds;
    char* const stage = lds + kHbDzBytes;
    const HbProblem& P = args.p[blockIdx.y];
    const int s = blockIdx.x;
    const int t_begin = s * args.tiles_per;
    const int t_end = min(args.tiles, t_begin + args.tiles_per);

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if constexpr (PRIO) {  // static priority for the second-dispatched half (MI355X_MICROARCH.md, two waves per SIMD)
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const int g1 = (lane >> 4) & 1;  // transposed reads: which 16 of a block's 32 columns
    const int tq = (lane >> 2) & 3;  //   row within the 4-row group
    const int tp = lane & 3;         //   column quad

    // LDS lane address parts (the dZ planes start at LDS address 0): la[c & 3] = hb_dz_off(l32, 16 c + 8 h) - c * 2 KiB
    // for the input gradient's row fragments; lt[nb & 1][hi] = hb_dz_off(4 h + tq + 8 hi, 32 nb + 16 g1 + 4 tp) -
    // 2 (nb >> 1) * 4 KiB for the weight gradient's transposed reads; la2 / lt2: the same + two planes
    const int lbase = static_cast<int>(reinterpret_cast<uintptr_t>(dzl));
    int la[4], la2[4], lt[2][2], lt2[2][2];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        la[c] = lbase + hb_dz_off(l32, 16 * c + 8 * h) - c * kHbChunkB;
        la2[c] = la[c] + 2 * kHbPlane;
    }
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int hi = 0; hi < 2; ++hi) {
            lt[nb][hi] = lbase + hb_dz_off(4 * h + tq + 8 * hi, 32 * nb + 16 * g1 + 4 * tp);
            lt2[nb][hi] = lt[nb][hi] + 2 * kHbPlane;
        }

    f32x16 dw[8];
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) dw[nb] = f32x16{};
    float4 csum = make_float4(0.f, 0.f, 0.f, 0.f);

    // this wave's B fragments: image row 32 w + l32 (output column), half h, swizzled as the image stores it; the
    // chunk and plane offsets ride in soffset
    const int brow = 32 * wave + l32;
    const int boff = (brow * 2 + (h ^ ((brow >> 3) & 1))) * 16;
    const __amdgpu_buffer_rsrc_t rimg = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint4*>(P.img), 0, static_cast<uint32_t>(kHbChunks * kHbImgChunkU * 16), kHbRsrcFlags);
    auto bload = [&](int c, int q) {
        return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rimg, boff, (c * kHbImgChunkU + q * kHbImgPlaneU) * 16, 0));
    };

    // prologue: the first tile's H stage and dZ planes
    {
        const int64_t row0 = static_cast<int64_t>(t_begin) * kHbT;
        hb_dma_h(hb_tile_rsrc(P.h, row0), stage);
        float4 v[8];
        hb_load_dz(hb_tile_rsrc(P.dz, row0), v);
        hb_store_dz(v, dzl, csum);
    }
    __syncthreads();

    for (int t = t_begin; t < t_end; ++t) {
        const int64_t row0 = static_cast<int64_t>(t) * kHbT;
        const bool has_next = t + 1 < t_end;
        HB_STAMP(0);
        // ---- input gradient main loop: dZ rows (LDS, resident) x W^T columns (global, two chunks ahead).  Block
        // b = 2 c + i is chunk c of row block i; the A fragments of block b + 1 are read while block b's MFMAs run.
        f32x16 acc[2] = {f32x16{}, f32x16{}};
        uint4 bq[BD + 1][3];  // ring of image chunks in flight (BD ahead)
#pragma unroll
        for (int c = 0; c < BD; ++c)
#pragma unroll
            for (int q = 0; q < 3; ++q) bq[c][q] = bload(c, q);
        auto read_a = [&](int b, bf16x8 (&a)[3]) {
            // hb_dz_off(32 i + l32, 16 c + 8 h) = lane part (by c & 3) + c * 2 KiB + i * 1 KiB: the constant in the
            // immediate offset (plane 2 from a second base: the field holds 16 bits)
            const int c = b >> 1, ci = c * kHbChunkB + (b & 1) * 1024;
            a[0] = hb_read16(la[c & 3] + ci);
            a[1] = hb_read16(la[c & 3] + ci + kHbPlane);
            a[2] = hb_read16(la2[c & 3] + ci);
        };
        bf16x8 af[2][3];
        if (LA) read_a(0, af[0]);
#pragma unroll
        for (int b = 0; b < 2 * kHbChunks; ++b) {
            const int c = b >> 1;
            if ((b & 1) == 0 && c + BD < kHbChunks) {
#pragma unroll
                for (int q = 0; q < 3; ++q) bq[(c + BD) % (BD + 1)][q] = bload(c + BD, q);
            }
            if (LA && b + 1 < 2 * kHbChunks) read_a(b + 1, af[(b + 1) & 1]);
            if (!LA) read_a(b, af[b & 1]);
            bf16x8 bf[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) bf[q] = __builtin_bit_cast(bf16x8, bq[c % (BD + 1)][q]);
            acc[b & 1] = mfma_x6(af[b & 1], bf, acc[b & 1]);
            __builtin_amdgcn_sched_barrier(0);  // two blocks' fragments live at a time (the 128 dW registers stay)
        }
        // ---- epilogue: H from this wave's stage region (its own DMA: no workgroup barrier), ELU', dZp out
        HB_STAMP(1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);  // the main loop's registers die here (nothing of the epilogue moves up)
        HB_STAMP(2);
        float hr[2][16];
        {
            // H in the accumulator layout; dZp = acc * ELU'(H) (epilogue_tiles_impl's bits) written back over the
            // same region words, then read row-contiguous and stored as 16-byte units: 8 stores per lane instead of
            // 32 4-byte ones
            // row 32 i + 4 h + rr (rr = (r & 3) + 8 (r >> 2), bit 2 clear) sits in slot 32 i + rr + 5 h (rr even) or
            // 32 i + rr + 3 h (rr odd): two lane bases, the rest in the immediate offsets
            float* const reg = reinterpret_cast<float*>(stage + wave * kHbHRegion) + l32;
            float* const hs[2] = {reg + 5 * h * 32, reg + 3 * h * 32};
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) hr[i][r] = hs[r & 1][(32 * i + (r & 3) + 8 * (r >> 2)) * 32];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = acc[i][r];
                    const float hv = hr[i][r];
                    const float g = v * (hv + 1.f);  // ELU'(z) = 1 if z > 0 else h + 1
                    hs[r & 1][(32 * i + (r & 3) + 8 * (r >> 2)) * 32] = hv > 0.f ? v : g;
                }
            // the dword writes retire before the 16-byte reads (the LDS does not keep that order by itself)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
                P.dz_prev + row0 * kHbW + 32 * wave, 0, static_cast<uint32_t>(kHbT * kHbW * 4), kHbRsrcFlags);
            const float* rs = reinterpret_cast<const float*>(stage + wave * kHbHRegion) + hb_hslot(lane >> 3) * 32 +
                              4 * (lane & 7);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const u32x4 sv = *reinterpret_cast<const u32x4*>(rs + 8 * j * 32);  // row 8 j + lane / 8
                __builtin_amdgcn_raw_buffer_store_b128(sv, rc, ((lane >> 3) * kHbW + 4 * (lane & 7)) * 4,
                                                       8 * j * kHbW * 4, 2 /* nt */);
                // VMEM store-data hazard (mlp_gemm.hip epilogue_tiles_staged): keep the data registers live past wait
                // states of their own after the 16-byte store
                asm volatile("s_nop 3" ::"v"(sv) : "memory");
            }
            // the next tile's H into the (now read) region: it lands during this tile's weight gradient
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (has_next) hb_dma_h(hb_tile_rsrc(P.h, row0 + kHbT), stage);
        }
        float4 vn[8];
        HB_STAMP(3);
        // ---- weight gradient of the tile: dW[n][32 w + l32] += sum over rows of dZ[m][n] H[m][32 w + l32].  Block
        // k = 8 (2 i + st) + nb: row step (i, st), column block nb; the dZ^T fragments of block k + 1 are read while
        // block k's MFMAs run.
        auto read_t = [&](int k, bf16x8 (&a)[3]) {
            // rows 32 i + 16 st + 4 h + tq (lo) and + 8 (hi), columns 32 nb + 16 g1 + 4 tp: lane part by (nb & 1,
            // lo / hi), the rest constant
            const int nb = k & 7, i = k >> 4, st = (k >> 3) & 1;
            const int ci = 2 * (nb >> 1) * 2 * kHbChunkB + (32 * i + 16 * st) * 32;
            const int b0 = lt[nb & 1][0] + ci, b1 = lt[nb & 1][1] + ci;
            const int c0 = lt2[nb & 1][0] + ci, c1 = lt2[nb & 1][1] + ci;
            a[0] = hb_cat(hb_tr(b0), hb_tr(b1));
            a[1] = hb_cat(hb_tr(b0 + kHbPlane), hb_tr(b1 + kHbPlane));
            a[2] = hb_cat(hb_tr(c0), hb_tr(c1));
        };
        bf16x8 tf[2][3];
        bf16x8 hb[3];
        if (LA) read_t(0, tf[0]);
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            const int nb = k & 7, i = k >> 4, st = (k >> 3) & 1;
            if (nb == 0) {
                // B = H rows pi(8 h + t) of column 32 w + l32: accumulator entries r = 8 st + t of block i
                uint32_t p0[4], p1[4], p2[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float x = hr[i][8 * st + 2 * j], y = hr[i][8 * st + 2 * j + 1];
                    p0[j] = split_pair(x, y);
                    p1[j] = split_pair(x, y);
                    p2[j] = pack_pair(x, y);
                }
                hb[0] = __builtin_bit_cast(bf16x8, make_uint4(p0[0], p0[1], p0[2], p0[3]));
                hb[1] = __builtin_bit_cast(bf16x8, make_uint4(p1[0], p1[1], p1[2], p1[3]));
                hb[2] = __builtin_bit_cast(bf16x8, make_uint4(p2[0], p2[1], p2[2], p2[3]));
                // the next tile's dZ into registers once H block 0 is dead (~8 blocks of MFMAs before its split into
                // bf16 planes at k = 16 .. 23, beside the MFMAs: the phase after the loop only writes them to LDS)
                if (k == 8 && has_next) hb_load_dz(hb_tile_rsrc(P.dz, row0 + kHbT), vn);
            }
            if (LA && k + 1 < 32) read_t(k + 1, tf[(k + 1) & 1]);
            if (!LA) read_t(k, tf[k & 1]);
            dw[nb] = mfma_x6(tf[k & 1], hb, dw[nb]);
            __builtin_amdgcn_sched_barrier(0);
        }
        HB_STAMP(4);
        __syncthreads();  // every wave has read the dZ planes (and, in the epilogue, the H stage)
        HB_STAMP(5);
        if (has_next) {
            hb_store_dz(vn, dzl, csum);
            __syncthreads();
        }
        HB_STAMP(6);
    }

    // ---- the slice's partial row: dW (lane: column 32 w + l32 of rows 32 nb + (r & 3) + 8 (r >> 2) + 4 h), then db
    float* out = P.part + static_cast<int64_t>(s) * kHbPartFloats;
#pragma unroll
    for (int nb = 0; nb < 8; ++nb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
            out[(32 * nb + (r & 3) + 8 * (r >> 2) + 4 * h) * kHbW + 32 * wave + l32] = dw[nb][r];
    float4* red = reinterpret_cast<float4*>(stage);  // free: the last tile's H was read before the last barrier
    red[threadIdx.x] = csum;
    __syncthreads();
    if (threadIdx.x < 64) {
        float4 a = red[threadIdx.x];
#pragma unroll
        for (int g = 1; g < 8; ++g) {
            const float4 b = red[64 * g + threadIdx.x];
            a.x += b.x;
            a.y += b.y;
            a.z += b.z;
            a.w += b.w;
        }
        reinterpret_cast<float4*>(out + kHbW * kHbW)[threadIdx.x] = a;
    }
}

int64_t hb_tiles_per(int64_t tiles) {
    const int64_t s = std::min<int64_t>(kHbMaxSlices, tiles);
    return ceil_div(tiles, s);
}

}  // namespace
}  // namespace rslrl

using namespace rslrl;

#ifdef RSLRL_HB_STAMPS
extern "C" int rslrl_hb_debug_stamps(void* buf) {  // diagnostic build only
    uint64_t* p = static_cast<uint64_t*>(buf);
    return static_cast<int>(hipMemcpyToSymbol(HIP_SYMBOL(g_hb_stamps), &p, sizeof(p)));
}
#endif

extern "C" int64_t rslrl_hidden_bwd_slices(int64_t M) {
    if (M < kHbT || M % kHbT || M / kHbT > INT32_MAX) return 0;
    const int64_t tiles = M / kHbT;
    return ceil_div(tiles, hb_tiles_per(tiles));
}

extern "C" size_t rslrl_hidden_bwd_partial_floats(void) { return kHbPartFloats; }

extern "C" int rslrl_hidden_bwd_pair(const rslrl_hidden_bwd_problem_t* p0, const rslrl_hidden_bwd_problem_t* p1,
                                     int64_t M, int32_t width, rslrl_stream_t stream) {
    if (!p0 || width != kHbW) return RSLRL_E_INVALID_ARGUMENT;
    if (M < kHbT || M % kHbT || M / kHbT > INT32_MAX) return M == 0 ? RSLRL_OK : RSLRL_E_UNSUPPORTED;
    const rslrl_hidden_bwd_problem_t* a[2] = {p0, p1};
    const int n = p1 ? 2 : 1;
    HbArgs args{};
    for (int i = 0; i < n; ++i) {
        const rslrl_hidden_bwd_problem_t* q = a[i];
        if (!q->dz || !q->h || !q->bimage || !q->dz_prev || !q->partials) return RSLRL_E_INVALID_ARGUMENT;
        const uintptr_t bits = reinterpret_cast<uintptr_t>(q->dz) | reinterpret_cast<uintptr_t>(q->h) |
                               reinterpret_cast<uintptr_t>(q->bimage) | reinterpret_cast<uintptr_t>(q->dz_prev) |
                               reinterpret_cast<uintptr_t>(q->partials);
        if (bits & 15) return RSLRL_E_MISALIGNED;
        args.p[i] = HbProblem{q->dz, q->h, static_cast<const uint4*>(q->bimage), q->dz_prev, q->partials};
    }
    const int64_t tiles = M / kHbT;
    const int64_t per = hb_tiles_per(tiles);
    args.tiles = static_cast<int>(tiles);
    args.tiles_per = static_cast<int>(per);
    const dim3 grid(static_cast<unsigned>(ceil_div(tiles, per)), static_cast<unsigned>(n));
    int bd = kHbBDepth, la = 0;
    if (const char* e = std::getenv("RSLRL_HB_VARIANT")) {  // "BD,LA" (A/B builds in one process)
        bd = std::atoi(e);
        const char* c = std::strchr(e, ',');
        la = c ? std::atoi(c + 1) : 0;
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 blk(kHbThreads);
    // measured at 393,216 rows (scripts/hidden_bwd_probe.py --variants, one process): BD,LA = 1,0 1067 us, 1,1 1094,
    // 2,0 1110, 2,1 1127, 3,1 1216 -- the fewer registers live, the faster (3,1 spills 37 VGPRs); the default adds
    // s_setprio 1 for waves 4-7 (1048 vs 1055 and 1043 vs 1047 us in two runs, profiles/r5_hb_variants.json)
    if (bd == 2 && la == 0) hipLaunchKernelGGL((hidden_bwd_kernel<2, 0>), grid, blk, 0, st, args);
    else if (bd == 2) hipLaunchKernelGGL((hidden_bwd_kernel<2, 1>), grid, blk, 0, st, args);
    else if (la == 1) hipLaunchKernelGGL((hidden_bwd_kernel<1, 1>), grid, blk, 0, st, args);
    else if (la == 2) hipLaunchKernelGGL((hidden_bwd_kernel<1, 0, 1>), grid, blk, 0, st, args);  // LA 2: prio
    else if (la == 3) hipLaunchKernelGGL((hidden_bwd_kernel<1, 1, 1>), grid, blk, 0, st, args);
    else if (la == 4) hipLaunchKernelGGL((hidden_bwd_kernel<1, 0, 0>), grid, blk, 0, st, args);  // LA 4: no prio
    else hipLaunchKernelGGL((hidden_bwd_kernel<1, 0, 1>), grid, blk, 0, st, args);
    return launch_status();
}
