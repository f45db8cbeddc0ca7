// The rollout's whole actor and critic forward in one launch (round 6): policy.act + policy.evaluate of one env step
// (rsl_rl/algorithms/ppo.py:155-156 through rsl_rl/networks/mlp.py:106-114 -- Linear + ELU hidden layers, then the
// output Linear), on x6 split-bf16 MFMAs, with no hidden activation reaching HBM (rslrl_rollout_mlp_pair).
//
// The layer-by-layer launches this replaces (rslrl_linear_gemm_pair for each hidden layer, then the fused last hidden +
// output layer) write every hidden activation to HBM and read it back, and at a rollout's M (one row per env: 16,384
// per GPU at C4 on 8 GPUs) each launch holds one tile per CU, so its pipeline fill and tail are most of its time.
// Here a workgroup keeps its 64-row tile's activations in LDS from the observation to the outputs:
//  * 4 waves; wave w owns output columns [64 w, 64 w + 64) of the tile's 64 rows (2 x 2 blocks of 32 x 32 on
//    C^T accumulators: lane (l32, h) holds row 32 i + l32 and columns 32 j + (r & 3) + 8 (r >> 2) + 4 h);
//  * the layer input: the observations straight from global memory (first layer), then the previous layer's output
//    as fp32 in LDS (64 KiB, 16-byte units XOR-swizzled by row & 15: conflict-free for the epilogue's row-quad
//    writes and the fragment reads); each wave splits the 8 values of a fragment into the three bf16 planes as it
//    reads them (split4: the planes the layer-by-layer kernels stage);
//  * weight fragments from the layout-0 images (L2-resident, one chunk ahead in registers), no LDS, no barrier;
//  * two workgroups per CU (64 KiB of LDS, <= 256 registers each): one's epilogues and barriers beside the other's
//    MFMAs.
// Bits.  Every output is the same sequence of fp32 operations as in the layer-by-layer path, so the results are
// identical (tests/test_gpu_rollout_mlp.py): the hidden layers' MFMAs take the weight fragment as the A operand (C^T)
// but issue the six products in the C-orientation kernels' order (mfma_x6(x, w): x2 w0, x0 w2, x1 w1, x1 w0, x0 w1,
// x0 w0), chunks in order from zero accumulators; + b, ELU (elu_neg: mlp_gemm.hip's expression); the last hidden layer
// in the fused output kernel's order (mfma_x6(w, x), C^T), its output layer as that kernel's epilogue computes it --
// x6 MFMAs over (j, s2) per 64-column group (> 4 outputs) or fp32 fma chains (<= 4 outputs: the value head), the four
// column groups' partials added in order, + the output bias.
#include "common.h"
#include "x6_split.h"

namespace rslrl {
namespace {

constexpr int kRmT = 64;                   // rows per tile
constexpr int kRmThreads = 256;            // 4 waves
constexpr int kRmHidden = 4;               // hidden layers supported (256 wide each)
constexpr int kRmOutMax = 16;              // output width
constexpr int kRmImgPlaneU = 256 * 32 / 16;  // 16-byte units of one plane of one image chunk (layout 0)
constexpr int kRmImgChunkU = 3 * kRmImgPlaneU;
constexpr int kRmOutPlaneUnits = 4 * 2 * 2 * 3 * 2 * 32;  // mlp_gemm.hip kOutImagePlaneUnits (BIMAGE_LAYOUT_OUT)
constexpr uint32_t kRmRsrcFlags = 0x00020000;
#ifndef RSLRL_RM_COOP
#define RSLRL_RM_COOP 1  // cooperative per-chunk split into a plane stage (A/B knob: 0 = every wave splits on read)
#endif
constexpr int kRmStagePlane = kRmT * 32;          // one bf16 plane of one k-chunk: 2 KiB
constexpr int kRmStageBuf = 3 * kRmStagePlane;    // 6 KiB
constexpr int kRmLds = kRmT * 256 * 4 + (RSLRL_RM_COOP ? 2 * kRmStageBuf : 0);  // 76 KiB: two workgroups per CU

struct RmProblem {
    const float* x;                 // [M, K0]
    const uint4* img[kRmHidden];    // layout-0 images of the hidden layers' weights
    const float* bias[kRmHidden];   // [256] each
    const uint4* oimg;              // output layer image (BIMAGE_LAYOUT_OUT)
    const float* obias;             // [nout]
    float* y;                       // [M, nout]
    float* sample;                  // [M, nout] standard normals in, actions out (or null)
    const float* sample_scale;      // [nout]
    int nout;
};

struct RmArgs {
    RmProblem p[2];
    int hidden;  // hidden layers (2..kRmHidden)
};

// mlp_gemm.hip elu_neg / mlp_fwd_stream.hip fs_elu_neg: the same expression (tests/test_elu_poly.py)
__device__ __forceinline__ float rm_elu_neg(float v) {
    float t = __fmaf_rn(v, 0.0011216326f, 0.008187376f);
    t = __fmaf_rn(v, t, 0.04162908f);
    t = __fmaf_rn(v, t, 0.16666223f);
    t = __fmaf_rn(v, t, 0.49999982f);
    t = __fmaf_rn(v, t, 1.0f);
    const float poly = v * t;
    const float e = __expf(v) - 1.0f;
    return v > -0.5f ? poly : e;
}

__device__ __forceinline__ float rm_elu(float v) {
    const float n = rm_elu_neg(fminf(v, 0.f));
    return v > 0.f ? v : n;
}

// 8 consecutive k values -> the fragment's three bf16 planes (store_a_split + read_frag's bits)
__device__ __forceinline__ void rm_split8(const float4& lo4, const float4& hi4, bf16x8 (&f)[3]) {
    uint2 lo[3], hi[3];
    split4(lo4, lo[0], lo[1], lo[2]);
    split4(hi4, hi[0], hi[1], hi[2]);
#pragma unroll
    for (int q = 0; q < 3; ++q) f[q] = __builtin_bit_cast(bf16x8, make_uint4(lo[q].x, lo[q].y, hi[q].x, hi[q].y));
}

// the six products in the C-orientation kernels' order (mfma_x6(x, w)) on the C^T tile: MFMA(w_q, x_p) = MFMA(x_p, w_q)^T
__device__ __forceinline__ f32x16 mfma_x6_ct(const bf16x8 (&x)[3], const bf16x8 (&w)[3], f32x16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[2], x[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[0], acc, 0, 0, 0);
    return acc;
}

using u32x2 = __attribute__((ext_vector_type(2))) unsigned int;

__device__ __forceinline__ bf16x8 rm_lds_frag(int addr) {
    typedef __attribute__((address_space(3))) bf16x8 lds_b8;
    return *reinterpret_cast<const lds_b8*>(addr);
}

// workgroup barrier for LDS hand-offs only: the register prefetches in flight (weights, biases) stay in flight
// (__syncthreads' fence would wait for them: vmcnt(0))
__device__ __forceinline__ void rm_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ float4 rm_lds_read(int addr) {
    typedef __attribute__((address_space(3))) f32x4 lds_f4;
    const f32x4 v = *reinterpret_cast<const lds_f4*>(addr);
    return make_float4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ void rm_lds_write(int addr, float4 v) {
    typedef __attribute__((address_space(3))) f32x4 lds_f4;
    *reinterpret_cast<lds_f4*>(addr) = f32x4{v.x, v.y, v.z, v.w};
}

// One problem's forward over one 64-row tile.  NR: 4 = output layer on x6 MFMAs (> 4 outputs), 1 = fp32 fma chains.
// KC0: 16-deep chunks of the first layer's input.
template <int KC0, int NR>
__device__ __forceinline__ void rm_body(const RmProblem& P, int hidden, char* lds) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const int s = l32 & 15;  // the LDS swizzle of this lane's rows (32 i + l32)
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * kRmT;
    const int lbase = static_cast<int>(reinterpret_cast<uintptr_t>(lds)) + l32 * 1024;

    // H in LDS: row r, 16-byte unit u (columns 4 u .. 4 u + 3) at r * 1024 + 16 (u ^ (r & 15))
    // fragment reads of chunk c: units 4 c + 2 h (+ 1), row 32 i + l32 -> lbase + rd[c & 3][e] + 256 (c >> 2) + 32 KiB i
    int rd[4][2];
#pragma unroll
    for (int cc = 0; cc < 4; ++cc)
#pragma unroll
        for (int e = 0; e < 2; ++e) rd[cc][e] = lbase + (((4 * cc + 2 * h + e) ^ s) << 4);
    // epilogue writes: unit 16 w + 8 j + 2 g + h -> lbase + 256 w + wr[j][g] + 32 KiB i
    auto wr_addr = [&](int j, int g) { return lbase + 256 * wave + (((8 * j + 2 * g + h) ^ s) << 4); };

    // weight fragment (image row n = 64 w + 32 j + l32, half h; rows swizzled by (n >> 3) & 1 = (l32 >> 3) & 1)
    const int wvoff = ((64 * wave + l32) * 2 + (h ^ ((l32 >> 3) & 1))) * 16;
    auto wload = [&](__amdgpu_buffer_rsrc_t r, int c, int j, int q) {
        return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                              r, wvoff + 1024 * j, (c * kRmImgChunkU + q * kRmImgPlaneU) * 16, 0));
    };
    auto img_rsrc = [&](int l, int chunks) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(P.img[l]), 0,
                                                 static_cast<uint32_t>(chunks * kRmImgChunkU * 16), kRmRsrcFlags);
    };

    f32x16 acc[2][2];
    // loaded ahead so that no layer start or epilogue waits out an L2 round trip: the next square layer's chunk-0 weight
    // fragments (issued in the layer before, ahead of its epilogue), the next epilogue's bias quads (columns
    // 64 w + 32 j + 8 g + 4 h; issued right after the epilogue before it), the output layer's weights (last chunk of the
    // last hidden layer)
    bf16x8 w0n[2][3];
    float4 bn[2][4];
    uint4 ow[2][2][3];    // NR 4: output-layer image fragments [j][s2][plane]
    float4 vw[2][2][2];   // NR 1: output 0's fp32 weights [j][s2][half]
    auto load_bias = [&](int l) {
        const float* bias = P.bias[l] + 64 * wave + 4 * h;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) bn[j][g] = *reinterpret_cast<const float4*>(bias + 32 * j + 8 * g);
    };
    [[maybe_unused]] auto load_w0 = [&](int l) {  // the split-on-read form (RSLRL_RM_COOP 0)
        const __amdgpu_buffer_rsrc_t rw = img_rsrc(l, 16);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q) w0n[j][q] = wload(rw, 0, j, q);
    };
    const uint4* oimg = P.oimg + wave * (2 * 2 * 3 * 64);
    const float4* owf = reinterpret_cast<const float4*>(P.oimg + kRmOutPlaneUnits) + 2 * (wave * 2 * 2 * 2 * 32 + h * 32);
    // (fp32 section: 2 ((((w * 2 + j) * 2 + s2) * 2 + h) * 32 + o) float4 pairs -- mlp_gemm.hip's out-image layout)
    auto owf_at = [&](int j, int s2, int o) { return owf + 2 * ((j * 2 + s2) * 2 * 32 + o); };
    auto load_out_weights = [&]() {
        if constexpr (NR == 1) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    vw[j][s2][0] = owf_at(j, s2, 0)[0];
                    vw[j][s2][1] = owf_at(j, s2, 0)[1];
                }
        } else if (!RSLRL_RM_COOP) {  // (the cooperative form reads them where they are used: registers)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                    for (int q = 0; q < 3; ++q) ow[j][s2][q] = oimg[((j * 2 + s2) * 3 + q) * 64 + lane];
        }
    };

#if RSLRL_RM_COOP
    // Cooperative split (the default): per k-chunk each wave splits a quarter of the chunk -- rows 16 w + (lane & 15),
    // column quad lane >> 4 -- into the three planes of a double-buffered 6 KiB stage past H, and after a workgroup
    // barrier every wave reads its fragments from the stage: each value is split once instead of once per wave (the
    // split was ~3 of the ~6 VALU per MFMA of an issue-bound loop).  Stage plane: [64 rows][32 bytes], 16-byte halves
    // swapped when (row >> 3) & 1 (conflict-free ds_write_b64 quads and ds_read_b128 fragments).
    char* const stage = lds + kRmT * 256 * 4;
    const int srow = 16 * wave + (lane & 15), squad = lane >> 4;
    const int s_rdb = static_cast<int>(reinterpret_cast<uintptr_t>(lds)) + srow * 1024;
    int s_rq[4];  // fp32 H quad of chunk c: units 4 c + squad, swizzled by srow & 15 -> s_rdb + s_rq[c & 3] + 256 (c >> 2)
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) s_rq[cc] = ((4 * cc + squad) ^ (srow & 15)) << 4;
    const int s_wr = static_cast<int>(reinterpret_cast<uintptr_t>(stage)) + srow * 32 +
                     16 * ((squad >> 1) ^ ((srow >> 3) & 1)) + 8 * (squad & 1);
    int f_rd[2], fo[2];  // fragment (row 32 i + l32, half h) of a plane: offset fo, in the stage f_rd
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = 32 * i + l32;
        fo[i] = r * 32 + 16 * (h ^ ((r >> 3) & 1));
        f_rd[i] = static_cast<int>(reinterpret_cast<uintptr_t>(stage)) + fo[i];
    }
    // ---- first layer: the X tile split once, cooperatively, into planes in the H region (free until the first
    // epilogue; plane q: [KC0 chunks][64 rows][32 bytes] as the stage), then fragments from LDS, C order
    {
        constexpr int K0 = 16 * KC0;
        constexpr int kXPlane = KC0 * kRmStagePlane;
        typedef __attribute__((address_space(3))) u32x2 lds_u2;
        const int xbase = static_cast<int>(reinterpret_cast<uintptr_t>(lds));
        const float4* xg = reinterpret_cast<const float4*>(P.x + row0 * K0);
        float4 xq[KC0];
#pragma unroll
        for (int k = 0; k < KC0; ++k) xq[k] = xg[threadIdx.x + kRmThreads * k];  // unit u: row u / 4 KC0, quad u % 4 KC0
        const __amdgpu_buffer_rsrc_t rw = img_rsrc(0, KC0);
        bf16x8 wf[2][2][3];  // [slot][j][q]
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q) wf[0][j][q] = wload(rw, 0, j, q);
#pragma unroll
        for (int k = 0; k < KC0; ++k) {
            const int u = threadIdx.x + kRmThreads * k;
            const int row = u / (4 * KC0), quad = u % (4 * KC0);
            const int q4 = quad & 3;
            uint2 w[3];
            split4(xq[k], w[0], w[1], w[2]);
            const int off = xbase + (quad >> 2) * kRmStagePlane + row * 32 + 16 * ((q4 >> 1) ^ ((row >> 3) & 1)) +
                            8 * (q4 & 1);
#pragma unroll
            for (int q = 0; q < 3; ++q) *reinterpret_cast<lds_u2*>(off + q * kXPlane) = u32x2{w[q].x, w[q].y};
        }
        rm_barrier();
#pragma unroll
        for (int c = 0; c < KC0; ++c) {
            const int sl = c & 1;
            bf16x8 xf[2][3];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int q = 0; q < 3; ++q) xf[i][q] = rm_lds_frag(xbase + fo[i] + c * kRmStagePlane + q * kXPlane);
            if (c + 1 < KC0) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int q = 0; q < 3; ++q) wf[sl ^ 1][j][q] = wload(rw, c + 1, j, q);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = mfma_x6_ct(xf[i], wf[sl][j], c == 0 ? f32x16{} : acc[i][j]);
        }
        rm_barrier();  // every wave has read the X planes: the epilogue may write H1 over them
    }
#else
    // ---- first layer: X from global memory (row 32 i + l32, columns 16 c + 8 h .. + 7), C order
    load_bias(0);
    {
        constexpr int K0 = 16 * KC0;
        const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(P.x + row0 * K0), 0, static_cast<uint32_t>(kRmT * K0 * 4), kRmRsrcFlags);
        const __amdgpu_buffer_rsrc_t rw = img_rsrc(0, KC0);
        auto xload = [&](int c, int i, int e) {
            return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  rx, ((32 * i + l32) * K0 + 8 * h + 4 * e) * 4, 16 * c * 4, 0));
        };
        float4 xv[2][2][2];  // [slot][i][e]
        bf16x8 wf[2][2][3];  // [slot][j][q]
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 2; ++e) xv[0][i][e] = xload(0, i, e);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q) wf[0][j][q] = wload(rw, 0, j, q);
#pragma unroll
        for (int c = 0; c < KC0; ++c) {
            const int sl = c & 1;
            if (c + 1 < KC0) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int q = 0; q < 3; ++q) wf[sl ^ 1][j][q] = wload(rw, c + 1, j, q);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int e = 0; e < 2; ++e) xv[sl ^ 1][i][e] = xload(c + 1, i, e);
            } else {
                load_w0(1);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                bf16x8 xf[3];
                rm_split8(xv[sl][i][0], xv[sl][i][1], xf);
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = mfma_x6_ct(xf, wf[sl][j], c == 0 ? f32x16{} : acc[i][j]);
            }
        }
    }

#endif

    // + b, ELU, fp32 into LDS (the caller has made sure no wave still reads the previous layer's H); then the next
    // epilogue's bias
    auto epilogue_to_lds = [&](int l) {
#if RSLRL_RM_COOP
        load_bias(l);  // in flight behind the other workgroup's MFMAs
#endif
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    float4 v;
                    v.x = rm_elu(acc[i][j][4 * g + 0] + bn[j][g].x);
                    v.y = rm_elu(acc[i][j][4 * g + 1] + bn[j][g].y);
                    v.z = rm_elu(acc[i][j][4 * g + 2] + bn[j][g].z);
                    v.w = rm_elu(acc[i][j][4 * g + 3] + bn[j][g].w);
                    rm_lds_write(wr_addr(j, g) + 32768 * i, v);
                }
#if !RSLRL_RM_COOP
        load_bias(l + 1);
#endif
    };

    // a square 256 x 256 layer over H in LDS: 16 chunks, weight fragments and H one chunk ahead (chunk 0's weights in
    // w0n).  CT: C order (hidden layers), else the fused output kernel's order (the last hidden layer)
#if RSLRL_RM_COOP
    auto stage_chunk = [&](int c, int buf) {
        typedef __attribute__((address_space(3))) u32x2 lds_u2;
        uint2 w[3];
        split4(rm_lds_read(s_rdb + s_rq[c & 3] + 256 * (c >> 2)), w[0], w[1], w[2]);
#pragma unroll
        for (int q = 0; q < 3; ++q)
            *reinterpret_cast<lds_u2*>(s_wr + buf * kRmStageBuf + q * kRmStagePlane) = u32x2{w[q].x, w[q].y};
    };
    auto square_layer = [&](int l, auto ct) {
        constexpr bool CT = decltype(ct)::value;
        const __amdgpu_buffer_rsrc_t rw = img_rsrc(l, 16);
        bf16x8 wf[2][2][3];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q) wf[0][j][q] = wload(rw, 0, j, q);  // in flight over the stage's barrier
        stage_chunk(0, 0);
        rm_barrier();
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            const int sl = c & 1;
            bf16x8 xf[2][3];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int q = 0; q < 3; ++q) xf[i][q] = rm_lds_frag(f_rd[i] + sl * kRmStageBuf + q * kRmStagePlane);
            if (c + 1 < 16) {
                stage_chunk(c + 1, sl ^ 1);
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int q = 0; q < 3; ++q) wf[sl ^ 1][j][q] = wload(rw, c + 1, j, q);
            }
            // (the next layer's first weights, the output layer's weights and the biases are loaded after the loop:
            // registers)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const f32x16 a0 = c == 0 ? f32x16{} : acc[i][j];
                    acc[i][j] = CT ? mfma_x6_ct(xf[i], wf[sl][j], a0) : mfma_x6(wf[sl][j], xf[i], a0);
                }
            if (c + 1 < 16) rm_barrier();  // chunk c + 1 staged; stage buffer sl free again
        }
    };
#else
    auto square_layer = [&](int l, auto ct) {
        constexpr bool CT = decltype(ct)::value;
        const __amdgpu_buffer_rsrc_t rw = img_rsrc(l, 16);
        float4 hv[2][2][2];  // [slot][i][e]
        bf16x8 wf[2][2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 2; ++e) hv[0][i][e] = rm_lds_read(rd[0][e] + 32768 * i);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q) wf[0][j][q] = w0n[j][q];
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            const int sl = c & 1;
            if (c + 1 < 16) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int q = 0; q < 3; ++q) wf[sl ^ 1][j][q] = wload(rw, c + 1, j, q);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int e = 0; e < 2; ++e)
                        hv[sl ^ 1][i][e] = rm_lds_read(rd[(c + 1) & 3][e] + 256 * ((c + 1) >> 2) + 32768 * i);
            } else if (CT) {
                load_w0(l + 1);
            } else {
                load_out_weights();
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                bf16x8 xf[3];
                rm_split8(hv[sl][i][0], hv[sl][i][1], xf);
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const f32x16 a0 = c == 0 ? f32x16{} : acc[i][j];
                    acc[i][j] = CT ? mfma_x6_ct(xf, wf[sl][j], a0) : mfma_x6(wf[sl][j], xf, a0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };

#endif

    epilogue_to_lds(0);
    __syncthreads();
    for (int l = 1; l + 1 < hidden; ++l) {
        square_layer(l, std::integral_constant<bool, true>{});
        __syncthreads();  // every wave has read H_l
        epilogue_to_lds(l);
        __syncthreads();
    }
    square_layer(hidden - 1, std::integral_constant<bool, false>{});
    __syncthreads();  // the output partials reuse the LDS

    // ---- the last hidden layer's epilogue and the output layer (mlp_gemm.hip kEpiBiasEluOut, NR 4 / NR 1)
    // red: [w][i][o][32 rows] partials of the 64-column group w
    float* red = reinterpret_cast<float*>(lds);
    const int nout = P.nout;
#if RSLRL_RM_COOP
    load_out_weights();  // in flight behind the other workgroup's MFMAs
    load_bias(hidden - 1);
#endif
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        f32x16 oacc = f32x16{};
        float oval[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            float v[16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                v[4 * g + 0] = rm_elu(acc[i][j][4 * g + 0] + bn[j][g].x);
                v[4 * g + 1] = rm_elu(acc[i][j][4 * g + 1] + bn[j][g].y);
                v[4 * g + 2] = rm_elu(acc[i][j][4 * g + 2] + bn[j][g].z);
                v[4 * g + 3] = rm_elu(acc[i][j][4 * g + 3] + bn[j][g].w);
            }
            if constexpr (NR == 1) {
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                    for (int o = 0; o < 4; ++o) {
                        if (o >= nout) break;
                        const float4 w0 = o == 0 ? vw[j][s2][0] : owf_at(j, s2, o)[0];
                        const float4 w1 = o == 0 ? vw[j][s2][1] : owf_at(j, s2, o)[1];
                        const float w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
                        for (int t = 0; t < 8; ++t) oval[o] = fmaf(v[8 * s2 + t], w[t], oval[o]);
                    }
            } else {
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    bf16x8 vb[3], wa[3];
                    rm_split8(make_float4(v[8 * s2], v[8 * s2 + 1], v[8 * s2 + 2], v[8 * s2 + 3]),
                              make_float4(v[8 * s2 + 4], v[8 * s2 + 5], v[8 * s2 + 6], v[8 * s2 + 7]), vb);
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        wa[q] = __builtin_bit_cast(bf16x8, RSLRL_RM_COOP ? oimg[((j * 2 + s2) * 3 + q) * 64 + lane]
                                                                          : ow[j][s2][q]);
                    oacc = mfma_x6(wa, vb, oacc);
                }
            }
        }
        float* rd_out = red + (wave * 2 + i) * kRmOutMax * 32;
        if constexpr (NR == 1) {  // the two lane halves hold different columns of the same row
#pragma unroll
            for (int o = 0; o < 4; ++o) {
                const float t = oval[o] + __shfl_xor(oval[o], 32, 64);
                if (h == 0 && o < nout) rd_out[o * 32 + l32] = t;
            }
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = (r & 3) + 8 * (r >> 2) + 4 * h;
                if (o < nout) rd_out[o * 32 + l32] = oacc[r];
            }
        }
    }
    // this thread's output elements (consecutive lanes take consecutive rows of one output: their partials sit in
    // consecutive banks; output-major lanes hit 3 banks per 32 lanes): their bias and the sample's normal and scale
    // are loaded before the barrier, so the loads' latency overlaps its wait
    constexpr int kPer = kRmT * kRmOutMax / kRmThreads;
    float ob[kPer], se[kPer], ss[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int idx = threadIdx.x + k * kRmThreads;
        if (idx < kRmT * nout) {
            const int rl = idx & (kRmT - 1), o = idx / kRmT;
            ob[k] = P.obias[o];
            if (P.sample) {
                se[k] = P.sample[(row0 + rl) * nout + o];
                ss[k] = P.sample_scale[o];
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int idx = threadIdx.x + k * kRmThreads;
        if (idx >= kRmT * nout) break;
        const int rl = idx & (kRmT - 1);
        const int o = idx / kRmT;
        const float* b = red + ((rl >> 5) * kRmOutMax + o) * 32 + (rl & 31);
        constexpr int kW = 2 * kRmOutMax * 32;  // stride of the column group w
        const float sum = ((b[0] + b[kW]) + b[2 * kW]) + b[3 * kW];
        const float mu = sum + ob[k];
        const int64_t e = (row0 + rl) * nout + o;
        P.y[e] = mu;
        if (P.sample)  // the Normal sample (rslrl_normal_affine's expression): eps * sigma, then + mu
            P.sample[e] = __fadd_rn(__fmul_rn(se[k], ss[k]), mu);
    }
}

template <int KC0, int NR0, int NR1>
__global__ __launch_bounds__(kRmThreads, 2) void rollout_mlp_kernel(RmArgs a) {
    __shared__ __attribute__((aligned(16))) char lds[kRmLds];
    // (distinct opaque markers open the two branches: the bodies' common index arithmetic stays inside each)
    if (blockIdx.y == 0) {
        asm volatile("; rollout mlp: problem 0" ::: "memory");
        rm_body<KC0, NR0>(a.p[0], a.hidden, lds);
    } else {
        asm volatile("; rollout mlp: problem 1" ::: "memory");
        rm_body<KC0, NR1>(a.p[1], a.hidden, lds);
    }
}

template <int KC0>
void rm_launch(const RmArgs& a, int nr0, int nr1, int64_t M, int problems, hipStream_t st) {
    const dim3 g(static_cast<unsigned>(M / kRmT), static_cast<unsigned>(problems)), b(kRmThreads);
    if (nr0 == 4 && nr1 == 1) hipLaunchKernelGGL((rollout_mlp_kernel<KC0, 4, 1>), g, b, 0, st, a);
    else if (nr0 == 4) hipLaunchKernelGGL((rollout_mlp_kernel<KC0, 4, 4>), g, b, 0, st, a);
    else if (nr1 == 1) hipLaunchKernelGGL((rollout_mlp_kernel<KC0, 1, 1>), g, b, 0, st, a);
    else hipLaunchKernelGGL((rollout_mlp_kernel<KC0, 1, 4>), g, b, 0, st, a);
}

bool rm_aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace
}  // namespace rslrl

using namespace rslrl;

extern "C" int rslrl_rollout_mlp_pair(const rslrl_rollout_mlp_t* a0, const rslrl_rollout_mlp_t* a1, int64_t M,
                                      rslrl_stream_t stream) {
    if (!a0 || M < 0) return RSLRL_E_INVALID_ARGUMENT;
    if (M == 0) return RSLRL_OK;
    const int problems = a1 ? 2 : 1;
    const rslrl_rollout_mlp_t* in[2] = {a0, a1};
    const int k0 = a0->k0, hidden = a0->hidden;
    if (a1 && (a1->k0 != k0 || a1->hidden != hidden)) return RSLRL_E_UNSUPPORTED;
    if (M % kRmT || M / kRmT > INT32_MAX || k0 < 16 || k0 > 64 || k0 % 16 || hidden < 2 || hidden > kRmHidden)
        return RSLRL_E_UNSUPPORTED;
    RmArgs args{};
    args.hidden = hidden;
    int nr[2];
    nr[1] = 1;
    for (int i = 0; i < problems; ++i) {
        const rslrl_rollout_mlp_t& s = *in[i];
        if (s.nout < 1 || s.nout > kRmOutMax) return RSLRL_E_UNSUPPORTED;
        if (!s.x || !s.out_image || !s.out_bias || !s.y) return RSLRL_E_INVALID_ARGUMENT;
        if (s.sample && !s.sample_scale) return RSLRL_E_INVALID_ARGUMENT;
        if (!rm_aligned16(s.x) || !rm_aligned16(s.out_image)) return RSLRL_E_MISALIGNED;
        RmProblem& p = args.p[i];
        for (int l = 0; l < hidden; ++l) {
            if (!s.bimage[l] || !s.bias[l]) return RSLRL_E_INVALID_ARGUMENT;
            if (!rm_aligned16(s.bimage[l]) || !rm_aligned16(s.bias[l])) return RSLRL_E_MISALIGNED;
            p.img[l] = static_cast<const uint4*>(s.bimage[l]);
            p.bias[l] = s.bias[l];
        }
        p.x = s.x;
        p.oimg = static_cast<const uint4*>(s.out_image);
        p.obias = s.out_bias;
        p.y = s.y;
        p.sample = s.sample;
        p.sample_scale = s.sample_scale;
        p.nout = s.nout;
        nr[i] = s.nout <= 4 ? 1 : 4;  // the fused output kernel's choice (mlp_gemm.hip launch<kEpiBiasEluOut>)
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    switch (k0 / 16) {
        case 1: rm_launch<1>(args, nr[0], nr[1], M, problems, st); break;
        case 2: rm_launch<2>(args, nr[0], nr[1], M, problems, st); break;
        case 3: rm_launch<3>(args, nr[0], nr[1], M, problems, st); break;
        default: rm_launch<4>(args, nr[0], nr[1], M, problems, st); break;
    }
    return launch_status();
}
