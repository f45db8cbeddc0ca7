// Split-precision fp32 operands for the MFMA GEMMs (mlp_gemm.hip, mlp_wgrad.hip): "x6" (three bf16 planes,
// six products) and "h3" (two fp16 planes of a power-of-two scaled operand, three products; below).
//
// x6: three-way bf16 split.
//
// x = x0 + x1 + x2 with x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1), each rounded to nearest;
// the residuals are exact in fp32 and the sum is exact for normal x.  A product a * b is then evaluated
// as the six bf16 products a0b0 + a0b1 + a1b0 + a1b1 + a0b2 + a2b0 on the bf16 MFMA (exact products, fp32
// accumulation); the dropped a1b2 + a2b1 + a2b2 are below 2^-23 |ab|.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rslrl {

using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using bf16x2 = __attribute__((ext_vector_type(2))) __bf16;
using f32x2 = __attribute__((ext_vector_type(2))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;

// returns the packed bf16 pair (x, y) and leaves the fp32 residuals in x, y
__device__ __forceinline__ uint32_t split_pair(float& x, float& y) {
    const f32x2 v = {x, y};
    const uint32_t pk = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
    x -= __uint_as_float(pk << 16);
    y -= __uint_as_float(pk & 0xffff0000u);
    return pk;
}

__device__ __forceinline__ uint32_t pack_pair(float x, float y) {
    const f32x2 v = {x, y};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

// float4 -> three planes of 4 bf16 (8 bytes each)
__device__ __forceinline__ void split4(float4 v, uint2& p0, uint2& p1, uint2& p2) {
    p0.x = split_pair(v.x, v.y);
    p0.y = split_pair(v.z, v.w);
    p1.x = split_pair(v.x, v.y);
    p1.y = split_pair(v.z, v.w);
    p2.x = pack_pair(v.x, v.y);
    p2.y = pack_pair(v.z, v.w);
}

// the six products of one 32x32x16 k step, smallest terms first; a[q], b[q] are plane q of each operand
__device__ __forceinline__ f32x16 mfma_x6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
    return acc;
}

// ---- "h3": two fp16 planes, three products ---------------------------------------------------------
//
// x' = s x (s a power of two chosen from max |x| so that max |x'| < 2^15: exact) is split as x' = x0 + x1 + r
// with x0 = fp16(x'), x1 = fp16(x' - x0) (round to nearest; the residual is exact in fp32), |r| <= 2^-22 |x'|
// for |x'| >= 2^-3 (both planes normal) and |r| <= 2^-25 below (fp16 subnormal spacing, i.e. <= 2^-40 of the
// tensor's max).  a b = (a0b0 + a0b1 + a1b0) / (s_a s_b) + O(2^-21 |ab|) on v_mfma_f32_32x32x16_f16 (exact
// fp16 products, fp32 accumulation): half the MFMAs of x6.  The scale comes from the producer's max-abs
// (amax) of the operand, so precision is normwise per tensor (fp32 GEMMs are normwise accurate as well).
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
using f16x2 = __attribute__((ext_vector_type(2))) _Float16;

__device__ __forceinline__ uint32_t split_pair_h(float& x, float& y) {
    const f32x2 v = {x, y};
    const f16x2 h = __builtin_convertvector(v, f16x2);
    x -= static_cast<float>(h[0]);
    y -= static_cast<float>(h[1]);
    return __builtin_bit_cast(uint32_t, h);
}

__device__ __forceinline__ uint32_t pack_pair_h(float x, float y) {
    const f32x2 v = {x, y};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2));
}

// float4 (already scaled) -> two planes of 4 fp16 (8 bytes each)
__device__ __forceinline__ void split4_h(float4 v, uint2& p0, uint2& p1) {
    p0.x = split_pair_h(v.x, v.y);
    p0.y = split_pair_h(v.z, v.w);
    p1.x = pack_pair_h(v.x, v.y);
    p1.y = pack_pair_h(v.z, v.w);
}

__device__ __forceinline__ f32x16 mfma_h3(const f16x8 (&a)[2], const f16x8 (&b)[2], f32x16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], acc, 0, 0, 0);
    return acc;
}

// Power-of-two scale for an operand whose max |x| is amax: amax * s < 2^15 (fp16 max 65504); 1 for a zero or
// non-finite amax (NaN / inf then propagate as in fp32).  Exponent clamped so that s and 1 / s are normal.
__host__ __device__ __forceinline__ float h3_scale(float amax) {
    if (!(amax > 0.f) || !(amax <= 3.4e38f)) return 1.f;
    const int biased = static_cast<int>((__builtin_bit_cast(uint32_t, amax) >> 23) & 0xff);
    const int e = (biased == 0 ? 1 : biased) - 126;  // amax < 2^e (subnormal amax: clamped below anyway)
    int k = 15 - e;
    k = k > 100 ? 100 : (k < -100 ? -100 : k);
    return __builtin_bit_cast(float, static_cast<uint32_t>(127 + k) << 23);
}

// Arithmetic traits by plane count: 3 = x6 (bf16), 2 = h3 (fp16).
template <int PL>
struct Arith;

template <>
struct Arith<3> {
    using frag = bf16x8;
    static __device__ __forceinline__ void split(float4 v, uint2 (&p)[3]) { split4(v, p[0], p[1], p[2]); }
    static __device__ __forceinline__ f32x16 mfma(const frag (&a)[3], const frag (&b)[3], f32x16 acc) {
        return mfma_x6(a, b, acc);
    }
};

template <>
struct Arith<2> {
    using frag = f16x8;
    static __device__ __forceinline__ void split(float4 v, uint2 (&p)[2]) { split4_h(v, p[0], p[1]); }
    static __device__ __forceinline__ f32x16 mfma(const frag (&a)[2], const frag (&b)[2], f32x16 acc) {
        return mfma_h3(a, b, acc);
    }
};

}  // namespace rslrl
