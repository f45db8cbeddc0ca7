// Three-way bf16 split of fp32 operands for the "x6" GEMMs (mlp_gemm.hip, mlp_wgrad.hip).
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

}  // namespace rslrl
