// Characterise how v_mfma_f32_32x32x16_bf16 rounds when it adds its 16 exact products to the f32
// accumulator (does it round-to-nearest, truncate, or lose small addends?).  Output row 0, col 0 only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cmath>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k(const float* av, const float* bv, float c0, float* out) {
    // lane l: A[row l&31][k 8(l>>5)+j], B[k 8(l>>5)+j][col l&31]; only row 0 / col 0 nonzero
    const int l = threadIdx.x;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        const int kk = 8 * (l >> 5) + j;
        a[j] = (__bf16)((l & 31) == 0 ? av[kk] : 0.f);
        b[j] = (__bf16)((l & 31) == 0 ? bv[kk] : 0.f);
    }
    f32x16 c = {};
    c[0] = (l == 0) ? c0 : 0.f;
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    if (l == 0) out[0] = c[0];
}

static float run(const float* a, const float* b, float c0) {
    float *da, *db, *dout, r;
    hipMalloc(&da, 64); hipMalloc(&db, 64); hipMalloc(&dout, 4);
    hipMemcpy(da, a, 64, hipMemcpyHostToDevice); hipMemcpy(db, b, 64, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, c0, dout);
    hipMemcpy(&r, dout, 4, hipMemcpyDeviceToHost);
    hipFree(da); hipFree(db); hipFree(dout);
    return r;
}

int main() {
    float a[16], b[16];
    auto reset = [&] { for (int i = 0; i < 16; ++i) { a[i] = 0.f; b[i] = 0.f; } };
    // 1: sixteen products of 2^-25 onto 1.0: exact 1 + 2^-21
    reset(); for (int i = 0; i < 16; ++i) { a[i] = ldexpf(1, -12); b[i] = ldexpf(1, -13); }
    printf("t1 16x2^-25 + 1: got 1%+.3e exact %+.3e\n", run(a, b, 1.f) - 1.f, ldexpf(1, -21));
    // 2: one product 1.5 * 2^-24 onto 1: RNE -> 1 + 2^-23, truncation -> 1
    reset(); a[0] = 3 * ldexpf(1, -13); b[0] = ldexpf(1, -12);
    printf("t2 1.5*2^-24 + 1: got 1%+.3e (RNE %+.3e)\n", run(a, b, 1.f) - 1.f, ldexpf(1, -23));
    // 3: negative: -1.5*2^-24 onto 1: RNE -> 1 - 2^-24 (ulp below 1 is 2^-24)
    reset(); a[0] = -3 * ldexpf(1, -13); b[0] = ldexpf(1, -12);
    printf("t3 -1.5*2^-24 + 1: got 1%+.3e (exact %+.3e, RNE %+.3e)\n", run(a, b, 1.f) - 1.f, -1.5 * ldexpf(1, -24), -ldexpf(1, -24));
    // 4: 0.75 ulp product: RNE rounds up, truncation down
    reset(); a[0] = 3 * ldexpf(1, -14); b[0] = ldexpf(1, -11);
    printf("t4 0.75ulp + 1: got 1%+.3e (RNE %+.3e)\n", run(a, b, 1.f) - 1.f, ldexpf(1, -23));
    // 5: two products that cancel at large magnitude + a small one: 2^10 - 2^10 + 2^-20 onto 0
    reset(); a[0] = 1024.f; b[0] = 1.f; a[1] = -1024.f; b[1] = 1.f; a[2] = ldexpf(1, -10); b[2] = ldexpf(1, -10);
    printf("t5 cancel: got %.6e exact %.6e\n", run(a, b, 0.f), ldexpf(1, -20));
    // 6: 1 + 16 small positive products each 0.25 ulp: exact +4 quarter-ulps = +1 ulp
    reset(); for (int i = 0; i < 16; ++i) { a[i] = ldexpf(1, -13); b[i] = ldexpf(1, -12); }
    printf("t6 16 x 0.25ulp: got 1%+.3e exact %+.3e\n", run(a, b, 1.f) - 1.f, 16 * ldexpf(1, -25));
    return 0;
}
