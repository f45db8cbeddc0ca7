// Does v_mfma_f32_32x32x16_bf16 give the same bits for D = A B and for D^T = B^T A^T (operands swapped, output
// transposed)?  If so, an x6 chain on C^T accumulators with each product's operands swapped (same product order) is
// bit-identical to the C chain.  Random bf16 operands of mixed magnitudes, 1000 trials, fp32 accumulator chains.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/mfma_symmetry_probe.hip -o scripts/mfma_symmetry_probe.bin
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// A: [32 rows][16 k] bf16, B: [16 k][32 cols] bf16 (row-major); C chain of `steps` MFMAs over different A/B pairs
__global__ void chain(const uint16_t* A, const uint16_t* B, float* outC, float* outCT, int steps) {
    const int lane = threadIdx.x;
    const int l32 = lane & 31, h = lane >> 5;
    f32x16 c = {}, ct = {};
    for (int s = 0; s < steps; ++s) {
        const uint16_t* a = A + s * 32 * 16;
        const uint16_t* b = B + s * 16 * 32;
        // operand fragments of 32x32x16: lane holds row (A) / column (B) l32, k = 8 h .. 8 h + 7
        uint16_t fa[8], fb[8];
        for (int j = 0; j < 8; ++j) {
            fa[j] = a[l32 * 16 + 8 * h + j];
            fb[j] = b[(8 * h + j) * 32 + l32];
        }
        bf16x8 va, vb;
        memcpy(&va, fa, 16);
        memcpy(&vb, fb, 16);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, vb, c, 0, 0, 0);   // D = A B
        ct = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vb, va, ct, 0, 0, 0);  // D^T = B^T A^T
    }
    // D[i][j]: lane holds column l32, rows (r & 3) + 8 (r >> 2) + 4 h; D^T[j][i] the same positions transposed
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        outC[row * 32 + l32] = c[r];
        outCT[l32 * 32 + row] = ct[r];  // element (row of D^T = l32's ... ) -> stored as D[row][l32] transposed back
    }
}

static uint16_t to_bf16(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    return static_cast<uint16_t>((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

int main() {
    const int steps = 6, trials = 1000;
    std::mt19937 rng(1);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::uniform_int_distribution<int> ex(-20, 20);
    uint16_t *dA, *dB;
    float *dC, *dCT;
    hipMalloc(&dA, steps * 512 * 2);
    hipMalloc(&dB, steps * 512 * 2);
    hipMalloc(&dC, 1024 * 4);
    hipMalloc(&dCT, 1024 * 4);
    std::vector<uint16_t> A(steps * 512), B(steps * 512);
    std::vector<float> C(1024), CT(1024);
    long mism = 0, total = 0;
    for (int t = 0; t < trials; ++t) {
        for (auto& v : A) v = to_bf16(std::ldexp(nd(rng), ex(rng) / 4));
        for (auto& v : B) v = to_bf16(std::ldexp(nd(rng), ex(rng) / 4));
        hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, dA, dB, dC, dCT, steps);
        hipMemcpy(C.data(), dC, 4096, hipMemcpyDeviceToHost);
        hipMemcpy(CT.data(), dCT, 4096, hipMemcpyDeviceToHost);
        // CT was stored transposed: CT[l32 * 32 + row] holds D^T's (l32-th row?) -- compare D[i][j] with D^T[j][i]
        for (int i = 0; i < 32; ++i)
            for (int j = 0; j < 32; ++j) {
                ++total;
                // D^T computed with A := B^T: D^T[p][q] at lane column q, row p.  The kernel wrote ct (D^T[row][l32])
                // to CT[l32 * 32 + row], i.e. CT[q * 32 + p] = D^T[p][q] = D[q][p] -> CT[i * 32 + j] = D[i][j]
                if (memcmp(&C[i * 32 + j], &CT[i * 32 + j], 4) != 0) ++mism;
            }
    }
    printf("{\"elements\": %ld, \"bit_mismatches\": %ld, \"steps\": %d}\n", total, mism, steps);
    return 0;
}
