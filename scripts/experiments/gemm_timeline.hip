// Diagnostic: per-workgroup timeline of the x6 forward GEMM (s_memrealtime stamps at start, end of the
// main loop, end of the epilogue; 100 MHz) to see whether memory-bound epilogues overlap other
// workgroups' MFMA phases.  Builds mlp_gemm.hip with RSLRL_STAMPS.  Output: CSV on stdout.
#define RSLRL_STAMPS 1
#include "../../rsl_rl_amd/csrc/mlp_gemm.hip"
#include <cstdio>
#include <vector>
#include <cstdlib>

int main(int argc, char** argv) {
    const int64_t M = 393216;
    const int K = argc > 1 ? atoi(argv[1]) : 256, N = 256;
    float *x, *w, *b, *y;
    void* img;
    hipMalloc(&x, M * K * 4); hipMalloc(&w, N * K * 4); hipMalloc(&b, N * 4); hipMalloc(&y, M * N * 4);
    std::vector<float> hx(M * K);
    for (auto& v : hx) v = (rand() / (float)RAND_MAX) * 2.f - 1.f;
    hipMemcpy(x, hx.data(), M * K * 4, hipMemcpyHostToDevice);
    std::vector<float> hw(N * K);
    for (auto& v : hw) v = ((rand() / (float)RAND_MAX) * 2.f - 1.f) * 0.06f;
    hipMemcpy(w, hw.data(), N * K * 4, hipMemcpyHostToDevice);
    hipMemset(b, 0, N * 4);
    hipMalloc(&img, rslrl_linear_bimage_bytes(K));
    rslrl_linear_prepare_bimage(w, N, K, 0, img, nullptr);
    uint64_t* st;
    const int64_t tiles = M / 128;
    hipMalloc(&st, tiles * 2 * 6 * 8);
    hipMemcpyToSymbol(HIP_SYMBOL(rslrl::g_stamps), &st, sizeof(st));
    for (int i = 0; i < 10; ++i) rslrl_linear_fwd(x, M, K, w, N, b, 1, y, img, nullptr);
    hipDeviceSynchronize();
    std::vector<uint64_t> h(tiles * 2 * 6);
    hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    printf("wg,wave,t0,t1,t2,xcc,hwid,c0,c1\n");
    for (int64_t i = 0; i < tiles * 2; ++i)
        printf("%ld,%ld,%lu,%lu,%lu,%lu,%lu,%lu,%lu\n", i / 2, i % 2, h[6 * i], h[6 * i + 1], h[6 * i + 2],
               h[6 * i + 3] >> 32, h[6 * i + 3] & 0xffffffffu, h[6 * i + 4], h[6 * i + 5]);
    return 0;
}
