// Diagnostic: per-workgroup timeline of the critic's fused output layer (op 101: value head, H stored) and of the
// value head with its backward (op 200: rslrl_value_head_fwd_bwd) at M = 393216, from s_memrealtime / s_memtime
// stamps (RSLRL_STAMPS build): start, end of the main loop, end of the epilogue.  Prints a summary per op.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -mcode-object-version=5 \
//     scripts/experiments/value_head_timeline.hip rsl_rl_amd/csrc/status.cpp -I include -o vh_tl
#define RSLRL_STAMPS 1
#include "../../rsl_rl_amd/csrc/mlp_gemm.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

static void fill(float* d, size_t n, float scale, unsigned seed) {
    std::vector<float> h(n);
    srand(seed);
    for (auto& v : h) v = ((rand() / (float)RAND_MAX) * 2.f - 1.f) * scale;
    hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
}

int main() {
    const int64_t M = 393216;
    const int K = 256, N = 256;
    float *x, *w, *b, *y, *hh, *cs;
    void* img;
    hipMalloc(&x, M * K * 4); hipMalloc(&w, N * K * 4); hipMalloc(&b, N * 4); hipMalloc(&y, M * N * 4);
    hipMalloc(&hh, M * N * 4); hipMalloc(&cs, (M / 128) * N * 4);
    fill(x, M * K, 1.f, 1); fill(w, N * K, 0.06f, 2); fill(hh, M * N, 1.f, 3);
    hipMemset(b, 0, N * 4);
    hipMalloc(&img, rslrl_linear_bimage_bytes(K));
    rslrl_linear_prepare_bimage(w, N, K, 0, img, nullptr);
    const int64_t tiles = M / 128;
    uint64_t* st;
    hipMalloc(&st, tiles * 2 * 6 * 8);
    hipMemcpyToSymbol(HIP_SYMBOL(rslrl::g_stamps), &st, sizeof(st));
    float *wo, *bo, *yo;
    void* oimg;
    hipMalloc(&wo, 12 * K * 4); hipMalloc(&bo, 12 * 4); hipMalloc(&yo, M * 12 * 4);
    fill(wo, 12 * K, 0.06f, 4); hipMemset(bo, 0, 12 * 4);
    hipMalloc(&oimg, rslrl_linear_out_image_bytes());
    float *tv, *ret, *wpart;
    hipMalloc(&tv, M * 4); hipMalloc(&ret, M * 4); hipMalloc(&wpart, tiles * 260 * 4);
    fill(tv, M, 1.f, 5); fill(ret, M, 1.f, 6);
    for (int op : {100 + 1, 200, 100 + 1, 200}) {
        rslrl_linear_args_t a{};
        a.op = op; a.arith = RSLRL_ARITH_X6; a.a = x; a.M = M; a.K = K; a.N = N; a.bimage = img;
        a.bias = b; a.c = y; a.h = hh; a.colsum_partials = cs;
        if (op > 100) {  // fused last hidden + output layer with op - 100 outputs
            const int nout = op == 200 ? 1 : op - 100;
            rslrl_bimage_desc_t d{wo, oimg, nout, K, 0, RSLRL_BIMAGE_LAYOUT_OUT};
            rslrl_linear_prepare_bimages(&d, 1, nullptr);
            a.op = RSLRL_LINEAR_FWD_OUT; a.out_image = oimg; a.out_bias = bo; a.y = yo; a.nout = nout;
        }
        rslrl_value_head_args_t v{tv, ret, wo, 0.2f, 1.0f, 1, wpart, nullptr};
        for (int i = 0; i < 20; ++i) {
            const int rc = op == 200 ? rslrl_value_head_fwd_bwd(&a, &v, nullptr) : rslrl_linear_gemm(&a, nullptr);
            if (rc) { printf("op %d rc %d\n", op, rc); return 1; }
        }
        hipDeviceSynchronize();
        std::vector<uint64_t> h(tiles * 2 * 6);
        hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
        uint64_t t_min = ~0ull, t_max = 0;
        double ml = 0, ep = 0, clk = 0, busy = 0;
        std::vector<double> mls;
        for (int64_t i = 0; i < tiles; ++i) {
            const uint64_t* s = &h[12 * i];  // wave 0 of workgroup i
            t_min = std::min(t_min, s[0]);
            t_max = std::max(t_max, s[2]);
            ml += double(s[1] - s[0]);
            ep += double(s[2] - s[1]);
            busy += double(s[2] - s[0]);
            clk += double(s[5] - s[4]) / double(s[1] - s[0]) * 0.1;  // GHz
            mls.push_back(double(s[1] - s[0]));
        }
        std::sort(mls.begin(), mls.end());
        const double span = double(t_max - t_min);
        printf("op %d: span %.1f us  mean main loop %.2f us (p10 %.2f p90 %.2f)  mean epilogue %.2f us  clock %.2f GHz  "
               "slot occupancy %.3f (2 workgroups x 256 CUs)\n",
               op, span / 100, ml / tiles / 100, mls[tiles / 10] / 100, mls[9 * tiles / 10] / 100, ep / tiles / 100,
               clk / tiles, busy / (span * 512));
        // per-workgroup records for offline analysis: start, loop end, end (10 ns ticks from t_min), XCC, CU id
        char fn[64];
        snprintf(fn, sizeof(fn), "gpurun_out/vh_tl_op%d.csv", op);
        if (FILE* f = fopen(fn, "w")) {
            fprintf(f, "wg,t0,t1,t2,xcc,hwid\n");
            for (int64_t i = 0; i < tiles; ++i) {
                const uint64_t* s = &h[12 * i];
                fprintf(f, "%ld,%lu,%lu,%lu,%lu,%lu\n", i, s[0] - t_min, s[1] - t_min, s[2] - t_min, s[3] >> 32,
                        s[3] & 0xffffffffu);
            }
            fclose(f);
        }
    }
    return 0;
}
