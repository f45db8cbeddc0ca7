// Internal interface of the streaming hidden-layer forward (mlp_fwd_stream.hip), called by rslrl_linear_gemm_pair for
// RSLRL_LINEAR_FWD_ELU on x6 with N = 256, K = 256 or 48 and M a multiple of 128 (no C ABI of its own: same entry point, same
// bits as the tiled kernel).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

namespace rslrl {

struct FwdStreamProblem {
    const float* x;     // [M, K] layer input
    const void* img;    // x6 image of W (layout 0)
    const float* bias;  // [256]
    float* h;           // [M, 256] output ELU(x W^T + b)
};

bool fwd_stream_enabled();  // RSLRL_FWD_STREAM=0 keeps the tiled kernel (A/B)
bool fwd_stream_forced();   // RSLRL_FWD_STREAM=1 (or 48): every M, not only the sizes where it measured faster
bool fwd_stream48();        // RSLRL_FWD_STREAM=48: the 48-wide first layer too (opt-in: slower, see the call site)
int fwd_stream_pair(const FwdStreamProblem* p, int n, int64_t M, int K, hipStream_t st);  // K = 256 or 48


// the critic's fused head on the streaming main loop (default; RSLRL_VALUE_HEAD_STREAM=0: the tiled head); rslrl_value_head_fwd_bwd's
// inputs and outputs, the [dW | db] partials one 260-float row per slice (value_head_stream_rows(M) rows)
struct ValueHeadStreamArgs {
    const float* x;
    const void* img;
    const float* bias;
    const float* wv;
    const float* bv;
    const float* tv;
    const float* ret;
    float* dz;
    float* y;
    float* wpart;
    float clip, g;
    int clipped;
    int64_t M;
};
bool value_head_stream_enabled();
int value_head_stream(const ValueHeadStreamArgs& v, hipStream_t st);
int64_t value_head_stream_rows(int64_t M);

}  // namespace rslrl
