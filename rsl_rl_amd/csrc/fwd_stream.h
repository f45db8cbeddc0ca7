// Internal interface of the streaming hidden-layer forward (mlp_fwd_stream.hip), called by rslrl_linear_gemm_pair for
// RSLRL_LINEAR_FWD_ELU on x6 with K = N = 256 and M a multiple of 128 (no C ABI of its own: same entry point, same
// bits as the tiled kernel).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

namespace rslrl {

struct FwdStreamProblem {
    const float* x;     // [M, 256] layer input
    const void* img;    // x6 image of W (layout 0)
    const float* bias;  // [256]
    float* h;           // [M, 256] output ELU(x W^T + b)
};

bool fwd_stream_enabled();  // RSLRL_FWD_STREAM=0 keeps the tiled kernel (A/B)
int fwd_stream_pair(const FwdStreamProblem* p, int n, int64_t M, hipStream_t st);

}  // namespace rslrl
