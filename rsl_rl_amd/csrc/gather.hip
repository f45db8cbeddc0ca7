// Multi-field row gather on gfx950 -- the mini-batch assembly of rsl_rl/storage/rollout_storage.py:168-197.
//
// The reference gathers eight fields per mini-batch with separate index_select kernels
// (`field.flatten(0, 1)[batch_idx]`).  Here one launch moves every field: a 256-thread block owns a
// tile of kTileRows destination rows, stages their int32 source indices in LDS once, and then copies
// each field's rows with lanes-per-row = next power of two >= row units, so a row is read as one
// contiguous run (16-byte units when the row size and pointers allow it, 4-byte units otherwise) and
// the destination is written fully coalesced.

#include "common.h"

namespace rslrl {
namespace {

constexpr int kTileRows = 256;

struct GatherField {
    const void* src;
    void* dst;
    int32_t units;      // row size in units
    int32_t log2_lpr;   // log2(lanes per row), lanes per row <= kBlock
    int32_t vec16;      // 1: 16-byte units, 0: 4-byte units
};

struct GatherParams {
    GatherField f[RSLRL_MAX_GATHER_FIELDS];
    int32_t nf;
};

template <typename U>
__device__ __forceinline__ void copy_field(const U* __restrict__ src, U* __restrict__ dst, int units, int log2_lpr,
                                           const int32_t* __restrict__ rows_idx, int64_t row0, int nrows) {
    const int lpr = 1 << log2_lpr;
    const int rows_per_pass = kBlock >> log2_lpr;
    const int lane = threadIdx.x & (lpr - 1);
    const int rsub = threadIdx.x >> log2_lpr;
    for (int r = rsub; r < nrows; r += rows_per_pass) {
        const int64_t s = static_cast<int64_t>(rows_idx[r]) * units;
        const int64_t d = (row0 + r) * units;
        for (int c = lane; c < units; c += lpr) dst[d + c] = src[s + c];
    }
}

__global__ __launch_bounds__(kBlock) void gather_rows_kernel(GatherParams p, const int32_t* __restrict__ indices,
                                                             int64_t num_rows) {
    __shared__ int32_t idx[kTileRows];
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * kTileRows;
    const int nrows = static_cast<int>(min<int64_t>(kTileRows, num_rows - row0));
    for (int r = threadIdx.x; r < nrows; r += kBlock) idx[r] = indices[row0 + r];
    __syncthreads();
    for (int f = 0; f < p.nf; ++f) {
        const GatherField g = p.f[f];
        if (g.vec16)
            copy_field(static_cast<const float4*>(g.src), static_cast<float4*>(g.dst), g.units, g.log2_lpr, idx, row0,
                       nrows);
        else
            copy_field(static_cast<const float*>(g.src), static_cast<float*>(g.dst), g.units, g.log2_lpr, idx, row0,
                       nrows);
    }
}

int log2_ceil_pow2(int64_t x) {
    int l = 0;
    while ((int64_t{1} << l) < x && l < 8) ++l;  // lanes per row capped at kBlock = 2^8
    return l;
}

}  // namespace
}  // namespace rslrl

using namespace rslrl;

extern "C" int rslrl_gather_rows(const rslrl_gather_field_t* fields, int32_t num_fields, const int32_t* indices,
                                 int64_t num_rows, rslrl_stream_t stream) {
    if (num_fields < 0 || num_fields > RSLRL_MAX_GATHER_FIELDS || num_rows < 0) return RSLRL_E_INVALID_ARGUMENT;
    if (num_rows == 0 || num_fields == 0) return RSLRL_OK;
    if (!fields || !indices) return RSLRL_E_INVALID_ARGUMENT;
    GatherParams p{};
    p.nf = num_fields;
    for (int i = 0; i < num_fields; ++i) {
        const rslrl_gather_field_t& f = fields[i];
        if (!f.src || !f.dst || f.row_bytes <= 0 || (f.row_bytes & 3)) return RSLRL_E_INVALID_ARGUMENT;
        const bool v16 = (f.row_bytes % 16 == 0) && ((reinterpret_cast<uintptr_t>(f.src) & 15) == 0) &&
                         ((reinterpret_cast<uintptr_t>(f.dst) & 15) == 0);
        const int64_t units = f.row_bytes / (v16 ? 16 : 4);
        if (units > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
        p.f[i] = GatherField{f.src, f.dst, static_cast<int32_t>(units), log2_ceil_pow2(units), v16 ? 1 : 0};
    }
    const int64_t nb = ceil_div(num_rows, kTileRows);
    if (nb > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
    hipLaunchKernelGGL(gather_rows_kernel, dim3(static_cast<unsigned>(nb)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), p, indices, num_rows);
    return launch_status();
}
