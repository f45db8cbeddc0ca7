// Multi-field row gather on gfx950 -- the mini-batch assembly of rsl_rl/storage/rollout_storage.py:168-197.
//
// The reference gathers eight fields per mini-batch with separate index_select kernels
// (`field.flatten(0, 1)[batch_idx]`).  Here one launch moves every field: a 256-thread block owns a
// tile of kTileRows destination rows, stages their int32 source indices in LDS once, and then copies
// each field's rows with lanes-per-row = next power of two >= row units, so a row is read as one
// contiguous run (16-byte units when the row size and pointers allow it, 4-byte units otherwise) and
// the destination is written fully coalesced.

#include <algorithm>

#include "common.h"
#include "launch_timing.h"

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

// ------------------------------------------------------------------------------------------------
// Transition records: the gathered fields of an env-step side by side in one record (RolloutStorage's
// record layout), so a random row costs the record's own 128-byte lines (3 for the 352 used bytes of a
// 384-byte C3 record) instead of >= one line per field.  A 256-thread block owns kRecTile (or
// kRecTile / 2 for records over 128 floats) destination rows: it reads each source record's used prefix in
// 16-byte units into an LDS tile (rows padded by one unit against bank conflicts), then writes every field
// as one contiguous [rows, width] block -- both sides coalesced.
// ------------------------------------------------------------------------------------------------
namespace rslrl {
namespace {

constexpr int kRecTile = 64;
constexpr int kRecLdsUnits = kRecTile * 33;  // 64 rows x (32 + 1) or 32 rows x (64 + 1) units of 16 bytes

struct RecField {
    int32_t offset;  // floats
    int32_t width;   // floats
    int32_t vec16;
    float* dst;
};

struct RecParams {
    RecField f[RSLRL_MAX_GATHER_FIELDS];
    int32_t nf;
    int32_t units;  // 16-byte units read per record
    int32_t tile;   // rows per block
    int32_t r4;     // record stride in 16-byte units
    const float4* side;  // optional: one 16-byte unit per row index (the slot array), staged after the record's units
};

__global__ __launch_bounds__(kBlock) void gather_records_kernel(RecParams p, const float4* __restrict__ rec,
                                                                const int32_t* __restrict__ indices, int64_t num_rows) {
    __shared__ float4 tile[kRecLdsUnits];
    __shared__ int32_t ridx[kRecTile];
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * p.tile;
    const int nrows = static_cast<int>(min<int64_t>(p.tile, num_rows - row0));
    for (int r = threadIdx.x; r < nrows; r += kBlock) ridx[r] = indices[row0 + r];
    __syncthreads();
    const unsigned RU = static_cast<unsigned>(p.units);  // record units of a row
    const unsigned U = RU + (p.side ? 1u : 0u);            // + the side unit (slot array) when present
    const int s4 = static_cast<int>(U) + 1;
    const unsigned total = static_cast<unsigned>(nrows) * U;
    // four independent 16-byte loads in flight per thread before their LDS stores
    for (unsigned k0 = threadIdx.x; k0 < total; k0 += 4 * kBlock) {
        float4 v[4];
        unsigned slot[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const unsigned k = k0 + j * kBlock;
            const unsigned kk = k < total ? k : total - 1;
            const unsigned r = kk / U, u = kk - r * U;
            slot[j] = r * s4 + u;
            const int64_t src = static_cast<int64_t>(ridx[r]);
            v[j] = u < RU ? rec[src * p.r4 + u] : p.side[src];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (k0 + j * kBlock < total) tile[slot[j]] = v[j];
    }
    __syncthreads();
    const float* tf = reinterpret_cast<const float*>(tile);
    for (int f = 0; f < p.nf; ++f) {
        const RecField g = p.f[f];
        if (g.vec16) {
            const unsigned w4 = static_cast<unsigned>(g.width >> 2), o4 = static_cast<unsigned>(g.offset >> 2);
            float4* d = reinterpret_cast<float4*>(g.dst) + row0 * w4;
            const unsigned n = static_cast<unsigned>(nrows) * w4;
            for (unsigned k = threadIdx.x; k < n; k += kBlock) {
                const unsigned r = k / w4, c = k - r * w4;
                d[k] = tile[r * s4 + o4 + c];
            }
        } else {
            const unsigned w = static_cast<unsigned>(g.width);
            float* d = g.dst + row0 * w;
            const unsigned n = static_cast<unsigned>(nrows) * w;
            for (unsigned k = threadIdx.x; k < n; k += kBlock) {
                const unsigned r = k / w, c = k - r * w;
                d[k] = tf[(r * s4) * 4 + g.offset + c];
            }
        }
    }
}

// One thread per 16-byte unit of a slot: consecutive lanes cover a slot's units in order, so each slot
// leaves the store as whole 64-byte pieces (partial ones are read-modify-writes at the HBM).
__global__ __launch_bounds__(kBlock) void record_fill_slot_kernel(float* __restrict__ rec, int64_t R, int64_t offset,
                                                                  int su, const float* __restrict__ row, int rw,
                                                                  const float* c0, const float* c1, const float* c2,
                                                                  const float* c3, int nc, uint32_t total) {
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t k = blockIdx.x * kBlock + threadIdx.x; k < total; k += stride) {
        const uint32_t i = k / static_cast<uint32_t>(su);
        const int u = static_cast<int>(k - i * su);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int f = 4 * u + e;
            const int c = f - rw;
            v[e] = f < rw ? row[static_cast<int64_t>(i) * rw + f]
                          : c == 0 && nc > 0 ? c0[i]
                          : c == 1 && nc > 1 ? c1[i]
                          : c == 2 && nc > 2 ? c2[i]
                          : c == 3 && nc > 3 ? c3[i] : 0.f;
        }
        *reinterpret_cast<float4*>(rec + static_cast<int64_t>(i) * R + offset + 4 * u) = make_float4(v[0], v[1], v[2], v[3]);
    }
}

}  // namespace
}  // namespace rslrl

namespace {
int gather_records_impl(const float* records, int64_t record_floats, const rslrl_record_field_t* fields,
                        int32_t num_fields, const float* side, const rslrl_record_field_t* side_fields,
                        int32_t num_side, const int32_t* indices, int64_t num_rows, rslrl_stream_t stream) {
    if (num_fields < 0 || num_side < 0 || num_fields + num_side > RSLRL_MAX_GATHER_FIELDS || num_rows < 0)
        return RSLRL_E_INVALID_ARGUMENT;
    if (num_rows == 0 || num_fields + num_side == 0) return RSLRL_OK;
    if (!records || (num_fields && !fields) || !indices || record_floats <= 0 || (record_floats & 3))
        return RSLRL_E_INVALID_ARGUMENT;
    if (num_side && (!side || !side_fields)) return RSLRL_E_INVALID_ARGUMENT;
    if ((reinterpret_cast<uintptr_t>(records) & 15) || (side && (reinterpret_cast<uintptr_t>(side) & 15)))
        return RSLRL_E_MISALIGNED;
    RecParams p{};
    p.nf = num_fields + num_side;
    int64_t used = 0;
    for (int i = 0; i < num_fields; ++i) {
        const rslrl_record_field_t& f = fields[i];
        if (!f.dst || f.width < 1 || f.offset < 0 || f.offset + f.width > record_floats) return RSLRL_E_INVALID_ARGUMENT;
        used = std::max<int64_t>(used, f.offset + f.width);
    }
    if (used > RSLRL_MAX_RECORD_FLOATS) return RSLRL_E_UNSUPPORTED;
    p.units = static_cast<int32_t>((used + 3) / 4);
    const int64_t side_off = 4 * static_cast<int64_t>(p.units);  // the side unit's floats follow the record's units
    for (int i = 0; i < num_fields + num_side; ++i) {
        const bool is_side = i >= num_fields;
        const rslrl_record_field_t& f = is_side ? side_fields[i - num_fields] : fields[i];
        if (is_side && (!f.dst || f.width < 1 || f.offset < 0 || f.offset + f.width > 4)) return RSLRL_E_INVALID_ARGUMENT;
        const int64_t off = is_side ? side_off + f.offset : f.offset;
        const bool v16 = (f.width % 4 == 0) && (off % 4 == 0) && ((reinterpret_cast<uintptr_t>(f.dst) & 15) == 0);
        p.f[i] = RecField{static_cast<int32_t>(off), static_cast<int32_t>(f.width), v16 ? 1 : 0, f.dst};
    }
    p.side = num_side ? reinterpret_cast<const float4*>(side) : nullptr;
    const int32_t units_all = p.units + (num_side ? 1 : 0);
    p.tile = units_all <= 32 ? kRecTile : kRecTile / 2;
    if (static_cast<int64_t>(p.tile) * (units_all + 1) > kRecLdsUnits) return RSLRL_E_UNSUPPORTED;
    if (record_floats / 4 > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
    p.r4 = static_cast<int32_t>(record_floats / 4);
    const int64_t nb = ceil_div(num_rows, p.tile);
    if (nb > INT32_MAX) return RSLRL_E_INVALID_ARGUMENT;
    launch_timed(kTagGatherRecords, gather_records_kernel, dim3(static_cast<unsigned>(nb)), dim3(kBlock), 0,
                 reinterpret_cast<hipStream_t>(stream), p, reinterpret_cast<const float4*>(records), indices, num_rows);
    return launch_status();
}
}  // namespace

extern "C" int rslrl_gather_records(const float* records, int64_t record_floats, const rslrl_record_field_t* fields,
                                    int32_t num_fields, const int32_t* indices, int64_t num_rows,
                                    rslrl_stream_t stream) {
    return gather_records_impl(records, record_floats, fields, num_fields, nullptr, nullptr, 0, indices, num_rows,
                               stream);
}

extern "C" int rslrl_gather_records_side(const float* records, int64_t record_floats,
                                         const rslrl_record_field_t* fields, int32_t num_fields, const float* side,
                                         const rslrl_record_field_t* side_fields, int32_t num_side_fields,
                                         const int32_t* indices, int64_t num_rows, rslrl_stream_t stream) {
    return gather_records_impl(records, record_floats, fields, num_fields, side, side_fields, num_side_fields, indices,
                               num_rows, stream);
}

extern "C" int rslrl_record_fill_slot(float* records, int64_t record_floats, int64_t offset, int32_t slot_floats,
                                      const float* row_src, int32_t row_width, const float* const* columns,
                                      int32_t num_columns, int64_t n, rslrl_stream_t stream) {
    if (n < 0 || record_floats <= 0 || (record_floats & 3) || offset < 0 || (offset & 3) || slot_floats <= 0 ||
        (slot_floats & 3) || slot_floats > 64 || offset + slot_floats > record_floats || row_width < 0 ||
        num_columns < 0 || num_columns > 4 || row_width + num_columns > slot_floats)
        return RSLRL_E_INVALID_ARGUMENT;
    if (n == 0) return RSLRL_OK;
    if (!records || (row_width > 0 && !row_src) || (num_columns > 0 && !columns)) return RSLRL_E_INVALID_ARGUMENT;
    if (reinterpret_cast<uintptr_t>(records) & 15) return RSLRL_E_MISALIGNED;
    const float* c[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int j = 0; j < num_columns; ++j) {
        if (!columns[j]) return RSLRL_E_INVALID_ARGUMENT;
        c[j] = columns[j];
    }
    const int su = slot_floats / 4;
    if (n * su > UINT32_MAX / 2) return RSLRL_E_INVALID_ARGUMENT;
    const uint32_t total = static_cast<uint32_t>(n * su);
    const int64_t nb = std::min<int64_t>(ceil_div(total, kBlock), 8192);
    hipLaunchKernelGGL(record_fill_slot_kernel, dim3(static_cast<unsigned>(nb)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), records, record_floats, offset, su, row_src, row_width,
                       c[0], c[1], c[2], c[3], num_columns, total);
    return launch_status();
}
