// Host-side permutation with torch CPU randperm semantics -- rsl_rl/storage/rollout_storage.py:165.
//
// The reference draws `torch.randperm(num_mini_batches * mini_batch_size)` once per update and reuses
// it for every epoch.  On a CPU generator torch 2.x computes it as Fisher-Yates over the generator's
// 32-bit mt19937 stream: for i in [0, n-1): z = u32() % (n - i); swap(r[i], r[i + z]).  This file
// reproduces that permutation (and the generator-state advance) bit for bit from the state blob of
// torch.Generator.get_state(), then the caller uploads it (int32) for the device gathers.
//
// The serial chain is the swap sequence, not the RNG, so it is split in two passes:
//   1. draw all n-1 words in 624-word mt19937 blocks and reduce them mod (n - i) with an exact
//      double-reciprocal quotient + one-step correction (no integer division);
//   2. run the swaps with a software prefetch of r[i + z] kPrefetch iterations ahead, so the random
//      accesses of a 1.5 M-entry table overlap instead of serialising on cache misses.

#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/rslrl_amd.h"

namespace {

constexpr int kN = 624;
constexpr int kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu;
constexpr uint32_t kUpper = 0x80000000u;
constexpr uint32_t kLower = 0x7fffffffu;

// torch CPUGeneratorImplState (aten/src/ATen/CPUGeneratorImpl.cpp): legacy_pod {int64 seed; int32 left;
// int32 seeded; uint64 next; uint64 state[624]; double normal_x, normal_y, normal_rho; int32 valid}, then
// float next_float_normal_sample; bool valid.  5056 bytes on x86-64.
constexpr size_t kStateBytes = 5056;
constexpr size_t kOffLeft = 8;
constexpr size_t kOffNext = 16;
constexpr size_t kOffWords = 24;

struct Mt19937 {
    uint32_t s[kN];
    int left;  // words left before the next twist is due (torch: `--left == 0` triggers it)
    int next;  // index of the next output word

    inline uint32_t mix(uint32_t u, uint32_t v) const {
        const uint32_t y = (u & kUpper) | (v & kLower);
        return (y >> 1) ^ ((v & 1u) ? kMatrixA : 0u);
    }

    void twist() {
        int i = 0;
        for (; i < kN - kM; ++i) s[i] = s[i + kM] ^ mix(s[i], s[i + 1]);
        for (; i < kN - 1; ++i) s[i] = s[i + kM - kN] ^ mix(s[i], s[i + 1]);
        s[kN - 1] = s[kM - 1] ^ mix(s[kN - 1], s[0]);
        left = kN;
        next = 0;
    }

    static inline uint32_t temper(uint32_t y) {
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }

    // Fills out[0..count) with the next `count` outputs.
    void fill(uint32_t* out, int64_t count) {
        int64_t k = 0;
        while (k < count) {
            if (left <= 1) {  // the next call would twist first
                twist();
                // after a twist torch hands out s[0] with left = N - 1 remaining
                left = kN + 1;
            }
            // words available before the next twist: left - 1
            int64_t avail = static_cast<int64_t>(left) - 1;
            if (avail > count - k) avail = count - k;
            for (int64_t j = 0; j < avail; ++j) out[k + j] = temper(s[next + j]);
            next += static_cast<int>(avail);
            left -= static_cast<int>(avail);
            k += avail;
        }
    }
};

bool load_state(const uint8_t* blob, Mt19937& m) {
    int32_t left;
    uint64_t next;
    std::memcpy(&left, blob + kOffLeft, 4);
    std::memcpy(&next, blob + kOffNext, 8);
    if (left < 1 || left > kN || next > static_cast<uint64_t>(kN)) return false;
    if (left > 1 && static_cast<int64_t>(next) + left - 1 > kN) return false;  // would read past s[N-1]
    for (int i = 0; i < kN; ++i) {
        uint64_t w;
        std::memcpy(&w, blob + kOffWords + 8 * static_cast<size_t>(i), 8);
        m.s[i] = static_cast<uint32_t>(w);
    }
    m.left = left;
    m.next = static_cast<int>(next);
    return true;
}

void store_state(uint8_t* blob, const Mt19937& m) {
    const int32_t left = m.left;
    const uint64_t next = static_cast<uint64_t>(m.next);
    std::memcpy(blob + kOffLeft, &left, 4);
    std::memcpy(blob + kOffNext, &next, 8);
    for (int i = 0; i < kN; ++i) {
        const uint64_t w = m.s[i];
        std::memcpy(blob + kOffWords + 8 * static_cast<size_t>(i), &w, 8);
    }
}

// u mod m for u < 2^32, 1 <= m < 2^32, without a hardware divide: the double quotient is within one
// of floor(u / m), and the remainder is corrected into [0, m).
inline uint32_t mod_u32(uint32_t u, uint32_t m, double inv_m) {
    const int64_t q = static_cast<int64_t>(static_cast<double>(u) * inv_m);
    int64_t r = static_cast<int64_t>(u) - q * static_cast<int64_t>(m);
    if (r < 0) r += m;
    else if (r >= static_cast<int64_t>(m)) r -= m;
    return static_cast<uint32_t>(r);
}

constexpr int64_t kPrefetch = 24;

}  // namespace

extern "C" int rslrl_randperm_mt19937(uint8_t* state, size_t state_bytes, int64_t n, int32_t* out) {
    if (!state || state_bytes != kStateBytes) return RSLRL_E_BAD_GENERATOR_STATE;
    if (n < 0 || n >= (int64_t{1} << 31)) return RSLRL_E_INVALID_ARGUMENT;
    if (n > 0 && !out) return RSLRL_E_INVALID_ARGUMENT;
    Mt19937 m;
    if (!load_state(state, m)) return RSLRL_E_BAD_GENERATOR_STATE;
    for (int64_t i = 0; i < n; ++i) out[i] = static_cast<int32_t>(i);
    if (n > 1) {
        std::vector<uint32_t> z(static_cast<size_t>(n - 1));
        m.fill(z.data(), n - 1);
        for (int64_t i = 0; i < n - 1; ++i) {
            const uint32_t span = static_cast<uint32_t>(n - i);
            z[i] = mod_u32(z[i], span, 1.0 / static_cast<double>(span));
        }
        const int64_t last = n - 1;
        for (int64_t i = 0; i < last; ++i) {
            if (i + kPrefetch < last) __builtin_prefetch(out + (i + kPrefetch) + z[i + kPrefetch], 1, 0);
            const int64_t j = i + z[i];
            const int32_t t = out[i];
            out[i] = out[j];
            out[j] = t;
        }
    }
    store_state(state, m);
    return RSLRL_OK;
}
