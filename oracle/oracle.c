/*
 * CPU ORACLE for the rsl_rl PPO hot path -- TEST INFRASTRUCTURE ONLY.
 *
 * This file is a plain-C restatement of the reference algorithm, used solely as the checker in
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  It is never linked into,
 * loaded by, or called from the product (rsl_rl_amd/), which must fail loudly without its HIP
 * library.
 *
 * Parity is PINNED: every function here is checked against the golden vectors in tests/golden/
 * that tests/golden/make_golden.py captured by running the reference (rsl-rl-lib 3.1.0, torch
 * 2.10.0 CPU) in the build container (tests/test_oracle_golden.py).
 *
 * Build: oracle/Makefile  (gcc -O2 -ffp-contract=off: every fp32 operation is rounded separately,
 * exactly like the reference's one-ATen-kernel-per-operation evaluation).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* --------------------------------------------------------------------------------------------
 * GAE  --  rsl_rl/storage/rollout_storage.py:127-145
 *
 *   for step = T-1 .. 0:
 *     next_values        = last_values if step == T-1 else values[step+1]          (:131-134)
 *     next_is_not_terminal = 1.0 - dones[step].float()                             (:136)
 *     delta     = rewards[step] + next_is_not_terminal * gamma * next_values - values[step]  (:138)
 *     advantage = delta + next_is_not_terminal * gamma * lam * advantage           (:140)
 *     returns[step] = advantage + values[step]                                     (:142)
 *   advantages = returns - values                                                  (:145)
 *
 * Python evaluates `a * gamma * b` left to right: ((nnt*gamma)*b), and the Python-float scalars are
 * applied as fp32 (ATen opmath for float tensors).  `advantage` starts as the int 0, so at the
 * first step `nnt*gamma*lam*0` is +0 and delta + 0 == delta.
 * Layout: values/rewards/dones/returns/advantages are [T, N] row-major, last_values [N].
 * ------------------------------------------------------------------------------------------*/
void oracle_gae(const float* values, const float* rewards, const uint8_t* dones, const float* last_values,
                float gamma, float lam, int64_t T, int64_t N, float* returns, float* advantages) {
    for (int64_t n = 0; n < N; ++n) {
        float adv = 0.0f;
        for (int64_t t = T - 1; t >= 0; --t) {
            const int64_t i = t * N + n;
            const float next_v = (t == T - 1) ? last_values[n] : values[i + N];
            const float nnt = 1.0f - (float)dones[i];
            const float a = nnt * gamma;
            const float b = a * next_v;
            const float c = rewards[i] + b;
            const float delta = c - values[i];
            const float d = (nnt * gamma) * lam;
            const float e = d * adv;
            adv = delta + e;
            returns[i] = adv + values[i];
        }
    }
    for (int64_t i = 0; i < T * N; ++i) advantages[i] = returns[i] - values[i];
}

/* Advantage normalisation  --  rollout_storage.py:148-149 (and ppo.py:221-223 per mini-batch):
 *   adv = (adv - adv.mean()) / (adv.std() + 1e-8)        std = unbiased (correction 1)
 * The statistics are accumulated in double and rounded to fp32 once (torch rounds its fp32
 * reduction result to fp32 as well); the elementwise part is fp32 like the reference.
 * n == 1 gives std = NaN exactly like torch (division by n-1 = 0).                              */
void oracle_adv_stats(const float* adv, int64_t n, float* mean_out, float* std_out) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += (double)adv[i];
    const double mean = s / (double)n;
    double ss = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        const double d = (double)adv[i] - mean;
        ss += d * d;
    }
    *mean_out = (float)mean;
    *std_out = (float)sqrt(ss / (double)(n - 1));
}

void oracle_adv_normalize(float* adv, int64_t n, float eps) {
    float mean, std;
    oracle_adv_stats(adv, n, &mean, &std);
    const float denom = std + eps;
    for (int64_t i = 0; i < n; ++i) adv[i] = (adv[i] - mean) / denom;
}

/* --------------------------------------------------------------------------------------------
 * torch CPU randperm  --  called at rollout_storage.py:165 with a CPU device
 *
 * torch 2.10 (aten/src/ATen/native/TensorFactories.cpp, randperm_cpu) fills r[i] = i and then, for
 * n < 2^32, runs Fisher-Yates with the CPU generator's 32-bit mt19937 output:
 *     for i in 0 .. n-2:  z = random() % (n - i);  swap(r[i], r[i + z])
 * The generator state is torch's CPUGeneratorImplState byte blob (Generator.get_state()):
 *     int64 the_initial_seed; int32 left; int32 seeded; uint64 next; uint64 state[624];
 *     double normal_x, normal_y, normal_rho; int32 normal_is_valid; (pad) ;
 *     float next_float_normal_sample; bool is_next_float_normal_sample_valid; (pad)
 * mt19937 here follows the published MT19937 algorithm (Matsumoto & Nishimura 1998), with torch's
 * state convention: `left` words remain before a twist, `next` indexes the next word.
 * ------------------------------------------------------------------------------------------*/
#define MT_N 624
#define MT_M 397

typedef struct {
    uint32_t s[MT_N];
    int left;
    int next;
} oracle_mt_t;

static void mt_twist(oracle_mt_t* m) {
    for (int i = 0; i < MT_N; ++i) {
        const uint32_t y = (m->s[i] & 0x80000000u) | (m->s[(i + 1) % MT_N] & 0x7fffffffu);
        uint32_t v = m->s[(i + MT_M) % MT_N] ^ (y >> 1);
        if (y & 1u) v ^= 0x9908b0dfu;
        m->s[i] = v;
    }
    m->left = MT_N;
    m->next = 0;
}

static uint32_t mt_next(oracle_mt_t* m) {
    if (--m->left <= 0) mt_twist(m);
    uint32_t y = m->s[m->next++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

enum { ST_SEED = 0, ST_LEFT = 8, ST_SEEDED = 12, ST_NEXT = 16, ST_STATE = 24 };

static void mt_load(oracle_mt_t* m, const uint8_t* blob) {
    int32_t left;
    uint64_t next;
    memcpy(&left, blob + ST_LEFT, 4);
    memcpy(&next, blob + ST_NEXT, 8);
    for (int i = 0; i < MT_N; ++i) {
        uint64_t w;
        memcpy(&w, blob + ST_STATE + 8 * i, 8);
        m->s[i] = (uint32_t)w;
    }
    m->left = left;
    m->next = (int)next;
}

static void mt_store(const oracle_mt_t* m, uint8_t* blob) {
    const int32_t left = m->left;
    const uint64_t next = (uint64_t)m->next;
    memcpy(blob + ST_LEFT, &left, 4);
    memcpy(blob + ST_NEXT, &next, 8);
    for (int i = 0; i < MT_N; ++i) {
        const uint64_t w = m->s[i];
        memcpy(blob + ST_STATE + 8 * i, &w, 8);
    }
}

/* Writes perm[0..n) and advances the state blob in place (as torch.randperm does). */
void oracle_randperm(uint8_t* state_blob, int64_t n, int64_t* perm) {
    oracle_mt_t m;
    mt_load(&m, state_blob);
    for (int64_t i = 0; i < n; ++i) perm[i] = i;
    for (int64_t i = 0; i + 1 < n; ++i) {
        const int64_t z = (int64_t)(mt_next(&m) % (uint32_t)(n - i));
        const int64_t t = perm[i];
        perm[i] = perm[i + z];
        perm[i + z] = t;
    }
    mt_store(&m, state_blob);
}

/* Row gather  --  rollout_storage.py:188-197 (`x.flatten(0,1)[batch_idx]`). */
void oracle_gather_rows(const uint8_t* src, int64_t row_bytes, const int64_t* idx, int64_t count, uint8_t* dst) {
    for (int64_t r = 0; r < count; ++r) memcpy(dst + r * row_bytes, src + idx[r] * row_bytes, (size_t)row_bytes);
}
