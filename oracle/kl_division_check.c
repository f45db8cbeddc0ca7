/* Test infrastructure (not shipped): checks the division the loss kernel's shared-sigma KL uses
 * (csrc/ppo_loss.hip, ppo_loss_quad_kernel) against IEEE fp32 true division -- the reference's
 * `(old_sigma^2 + (old_mu - mu)^2) / (2 * sigma^2)` (rsl_rl/algorithms/ppo.py:262-266):
 *   r = RN(1/D), q0 = RN(n * r), q = fma(fma(-q0, D, n), r, q0)  ==  RN(n / D)
 * for n, D in [2^-60, 2^60] (the range the kernel admits to this path; Markstein's correction theorem).
 * Usage: kl_division_check [divisors] [numerators per divisor]; prints "tot <cases> bad <mismatches>". */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t st = 88172645463325252ull;
static uint64_t next(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
/* a float with random bits in [2^-60, 2^60] */
static float rand_in_range(void) {
    for (;;) {
        uint32_t u = (uint32_t)next() & 0x7fffffffu;
        float f;
        memcpy(&f, &u, 4);
        if (f >= 0x1p-60f && f <= 0x1p60f) return f;
    }
}

int main(int argc, char** argv) {
    const long nd = argc > 1 ? atol(argv[1]) : 20000, nn = argc > 2 ? atol(argv[2]) : 1000;
    long tot = 0, bad = 0;
    for (long di = 0; di < nd; ++di) {
        float D;
        if (di & 1) {
            D = rand_in_range();
        } else { /* D = 2 * sigma^2 for a policy-like sigma */
            const float s = (float)(next() % 1000000) * 3e-6f + 1e-3f;
            D = 2.0f * (s * s);
        }
        const float r = 1.0f / D;
        for (long i = 0; i < nn; ++i) {
            float n;
            if (i & 1) {
                n = rand_in_range();
            } else { /* old_sigma^2 + dmu^2 with policy-like magnitudes */
                const float os = (float)(next() % 1000000) * 3e-6f + 1e-3f;
                const float dm = ((float)(next() % 2000001) - 1e6f) * 1e-6f;
                n = os * os + dm * dm;
            }
            if (n < 0x1p-60f || n > 0x1p60f) continue;
            volatile float q = n / D;
            const float q0 = n * r;
            const float q1 = fmaf(fmaf(-q0, D, n), r, q0);
            ++tot;
            if (q1 != q) {
                if (bad < 5) printf("mismatch n=%a D=%a q=%a got %a\n", n, D, q, q1);
                ++bad;
            }
        }
    }
    printf("tot %ld bad %ld\n", tot, bad);
    return bad != 0;
}
