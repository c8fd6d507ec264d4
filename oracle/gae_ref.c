/*
 * ORACLE — test infrastructure only.  May be linked/called only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the CHECKER; never by the
 * product path (gymnasium-solver_amd/).
 *
 * Plain-C restatement of the reference's batched GAE(lambda):
 *   /root/reference/utils/returns_advantages.py:115-155
 *   (compute_batched_gae_advantages_and_returns), including the real-terminal mask
 *   of :6-16 (_real_terminal_mask / _non_terminal_float_mask).
 *
 * float32 numpy semantics reproduced exactly (NEP-50 weak python scalars):
 *   c1 = f32(gamma)                          -- `gamma * next_values[t]`          (:150)
 *   c2 = f32(gamma * gae_lambda in double)   -- `gamma * gae_lambda * gae`        (:151)
 *   nv[t] = v[t+1], nv[T-1] = last_values    (:135-137)
 *   nv = timeouts ? bootstrap : nv           (:140-142, only when bootstrap != NULL)
 *   nt = (done && !timeout) ? 0 : 1          (:145)
 *   delta = ((r + (c1*nv)*nt) - v)           (:150, left-to-right)
 *   gae   = delta + ((c2*gae)*nt)            (:151)
 *   ret   = adv + v                          (:154)
 * Build with -ffp-contract=off so no FMA contraction changes the rounding.
 * Pinned by tests/golden/gae.npz (generated from the reference by make_golden.py).
 */
#include <stdint.h>
#include <stdlib.h>

void oracle_gae_f32(const float *values, const float *rewards, const uint8_t *dones,
                    const uint8_t *timeouts, const float *bootstrap, const float *last_values,
                    int64_t T, int64_t N, double gamma, double gae_lambda, float *adv, float *ret)
{
    const float c1 = (float)gamma;
    const float c2 = (float)(gamma * gae_lambda);
    for (int64_t e = 0; e < N; ++e) {
        float gae = 0.0f;
        for (int64_t t = T - 1; t >= 0; --t) {
            const int64_t i = t * N + e;
            float nv = (t == T - 1) ? last_values[e] : values[i + N];
            if (bootstrap && timeouts[i]) nv = bootstrap[i];
            const float nt = (dones[i] && !timeouts[i]) ? 0.0f : 1.0f;
            float a = c1 * nv;
            a = a * nt;
            float delta = rewards[i] + a;
            delta = delta - values[i];
            float b = c2 * gae;
            b = b * nt;
            gae = delta + b;
            adv[i] = gae;
        }
    }
    for (int64_t i = 0; i < T * N; ++i) ret[i] = adv[i] + values[i];
}
