/* TEST INFRASTRUCTURE -- CPU restatement of the prioritized replay of
 * dqn-marl_amd/csrc/prio.hip (include/evacx.h, evx_prio_*), the parity checker of the
 * GPU trees. The reference has no prioritized replay (it samples its deque uniformly,
 * Louvre_Evacuation/agents/dqn_agent.py:132), so this restates the
 * proportional variant of Schaul et al. (2016) sequentially: leaf writes in batch order,
 * then every internal node recomputed from its children (node n = 2n + 2n+1, root 1,
 * slot i at leaf C + i), stratified sampling by descent. Philox4x32-10 as published by
 * Salmon et al. (2011) (Random123), pinned by its known-answer vectors in
 * tests/test_prio_cpu.py. Only tests/ may call this. */
#include <math.h>
#include <stdint.h>

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
    for (int i = 0; i < 10; i++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static void rebuild_all(double *sum, double *mn, int64_t C) {
    for (int64_t n = C - 1; n >= 1; n--) {
        sum[n] = sum[2 * n] + sum[2 * n + 1];
        mn[n] = fmin(mn[2 * n], mn[2 * n + 1]);
    }
}

void orc_prio_init(double *sum, double *mn, int64_t C, double *max_leaf) {
    for (int64_t i = 0; i < 2 * C; i++) {
        sum[i] = 0.0;
        mn[i] = INFINITY;
    }
    *max_leaf = 1.0;
}

void orc_prio_set_range(double *sum, double *mn, int64_t C, const double *max_leaf, int64_t pos, int64_t n_new,
                        int64_t n_hide) {
    for (int64_t k = 0; k < n_new + n_hide; k++) {
        const int64_t j = (pos + k) & (C - 1);
        sum[C + j] = k < n_new ? *max_leaf : 0.0;
        mn[C + j] = k < n_new ? *max_leaf : INFINITY;
    }
    rebuild_all(sum, mn, C);
}

void orc_prio_update(double *sum, double *mn, int64_t C, double *max_leaf, const int64_t *idx, const float *td_abs,
                     int B, double eps, double alpha) {
    for (int k = 0; k < B; k++) {
        const double p = pow((double)td_abs[k] + eps, alpha);
        sum[C + idx[k]] = p;
        mn[C + idx[k]] = p;
        if (p > *max_leaf) *max_leaf = p;
    }
    rebuild_all(sum, mn, C);
}

void orc_prio_sample(const double *sum, const double *mn, int64_t C, int B, double beta, uint64_t seed,
                     uint64_t offset, int64_t *idx_out, float *w_out) {
    const double total = sum[1];
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int k = 0; k < B; k++) {
        const uint64_t c = (uint64_t)k + offset;
        const uint32_t ctr[4] = {(uint32_t)c, (uint32_t)(c >> 32), 0x9e12a5u, 0u};
        uint32_t q[4];
        orc_philox4x32_10(ctr, key, q);
        const double U = ((double)(q[0] >> 5) * 67108864.0 + (double)(q[1] >> 6)) * (1.0 / 9007199254740992.0);
        double u = ((double)k + U) * (total / (double)B);
        int64_t node = 1;
        while (node < C) {
            const double l = sum[2 * node], r = sum[2 * node + 1];
            if (u < l || r <= 0.0) {
                node = 2 * node;
            } else {
                u -= l;
                node = 2 * node + 1;
            }
        }
        idx_out[k] = node - C;
        w_out[k] = total > 0.0 ? (float)pow(sum[node] / mn[1], -beta) : 0.f;
    }
}
