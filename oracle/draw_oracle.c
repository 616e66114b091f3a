/* TEST INFRASTRUCTURE (CPU oracle, never the product path): sequential restatements of the
 * build's counter-based draws, so the GPU's vectorised versions can be compared index for
 * index. The reference draws from CPython's MT19937 instead (agents/dqn_agent.py:106 act's
 * np.random.random() <= epsilon then random.randrange(5); :132 learn's random.sample); a
 * device-resident learner cannot consume one sequential stream per draw, so the build uses
 * Philox4x32-10 keyed by (seed, counter) -- these functions pin exactly which draws it makes.
 *   orc_epsilon_greedy : evx_act / the fused act's epsilon-greedy (csrc/qnet.hip act_kernel,
 *                        csrc/qmlp.hip fc3_act)
 *   orc_replay_indices : evx_replay_sample / _window (csrc/qnet.hip replay_sample_kernel)
 *   orc_dropout_keep   : the fused MLP kernels' dropout hash (csrc/qmlp.hip drop_row/drop_pair)
 */
#include <stdint.h>

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

static float u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }

/* argmax (first maximum, np.argmax) of row i, then with probability epsilon a uniform action:
 * Philox(ctr = (i + offset) lo, hi, 0xac7, 0; key = seed lo, hi); u01(x) <= epsilon -> (y * A) >> 32 */
void orc_epsilon_greedy(const float *Q, int n, int A, float epsilon, uint64_t seed, uint64_t offset, int32_t *out) {
    for (int i = 0; i < n; i++) {
        int best = 0;
        float bv = Q[(int64_t)i * A];
        for (int j = 1; j < A; j++)
            if (Q[(int64_t)i * A + j] > bv) {
                bv = Q[(int64_t)i * A + j];
                best = j;
            }
        if (epsilon > 0.f) {
            const uint64_t c = (uint64_t)i + offset;
            const uint32_t ctr[4] = {(uint32_t)c, (uint32_t)(c >> 32), 0xac7u, 0u};
            const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
            uint32_t r[4];
            orc_philox4x32_10(ctr, key, r);
            if (u01(r[0]) <= epsilon) best = (int)(((uint64_t)r[1] * (uint64_t)A) >> 32);
        }
        out[i] = best;
    }
}

static uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

/* sample i WITHOUT replacement (DQNAgent.learn's random.sample, agents/dqn_agent.py:132): ring slot
 * base + perm(i) (wrapped at capacity) for a keyed permutation perm of [0, size): a 6-round balanced
 * Feistel network on the smallest even width 2^w >= size, cycle-walked into [0, size). Round keys
 * k[r] = fmix32(q[r & 3] + r * 0x9e3779b9) from q = Philox(ctr = offset lo, hi, 0x5a3b1e, stream;
 * key = seed); round: (L, R) -> (R, L ^ (fmix32(R ^ k[r]) & mask)). stream: the agent of a
 * per-agent memory (evx_replay_sample_agents), else 0. */
void orc_replay_indices(int64_t base, int64_t size, int64_t capacity, int B, uint64_t seed, uint64_t offset,
                        uint32_t stream, int64_t *idx) {
    const uint32_t ctr[4] = {(uint32_t)offset, (uint32_t)(offset >> 32), 0x5a3b1eu, stream};
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t q[4], k[6];
    orc_philox4x32_10(ctr, key, q);
    for (int r = 0; r < 6; r++) k[r] = fmix32(q[r & 3] + (uint32_t)r * 0x9e3779b9u);
    int w = 2;
    while (w < 62 && (1ull << w) < (uint64_t)size) w += 2;
    const int half = w / 2;
    const uint64_t hmask = (1ull << half) - 1;
    for (int i = 0; i < B; i++) {
        uint64_t x = (uint64_t)i;
        do {
            uint64_t L = x >> half, R = x & hmask;
            for (int r = 0; r < 6; r++) {
                const uint64_t F = (uint64_t)fmix32((uint32_t)R ^ k[r]) & hmask;
                const uint64_t t = R;
                R = L ^ F;
                L = t;
            }
            x = (L << half) | R;
        } while (x >= (uint64_t)size);
        int64_t j = base + (int64_t)x;
        if (j >= capacity) j -= capacity;
        idx[i] = j;
    }
}

/* keep[r][c] of the fused MLP's dropout: one fmix32 hash per (row pair, column), low 16 bits
 * for the even row, high 16 for the odd; keep iff the 16-bit value >= floor(p * 65536) */
void orc_dropout_keep(uint32_t seed, uint32_t stream, float p, int rows, int cols, uint8_t *keep) {
    uint32_t thresh = p > 0.f ? (uint32_t)((double)p * 65536.0) : 0u;
    if (p > 0.f && thresh == 0u) thresh = 1u;
    const uint32_t s = fmix32(stream * 0x632be5abu + 0x9e3779b9u);
    for (int r = 0; r < rows; r++) {
        const uint32_t ph = fmix32(seed ^ s ^ ((uint32_t)(r >> 1) * 0x9e3779b1u));
        for (int c = 0; c < cols; c++) {
            const uint32_t h = fmix32(ph ^ ((uint32_t)c * 0x85ebca77u + 0x27d4eb2fu));
            const uint32_t v = (r & 1) ? (h >> 16) : (h & 0xffffu);
            keep[(int64_t)r * cols + c] = thresh ? (v >= thresh) : 1;
        }
    }
}
