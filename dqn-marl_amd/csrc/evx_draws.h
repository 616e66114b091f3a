// Counter-based draws shared by the learner's kernels (csrc/qnet.hip) and the fused replay push
// (csrc/env_step.hip): Philox4x32-10 (Salmon et al. 2011) and the keyed Feistel permutation the
// replay samples without replacement with (DQNAgent.learn's random.sample, agents/dqn_agent.py:132;
// restated on the CPU by oracle/draw_oracle.c).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace evxd {

struct u4 {
    uint32_t x, y, z, w;
};
__device__ __forceinline__ u4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0, h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
        c0 = h1 ^ c1 ^ k0;
        c1 = l1;
        c2 = h0 ^ c3 ^ k1;
        c3 = l0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return {c0, c1, c2, c3};
}
struct perm_key {
    uint32_t k[6];
    int half;       // bits per Feistel half
    uint64_t hmask; // (1 << half) - 1
};
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}
__device__ __forceinline__ perm_key make_perm_key(uint64_t n, uint64_t seed, uint64_t offset, uint32_t stream) {
    perm_key pk;
    const u4 q = philox((uint32_t)offset, (uint32_t)(offset >> 32), 0x5a3b1eu, stream, (uint32_t)seed,
                        (uint32_t)(seed >> 32));
    const uint32_t qq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int r = 0; r < 6; r++) pk.k[r] = fmix32(qq[r & 3] + (uint32_t)r * 0x9e3779b9u);
    int w = 2;
    while (w < 62 && (1ull << w) < n) w += 2;
    pk.half = w / 2;
    pk.hmask = (1ull << pk.half) - 1;
    return pk;
}
__device__ __forceinline__ uint64_t perm_apply(const perm_key& pk, uint64_t x, uint64_t n) {
    do {
        uint64_t L = x >> pk.half, R = x & pk.hmask;
#pragma unroll
        for (int r = 0; r < 6; r++) {
            const uint64_t F = (uint64_t)fmix32((uint32_t)R ^ pk.k[r]) & pk.hmask;  // R < 2^31
            const uint64_t t = R;
            R = L ^ F;
            L = t;
        }
        x = (L << pk.half) | R;
    } while (x >= n);
    return x;
}


}  // namespace evxd
