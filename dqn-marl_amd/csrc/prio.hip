// MI355X (gfx950) prioritized replay: sum / min segment trees over the replay ring.
//
// SURVEY §8f F2 (cfg5: 65536 envs x 32 agents, GPU-resident prioritized replay). The
// reference samples its deque uniformly (random.sample, agents/dqn_agent.py:132);
// this is the proportional variant of Schaul et al. (2016) with stratified sampling,
// restated on the CPU by oracle/prio_oracle.c (the parity checker).
//
// Layout: heap order, node n = child 2n (op) child 2n+1, root 1, slot i at leaf
// C + i, f64. Rebuilds never walk leaf-to-root per update (a 20-deep chain of
// dependent L2 round trips): a pass reduces aligned blocks of up to 1024 nodes of
// one level through 10 levels in LDS (one workgroup per block, both trees at once)
// and writes every node of the block's subtree, so the next pass sees 1024x fewer
// nodes. C = 2^20 is two passes; a range update (a push) touches only the blocks it
// covers. Every internal node is recomputed as left + right from final children, so
// the trees are a pure function of the leaves (deterministic, as the oracle's).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "evacx.h"

namespace evxp {

constexpr int BLK = 1024;  // nodes reduced per workgroup and pass (10 levels)
constexpr int NT = 256;

struct u4 {
    uint32_t x, y, z, w;
};
// Philox4x32-10 (Salmon et al. 2011), the generator of every other learner draw
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

__global__ __launch_bounds__(NT) void prio_init_kernel(evx_prio t) {
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i < 2 * t.capacity) {
        t.sum[i] = 0.0;
        t.mn[i] = INFINITY;
    }
    if (i < t.capacity) t.owner[i] = -1;
    if (i == 0) t.max_leaf[0] = 1.0;
}

// One pass over the level whose nodes are [base, 2 base): workgroup j reduces block
// (b0 + j) mod (base / bl) of bl nodes through log2(bl) levels. Leaf passes (base ==
// C) first apply a range update: slots whose offset from pos is < n_new take
// max_leaf, those below n_new + n_hide take 0 / +inf.
__global__ __launch_bounds__(NT) void tree_pass_kernel(evx_prio t, int64_t base, int bl, int64_t b0, int leaf_mode,
                                                       int64_t pos, int64_t n_new, int64_t n_hide) {
    __shared__ double ss[2][BLK], sm[2][BLK];
    const int64_t nb = base / bl;
    const int64_t b = (b0 + blockIdx.x) % nb;
    const int64_t first = base + b * bl;
    const double newp = leaf_mode ? t.max_leaf[0] : 0.0;
    for (int i = threadIdx.x; i < bl; i += NT) {
        double s = t.sum[first + i], m = t.mn[first + i];
        if (leaf_mode) {
            const int64_t slot = b * bl + i;
            const int64_t off = (slot - pos) & (t.capacity - 1);
            if (off < n_new) {
                s = newp;
                m = newp;
                t.sum[first + i] = s;
                t.mn[first + i] = m;
            } else if (off < n_new + n_hide) {
                s = 0.0;
                m = INFINITY;
                t.sum[first + i] = s;
                t.mn[first + i] = m;
            }
        }
        ss[0][i] = s;
        sm[0][i] = m;
    }
    __syncthreads();
    int cur = 0;
    int64_t lev = base;   // nodes of the current level start at lev
    int64_t off = b * bl; // this block's first node within its level
    for (int n = bl >> 1; n >= 1; n >>= 1) {
        lev >>= 1;
        off >>= 1;
        for (int i = threadIdx.x; i < n; i += NT) {
            const double s = ss[cur][2 * i] + ss[cur][2 * i + 1];
            const double m = fmin(sm[cur][2 * i], sm[cur][2 * i + 1]);
            ss[cur ^ 1][i] = s;
            sm[cur ^ 1][i] = m;
            t.sum[lev + off + i] = s;
            t.mn[lev + off + i] = m;
        }
        cur ^= 1;
        __syncthreads();
    }
}

// evx_prio_update: the last k of a slot owns it (a sequential loop's last write wins)
__global__ __launch_bounds__(NT) void prio_owner_kernel(evx_prio t, const int64_t* __restrict__ idx, int B) {
    const int k = blockIdx.x * NT + threadIdx.x;
    if (k < B) atomicMax(&t.owner[idx[k]], k);
}
__global__ __launch_bounds__(NT) void prio_leaf_kernel(evx_prio t, const int64_t* __restrict__ idx,
                                                       const float* __restrict__ td_abs, int B, double eps,
                                                       double alpha) {
    const int k = blockIdx.x * NT + threadIdx.x;
    if (k >= B) return;
    const int64_t j = idx[k];
    const double p = pow((double)td_abs[k] + eps, alpha);
    // every priority counts for the max (a sequential loop sees them all); non-negative
    // doubles order like their bit patterns
    atomicMax(reinterpret_cast<unsigned long long*>(t.max_leaf), (unsigned long long)__double_as_longlong(p));
    if (t.owner[j] != k) return;  // not the owner (or the owner already cleared it)
    t.sum[t.capacity + j] = p;
    t.mn[t.capacity + j] = p;
    t.owner[j] = -1;
}

__global__ __launch_bounds__(NT) void prio_sample_kernel(evx_replay rp, evx_prio t, int B, double beta, uint64_t seed,
                                                         uint64_t offset, evx_obs* __restrict__ s,
                                                         evx_obs* __restrict__ s2, int32_t* __restrict__ a,
                                                         float* __restrict__ r, uint8_t* __restrict__ done,
                                                         int64_t* __restrict__ idx_out, float* __restrict__ w_out) {
    const int k = blockIdx.x * NT + threadIdx.x;
    if (k >= B) return;
    const uint64_t c = (uint64_t)k + offset;
    const u4 q = philox((uint32_t)c, (uint32_t)(c >> 32), 0x9e12a5u, 0u, (uint32_t)seed, (uint32_t)(seed >> 32));
    const double U = ((double)(q.x >> 5) * 67108864.0 + (double)(q.y >> 6)) * (1.0 / 9007199254740992.0);
    const double total = t.sum[1];
    double u = ((double)k + U) * (total / (double)B);
    int64_t node = 1;
    const int64_t C = t.capacity;
    // two levels per round of loads: the children and the four grandchildren of node are read
    // together (independent loads), then the same two decisions as one level at a time (the same
    // comparisons and subtractions: the same leaf) -- half the dependent L2 round trips
    while (2 * node < C) {
        const double l = t.sum[2 * node], rr = t.sum[2 * node + 1];
        const double g0 = t.sum[4 * node], g1 = t.sum[4 * node + 1], g2 = t.sum[4 * node + 2], g3 = t.sum[4 * node + 3];
        double gl, gr;
        if (u < l || rr <= 0.0) {
            node = 2 * node;
            gl = g0;
            gr = g1;
        } else {
            u -= l;
            node = 2 * node + 1;
            gl = g2;
            gr = g3;
        }
        if (u < gl || gr <= 0.0) {
            node = 2 * node;
        } else {
            u -= gl;
            node = 2 * node + 1;
        }
    }
    if (node < C) {  // an odd number of levels: the last one alone
        const double l = t.sum[2 * node], rr = t.sum[2 * node + 1];
        if (u < l || rr <= 0.0) {
            node = 2 * node;
        } else {
            u -= l;
            node = 2 * node + 1;
        }
    }
    const int64_t j = node - C;
    const double p = t.sum[node];
    s[k] = rp.s[j];
    s2[k] = rp.s2[j];
    a[k] = rp.a[j];
    r[k] = rp.r[j];
    done[k] = rp.done[j];
    if (idx_out) idx_out[k] = j;
    if (w_out) w_out[k] = total > 0.0 ? (float)pow(p / t.mn[1], -beta) : 0.f;
}

}  // namespace evxp

namespace {
thread_local char g_perr[256] = "";
int pfail(int code, const char* msg) {
    snprintf(g_perr, sizeof(g_perr), "%s", msg);
    return code;
}
int plaunch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) return 0;
    snprintf(g_perr, sizeof(g_perr), "%s: %s", what, hipGetErrorString(e));
    return -5;
}
int check_tree(const evx_prio* t) {
    if (!t || !t->sum || !t->mn || !t->max_leaf || !t->owner) return pfail(-22, "prio: NULL tree");
    const int64_t C = t->capacity;
    if (C < 1024 || C > ((int64_t)1 << 26) || (C & (C - 1))) return pfail(-22, "prio: capacity must be 2^10..2^26");
    return 0;
}
// rebuild both trees over the leaf range [pos, pos + n) mod C (n >= C: everything),
// applying the range update of evx_prio_set_range in the leaf pass
int rebuild(const evx_prio* t, int64_t pos, int64_t n, int leaf_mode, int64_t n_new, int64_t n_hide,
            hipStream_t st) {
    int64_t base = t->capacity;
    int64_t lo = pos, cnt = n < t->capacity ? n : t->capacity;
    bool leaf = true;
    while (true) {
        const int bl = base < evxp::BLK ? (int)base : evxp::BLK;
        const int64_t nb = base / bl;
        const int64_t first = lo / bl, last = (lo + cnt - 1) / bl;
        int64_t nblk = last - first + 1;
        if (nblk > nb) nblk = nb;
        hipLaunchKernelGGL(evxp::tree_pass_kernel, dim3((unsigned)nblk), dim3(evxp::NT), 0, st, *t, base, bl,
                           first % nb, leaf && leaf_mode, pos, n_new, n_hide);
        int rc = plaunch("prio tree pass");
        if (rc) return rc;
        if (nb == 1) return 0;
        base = nb;
        lo = first % nb;
        cnt = nblk;
        leaf = false;
    }
}
}  // namespace

extern "C" {

const char* evx_prio_last_error(void) { return g_perr; }

int evx_prio_init(const evx_prio* t, void* stream) {
    if (int rc = check_tree(t)) return rc;
    hipLaunchKernelGGL(evxp::prio_init_kernel, dim3((unsigned)((2 * t->capacity + evxp::NT - 1) / evxp::NT)),
                       dim3(evxp::NT), 0, (hipStream_t)stream, *t);
    return plaunch("prio_init");
}

int evx_prio_set_range(const evx_prio* t, int64_t pos, int64_t n_new, int64_t n_hide, void* stream) {
    if (int rc = check_tree(t)) return rc;
    if (n_new < 0 || n_hide < 0 || n_new + n_hide > t->capacity) return pfail(-22, "prio_set_range: bad counts");
    if (n_new + n_hide == 0) return 0;
    pos &= t->capacity - 1;
    return rebuild(t, pos, n_new + n_hide, 1, n_new, n_hide, (hipStream_t)stream);
}

int evx_prio_update(const evx_prio* t, const int64_t* idx, const float* td_abs, int32_t B, double eps, double alpha,
                    void* stream) {
    if (int rc = check_tree(t)) return rc;
    if (B <= 0) return 0;
    if (!idx || !td_abs) return pfail(-22, "prio_update: NULL argument");
    const hipStream_t st = (hipStream_t)stream;
    const unsigned g = (unsigned)((B + evxp::NT - 1) / evxp::NT);
    hipLaunchKernelGGL(evxp::prio_owner_kernel, dim3(g), dim3(evxp::NT), 0, st, *t, idx, B);
    hipLaunchKernelGGL(evxp::prio_leaf_kernel, dim3(g), dim3(evxp::NT), 0, st, *t, idx, td_abs, B, eps, alpha);
    if (int rc = plaunch("prio_update")) return rc;
    return rebuild(t, 0, t->capacity, 0, 0, 0, st);
}

int evx_prio_sample(const evx_replay* rp, const evx_prio* t, int32_t B, double beta, uint64_t seed, uint64_t offset,
                    evx_obs* s, evx_obs* s2, int32_t* a, float* r, uint8_t* done, int64_t* idx_out, float* w_out,
                    void* stream) {
    if (int rc = check_tree(t)) return rc;
    if (!rp || rp->capacity != t->capacity) return pfail(-22, "prio_sample: ring and tree capacities differ");
    if (B <= 0) return 0;
    if (!s || !s2 || !a || !r || !done) return pfail(-22, "prio_sample: NULL output");
    hipLaunchKernelGGL(evxp::prio_sample_kernel, dim3((unsigned)((B + evxp::NT - 1) / evxp::NT)), dim3(evxp::NT), 0,
                       (hipStream_t)stream, *rp, *t, B, beta, seed, offset, s, s2, a, r, done, idx_out, w_out);
    return plaunch("prio_sample");
}

}  // extern "C"
