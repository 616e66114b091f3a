// Device helpers shared by the evacuation kernels (gfx950, wave64).
//
// MT19937 "ring": the reference consumes two Mersenne-Twister streams per env
// (CPython `random`, legacy `numpy.random`). MT19937's raw state sequence obeys
//     x[n] = x[n-227] ^ twist(x[n-624], x[n-623]),   n >= 624
// so a workgroup keeps a window of that sequence in LDS and extends it 227 words
// per barrier phase (all 227 are independent). Output j of the stream is
// temper(x[pos + j]); consumers read words at prefix-sum offsets in parallel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace evx {

constexpr int NT = 256;          // threads per env workgroup (4 waves)
constexpr int NWAVE = NT / 64;
constexpr int MT_N = 624;
constexpr int MT_LAG = 227;      // 624 - 397

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// Extend the raw sequence in `ring` (RING words, power of two) until front >= upto.
// Cooperative: every thread of the block calls with the same (front, upto).
// Generates exactly what is needed (no over-generation) so that a window of
// RING words stays readable behind the new front.
__device__ __forceinline__ void mt_ensure(uint32_t* ring, int mask, int& front, int upto) {
    while (front < upto) {
        const int cnt = min(MT_LAG, upto - front);
        const int t = threadIdx.x;
        if (t < cnt) {
            const int n = front + t;
            const uint32_t a = ring[(n - 624) & mask], b = ring[(n - 623) & mask];
            const uint32_t c = ring[(n - MT_LAG) & mask];
            const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
            ring[n & mask] = c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        __syncthreads();
        front += cnt;
    }
}

__device__ __forceinline__ uint32_t mt_word(const uint32_t* ring, int mask, int idx) {
    return mt_temper(ring[idx & mask]);
}

// random.random() / numpy random_sample(): 53-bit double from two words.
__device__ __forceinline__ double mt_double(const uint32_t* ring, int mask, int idx) {
    const uint32_t a = mt_word(ring, mask, idx) >> 5, b = mt_word(ring, mask, idx + 1) >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
}

__device__ __forceinline__ int bit_length(uint32_t n) { return n ? 32 - __clz(n) : 0; }

// Wave-level inclusive scan of an int (wave64, shfl_up).
__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Exclusive scan, in PERSON order, of one value per person of "row" k
// (persons k*NT .. k*NT+NT-1, owned one per thread). `wsum` is an LDS scratch of
// NWAVE ints. Returns this thread's exclusive offset within the row; `row_total`
// receives the row sum (uniform). Contains two barriers.
__device__ __forceinline__ int block_exscan(int v, int* wsum, int& row_total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int incl = wave_incl_scan(v);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NWAVE; i++) {
        const int s = wsum[i];
        before += (i < w) ? s : 0;
        tot += s;
    }
    __syncthreads();
    row_total = tot;
    return before + incl - v;
}

__device__ __forceinline__ int block_sum(int v, int* wsum) {
    const int s = wave_sum(v);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
    __syncthreads();
    int tot = 0;
#pragma unroll
    for (int i = 0; i < NWAVE; i++) tot += wsum[i];
    __syncthreads();
    return tot;
}

__device__ __forceinline__ double block_sum_d(double v, double* wsum) {
    const double s = wave_sum_d(v);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
    __syncthreads();
    double tot = 0;
#pragma unroll
    for (int i = 0; i < NWAVE; i++) tot += wsum[i];
    __syncthreads();
    return tot;
}

// 16-bit table entries packed two per 32-bit LDS word; atomic min via CAS.
__device__ __forceinline__ void lds_min16(uint32_t* tab, int idx, uint32_t v) {
    uint32_t* w = tab + (idx >> 1);
    const int sh = (idx & 1) * 16;
    uint32_t old = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (true) {
        const uint32_t cur = (old >> sh) & 0xffffu;
        if (cur <= v) return;
        const uint32_t nv = (old & ~(0xffffu << sh)) | (v << sh);
        const uint32_t prev = atomicCAS(w, old, nv);
        if (prev == old) return;
        old = prev;
    }
}

__device__ __forceinline__ uint32_t lds_read16(const uint32_t* tab, int idx) {
    return (tab[idx >> 1] >> ((idx & 1) * 16)) & 0xffffu;
}

__device__ __forceinline__ void lds_set16_ffff(uint32_t* tab, int idx) {
    atomicOr(tab + (idx >> 1), 0xffffu << ((idx & 1) * 16));
}

// numpy DOUBLE_pairwise_sum (PW_BLOCKSIZE 128), single lane, iterative.
__device__ inline double np_pairwise_leaf(const double* a, int n) {
    if (n < 8) {
        double res = 0.;
        for (int i = 0; i < n; i++) res += a[i];
        return res;
    }
    double r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
    int i;
    for (i = 8; i < n - (n % 8); i += 8) {
        r0 += a[i]; r1 += a[i + 1]; r2 += a[i + 2]; r3 += a[i + 3];
        r4 += a[i + 4]; r5 += a[i + 5]; r6 += a[i + 6]; r7 += a[i + 7];
    }
    double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; i++) res += a[i];
    return res;
}

__device__ inline double np_pairwise_sum(const double* a, int n) {
    // explicit post-order traversal of numpy's split tree
    int off[24], len[24];
    double left[24];
    char stage[24];
    int sp = 0;
    off[0] = 0; len[0] = n; stage[0] = 0;
    double ret = 0.0;
    while (true) {
        if (len[sp] <= 128) {
            ret = np_pairwise_leaf(a + off[sp], len[sp]);
            while (true) {
                if (sp == 0) return ret;
                sp--;
                if (stage[sp] == 1) {
                    left[sp] = ret;
                    stage[sp] = 2;
                    int n2 = len[sp] / 2;
                    n2 -= n2 % 8;
                    off[sp + 1] = off[sp] + n2;
                    len[sp + 1] = len[sp] - n2;
                    stage[sp + 1] = 0;
                    sp++;
                    break;
                }
                ret = left[sp] + ret;
            }
        } else {
            stage[sp] = 1;
            int n2 = len[sp] / 2;
            n2 -= n2 % 8;
            off[sp + 1] = off[sp];
            len[sp + 1] = n2;
            stage[sp + 1] = 0;
            sp++;
        }
    }
}

}  // namespace evx
