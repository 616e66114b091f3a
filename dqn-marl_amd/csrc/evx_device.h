// Device helpers shared by the evacuation kernels (gfx950, wave64).
//
// MT19937 "ring": the reference consumes two Mersenne-Twister streams per env
// (CPython `random`, legacy `numpy.random`). MT19937's raw state sequence obeys
//     x[n] = x[n-227] ^ twist(x[n-624], x[n-623]),   n >= 624
// so a wave keeps a window of that sequence in an LDS ring and extends it by up
// to 227 words per round (each depends only on words older than the round).
// Output j of the stream is temper(x[pos + j]); consumers read words at
// prefix-sum offsets in parallel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace evx {

constexpr int MT_N = 624;
constexpr int MT_LAG = 227;      // 624 - 397

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t mt_twist1(uint32_t lag, uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return lag ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
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

// Leaves of numpy's pairwise split tree (DOUBLE_pairwise_sum: blocks <= 128
// elements, split at n/2 rounded down to a multiple of 8), left to right.
// Single lane; `stk` is 64 ints of LDS (no private-memory stack). Returns the
// number of leaves (<= cap written to off/len).
__device__ inline int np_pairwise_leaves(int n, int* off, int* len, int cap, int* stk) {
    int* so = stk;
    int* sl = stk + 32;
    int sp = 1, nl = 0;
    so[0] = 0;
    sl[0] = n;
    while (sp > 0) {
        sp--;
        const int o = so[sp], l = sl[sp];
        if (l <= 128) {
            if (nl < cap) {
                off[nl] = o;
                len[nl] = l;
            }
            nl++;
        } else {
            int n2 = l / 2;
            n2 -= n2 % 8;
            so[sp] = o + n2; sl[sp] = l - n2; sp++;  // right pushed first -> left popped first
            so[sp] = o; sl[sp] = n2; sp++;
        }
    }
    return nl;
}

// Combine leaf sums in numpy's tree order (single lane). `stk`: 64 ints and
// `left`: 32 doubles of LDS.
__device__ inline double np_pairwise_combine(int n, const double* leafsum, int* stk, double* left) {
    int* ol = stk;
    int* st = stk + 32;
    int sp = 0, li = 0;
    ol[0] = n;
    st[0] = 0;
    double ret = 0.0;
    while (true) {
        if (ol[sp] <= 128) {
            ret = leafsum[li++];
            while (true) {
                if (sp == 0) return ret;
                sp--;
                if (st[sp] == 1) {
                    left[sp] = ret;
                    st[sp] = 2;
                    int n2 = ol[sp] / 2;
                    n2 -= n2 % 8;
                    ol[sp + 1] = ol[sp] - n2;
                    st[sp + 1] = 0;
                    sp++;
                    break;
                }
                ret = left[sp] + ret;
            }
        } else {
            st[sp] = 1;
            int n2 = ol[sp] / 2;
            n2 -= n2 % 8;
            ol[sp + 1] = n2;
            st[sp + 1] = 0;
            sp++;
        }
    }
}

}  // namespace evx
