// MI355X (gfx950) DQN learner kernels: the Q-network contractions on MFMA and the
// HBM-bound learner ops around them.
//
// Reference: Louvre_Evacuation/agents/dqn_agent.py
//   DQNNetwork (:15-61)        -> evx_gemm (Linear / im2col-conv layers), evx_im2col/col2im
//   DQNAgent.act (:101-124)    -> evx_act (argmax + epsilon-greedy)
//   DQNAgent.learn (:126-168)  -> evx_td_loss (gather, max, TD target, MSE, dQ),
//                                 evx_gemm backward, evx_colsum (bias grads),
//                                 evx_sumsq + evx_clip_adam (clip_grad_norm_ + Adam)
//   DQNAgent.memory (:88-99)   -> evx_replay_push / evx_replay_sample
// GEMMs take fp32 operands in HBM and compute either exact f32 (v_mfma_f32_32x32x2_f32:
// a k-ordered fmaf chain, used where parity with torch fp32 matters) or bf16 inputs
// with f32 accumulation (v_mfma_f32_32x32x16_bf16, the throughput path).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <type_traits>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "evacx.h"
#include "evx_host.h"
#include "evx_draws.h"

namespace evxq {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 64, BN = 64, BK = 32;

// Philox4x32-10, the replay permutation (evx_draws.h)
using evxd::u4;
using evxd::philox;
using evxd::perm_key;
using evxd::fmix32;
using evxd::make_perm_key;
using evxd::perm_apply;
__device__ __forceinline__ float u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }

// ------------------------------------------------------------------------ GEMM
template <typename T>
__device__ __forceinline__ T to_in(float v);
template <>
__device__ __forceinline__ float to_in<float>(float v) { return v; }
template <>
__device__ __forceinline__ __bf16 to_in<__bf16>(float v) { return (__bf16)v; }

template <typename TIn>
__global__ __launch_bounds__(256) void gemm_kernel(evx_gemm_desc g) {
    constexpr int PADK = sizeof(TIn) == 4 ? 1 : 8;
    __shared__ __attribute__((aligned(16))) TIn As[BM][BK + PADK];
    __shared__ __attribute__((aligned(16))) TIn Bs[BN][BK + PADK];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; r++) acc[r] = 0.f;
    const bool a_kc = g.sak == 1, b_nc = g.sbn == 1;
    for (int k0 = 0; k0 < g.K; k0 += BK) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int idx = tid + 256 * i;
            int mm, kk;
            if (a_kc) { mm = idx >> 5; kk = idx & 31; } else { kk = idx >> 6; mm = idx & 63; }
            const int gm = m0 + mm, gk = k0 + kk;
            const float v = (gm < g.M && gk < g.K) ? g.A[(int64_t)gm * g.sam + (int64_t)gk * g.sak] : 0.f;
            As[mm][kk] = to_in<TIn>(v);
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int idx = tid + 256 * i;
            int nn, kk;
            if (b_nc) { kk = idx >> 6; nn = idx & 63; } else { nn = idx >> 5; kk = idx & 31; }
            const int gn = n0 + nn, gk = k0 + kk;
            const float v = (gn < g.N && gk < g.K) ? g.B[(int64_t)gk * g.sbk + (int64_t)gn * g.sbn] : 0.f;
            Bs[nn][kk] = to_in<TIn>(v);
        }
        __syncthreads();
        const int ar = wm * 32 + (lane & 31), br = wn * 32 + (lane & 31), h = lane >> 5;
        if constexpr (sizeof(TIn) == 4) {
#pragma unroll
            for (int kk = 0; kk < BK / 2; kk++)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[ar][2 * kk + h], Bs[br][2 * kk + h], acc, 0, 0, 0);
        } else {
#pragma unroll
            for (int s = 0; s < BK / 16; s++) {
                const bf16x8 a = *reinterpret_cast<const bf16x8*>(&As[ar][16 * s + 8 * h]);
                const bf16x8 b = *reinterpret_cast<const bf16x8*>(&Bs[br][16 * s + 8 * h]);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
            }
        }
        __syncthreads();
    }
    // epilogue: C/D map of the 32x32 MFMA (col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5))
    const int gn = n0 + wn * 32 + (lane & 31);
    if (gn >= g.N) return;
    const float bias = g.bias ? g.bias[gn] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int gm = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (gm >= g.M) continue;
        float v = g.alpha * acc[r] + bias;
        if (g.flags & EVX_GEMM_RELU) v = v > 0.f ? v : 0.f;
        if (g.mask) v = g.mask[(int64_t)gm * g.ldm + gn] ? v * g.mask_scale : 0.f;
        if (g.gate) v = g.gate[(int64_t)gm * g.ldg + gn] > 0.f ? v : 0.f;
        float* cp = g.C + (int64_t)gm * g.ldc + gn;
        if (g.flags & EVX_GEMM_ACCUM) v += *cp;
        *cp = v;
    }
}

// ------------------------------------------------------------- GEMM, big tiles
// 128x128x32 block tile, 4 waves as 2x2, each wave 64x64 = 2x2 MFMA 32x32 tiles (64 f32
// accumulators per lane). The next K-tile is fetched into registers while the current
// one is multiplied (register double buffering, one barrier pair per K-step). gridDim.z
// splits K: each slice stores its raw partial into the workspace ws[z][M][N] (used for dW =
// dY^T X, whose M x N grid alone cannot fill 256 CUs, and long-K GEMMs with an epilogue);
// splitk_reduce_kernel adds the slices in slice order and applies the epilogue.
constexpr int TB = 128;
template <typename TIn>
__global__ __launch_bounds__(256) void gemm128_kernel(evx_gemm_desc g, int ksplit_len) {
    constexpr int PADK = sizeof(TIn) == 4 ? 1 : 8;
    __shared__ __attribute__((aligned(16))) TIn As[TB][BK + PADK];
    __shared__ __attribute__((aligned(16))) TIn Bs[TB][BK + PADK];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int m0 = blockIdx.y * TB, n0 = blockIdx.x * TB;
    const int kb = blockIdx.z * ksplit_len, ke = min(g.K, kb + ksplit_len);
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;
    const bool a_kc = g.sak == 1, b_nc = g.sbn == 1;
    float ra[16], rb[16];
    auto fetch = [&](int k0) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int idx = tid + 256 * i;
            int mm, kk;
            if (a_kc) { mm = idx >> 5; kk = idx & 31; } else { kk = idx >> 7; mm = idx & 127; }
            const int gm = m0 + mm, gk = k0 + kk;
            ra[i] = (gm < g.M && gk < ke) ? g.A[(int64_t)gm * g.sam + (int64_t)gk * g.sak] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int idx = tid + 256 * i;
            int nn, kk;
            if (b_nc) { kk = idx >> 7; nn = idx & 127; } else { nn = idx >> 5; kk = idx & 31; }
            const int gn = n0 + nn, gk = k0 + kk;
            rb[i] = (gn < g.N && gk < ke) ? g.B[(int64_t)gk * g.sbk + (int64_t)gn * g.sbn] : 0.f;
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int idx = tid + 256 * i;
            int mm, kk;
            if (a_kc) { mm = idx >> 5; kk = idx & 31; } else { kk = idx >> 7; mm = idx & 127; }
            As[mm][kk] = to_in<TIn>(ra[i]);
        }
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int idx = tid + 256 * i;
            int nn, kk;
            if (b_nc) { kk = idx >> 7; nn = idx & 127; } else { nn = idx >> 5; kk = idx & 31; }
            Bs[nn][kk] = to_in<TIn>(rb[i]);
        }
    };
    if (kb < ke) fetch(kb);
    for (int k0 = kb; k0 < ke; k0 += BK) {
        stash();
        __syncthreads();
        if (k0 + BK < ke) fetch(k0 + BK);  // in flight during the MFMAs below
        const int h = lane >> 5;
#pragma unroll
        for (int mi = 0; mi < 2; mi++) {
            const int ar = wm * 64 + mi * 32 + (lane & 31);
#pragma unroll
            for (int ni = 0; ni < 2; ni++) {
                const int br = wn * 64 + ni * 32 + (lane & 31);
                if constexpr (sizeof(TIn) == 4) {
#pragma unroll
                    for (int kk = 0; kk < BK / 2; kk++)
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(As[ar][2 * kk + h], Bs[br][2 * kk + h],
                                                                          acc[mi][ni], 0, 0, 0);
                } else {
#pragma unroll
                    for (int s = 0; s < BK / 16; s++) {
                        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&As[ar][16 * s + 8 * h]);
                        const bf16x8 b = *reinterpret_cast<const bf16x8*>(&Bs[br][16 * s + 8 * h]);
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[mi][ni], 0, 0, 0);
                    }
                }
            }
        }
        __syncthreads();
    }
    const bool split = gridDim.z > 1;
#pragma unroll
    for (int ni = 0; ni < 2; ni++) {
        const int gn = n0 + wn * 64 + ni * 32 + (lane & 31);
        if (gn >= g.N) continue;
        const float bias = g.bias ? g.bias[gn] : 0.f;
#pragma unroll
        for (int mi = 0; mi < 2; mi++) {
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int gm = m0 + wm * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (gm >= g.M) continue;
                float* cp = g.C + (int64_t)gm * g.ldc + gn;
                if (split) {  // this K slice's partial, summed in slice order by splitk_reduce_kernel
                    g.ws[((int64_t)blockIdx.z * g.M + gm) * g.N + gn] = g.alpha * acc[mi][ni][r];
                    continue;
                }
                float v = g.alpha * acc[mi][ni][r] + bias;
                if (g.flags & EVX_GEMM_RELU) v = v > 0.f ? v : 0.f;
                if (g.mask) v = g.mask[(int64_t)gm * g.ldm + gn] ? v * g.mask_scale : 0.f;
                if (g.gate) v = g.gate[(int64_t)gm * g.ldg + gn] > 0.f ? v : 0.f;
                if (g.flags & EVX_GEMM_ACCUM) v += *cp;
                *cp = v;
            }
        }
    }
}

// gemm128 in the f32-accurate x3 mode (EVX_PREC_X3, as the fused MLP's): every f32 operand is
// staged in LDS as bf16 hi = bf16(v) and lo = bf16(v - hi), a product as hi*hi + hi*lo + lo*hi
// on v_mfma_f32_32x32x16_bf16 (relative error ~2^-17 per product, f32 accumulation): 3 bf16
// MFMAs per 16-deep step instead of 8 f32 32x32x2 ones, and 16-B LDS reads instead of 4-B.
//
// CM selects an implicit-GEMM 3x3 convolution (padding 1, 11x11 maps, pixel-major [B*121][C]
// activations, agents/dqn_agent.py:22-24,48-50) in place of im2col + GEMM: the operand is
// gathered from the activations during the tile fetch (cs = the gathered tensor's channels).
//   CV_FWD: Y = X (*) W. A(m, k) = X[pixel m shifted by tap][c], k = tap*cs + c (one tap
//           per K-tile when cs >= 32: contiguous channel runs); B(k, n) = W[c*sbk + n*sbn + tap].
//   CV_DX:  dX = dY (*) flip(W): A(m, k) = dY[pixel m shifted by -tap][o], k = tap*cs + o;
//           B the same gather of W (c*sbk -> o*9N, n*sbn -> n*9); the ReLU-backward gate
//           of the layer below rides the epilogue (no col2im / relu_grad pass).
//   CV_DW:  dW[o][c*9+tap] = sum_m dY[m][o] X[pixel m shifted by tap][c]: B(k = m, n) gathered.
enum { CV_NONE = 0, CV_FWD = 1, CV_DX = 2, CV_DW = 3 };
__device__ __forceinline__ uint32_t div121(uint32_t m) { return __umulhi(m, 35495598u); }  // m < 2^26
__device__ __forceinline__ int div11(int p) { return (p * 187) >> 11; }                     // p < 121
// SPL (CV_NONE, EVX_GEMM_SPLIT_AB): A and B already hold bf16 hi / lo planes, k-contiguous; a
// K tile is staged as 16-B pieces (2 per thread and plane) with no per-element split
// VEC (CV_NONE f32 operands, host-checked strides / alignment): a k-contiguous operand staged from
// 16-B global loads of 4 consecutive k (8-B hi / lo LDS stores) instead of 4-B loads of one --
// bit 0: A (sak 1), bit 2: B (sbk 1). (m / n-contiguous operands vectorised along m / n measured
// slower -- 4-way LDS bank conflicts on the 2-byte stores: fc1's dW 132 -> 263 us -- and keep the
// one-element path.)
enum { VA_K = 1, VB_K = 4 };
template <int CM, bool SPL = false, int VEC = 0>
__global__ __launch_bounds__(256) void gemm128x3_kernel(evx_gemm_desc g, int ksplit_len, int cs) {
    constexpr int PK = BK + 8;  // row pitch (bf16): 20 words, conflict-free 16-B reads
    __shared__ __attribute__((aligned(16))) __bf16 As[2][TB][PK];
    __shared__ __attribute__((aligned(16))) __bf16 Bs[2][TB][PK];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int m0 = blockIdx.y * TB, n0 = blockIdx.x * TB;
    const int kb = blockIdx.z * ksplit_len, ke = min(g.K, kb + ksplit_len);
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;
    const bool a_kc = CM == CV_FWD || CM == CV_DX || g.sak == 1;
    const bool b_nc = CM == CV_DW || (CM == CV_NONE && g.sbn == 1);
    float ra[16], rb[16];
    // Staging: a k-contiguous operand (A with a_kc, B with !b_nc -- every conv forward / dX operand
    // and the fc layers') is held as k pairs: thread t takes rows (t >> 4) + 16 i (i < 8) at
    // k = 2 (t & 15) + {0, 1} and stages each pair's hi and lo as one 4-byte LDS store (was 64
    // 2-byte stores per thread per K-tile, lane pairs sharing a word). The transposed layouts keep
    // one k per thread (rows t & 127, k = (t >> 7) + 2 i).
    // CV_FWD / CV_DX: this thread's A rows are m0 + (t >> 4) + 16 i; their pixel index p0 (i = 0)
    // steps by 16 (mod 121). CV_DW: this thread's column n = n0 + (tid & 127) is fixed.
    const int pa0 = (int)((uint32_t)(m0 + (tid >> 4)) - div121((uint32_t)(m0 + (tid >> 4))) * 121u);
    int dw_c = 0, dw_dy = 0, dw_dx = 0;
    if constexpr (CM == CV_DW) {
        const int n = n0 + (tid & 127);
        dw_c = n / 9;
        const int tap = n - dw_c * 9;
        dw_dy = tap / 3 - 1;
        dw_dx = tap - (tap / 3) * 3 - 1;
    }
    const int kp = 2 * (tid & 15), rp = tid >> 4;  // pair layout: k offset, first row
    bf16x8 sa[2][2], sb[2][2];                     // SPL: [plane][piece], piece i: row (tid + 256 i) >> 2
    float4 va4[4], vb4[4];  // VEC pieces: k-vector (row (t >> 3) + 32 i, k 4 (t & 7)) or m / n-vector
                            // (k (t >> 5) + 8 i, rows 4 (t & 31) .. + 3)
    auto fetch = [&](int k0) {
        if constexpr ((VEC & VA_K) != 0) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int gm = m0 + (tid >> 3) + 32 * i, gk = k0 + 4 * (tid & 7);
                va4[i] = gm < g.M && gk < ke ? *reinterpret_cast<const float4*>(g.A + (int64_t)gm * g.sam + gk)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        if constexpr ((VEC & VB_K) != 0) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int gn = n0 + (tid >> 3) + 32 * i, gk = k0 + 4 * (tid & 7);
                vb4[i] = gn < g.N && gk < ke ? *reinterpret_cast<const float4*>(g.B + (int64_t)gn * g.sbn + gk)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        if constexpr (SPL) {
            const __bf16* ah = reinterpret_cast<const __bf16*>(g.A);
            const __bf16* bh = reinterpret_cast<const __bf16*>(g.B);
            const int64_t alo = (int64_t)g.M * g.sam, blo = (int64_t)g.N * g.sbn;
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int pc = tid + 256 * i, row = pc >> 2, kq = k0 + (pc & 3) * 8;
                const int gm = m0 + row, gn = n0 + row;
                const bool ka = kq < ke;
#pragma unroll
                for (int pl = 0; pl < 2; pl++) {
                    bf16x8 va, vb;
#pragma unroll
                    for (int e = 0; e < 8; e++) {
                        va[e] = (__bf16)0.f;
                        vb[e] = (__bf16)0.f;
                    }
                    if (ka && gm < g.M) va = *reinterpret_cast<const bf16x8*>(ah + pl * alo + (int64_t)gm * g.sam + kq);
                    if (ka && gn < g.N) vb = *reinterpret_cast<const bf16x8*>(bh + pl * blo + (int64_t)gn * g.sbn + kq);
                    sa[pl][i] = va;
                    sb[pl][i] = vb;
                }
            }
        } else if constexpr (CM == CV_FWD || CM == CV_DX) {
            int64_t toff[2], boff[2];
            int dyq[2], dxq[2];
            bool kin[2];
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const int k = k0 + kp + q;
                const int tap = k / cs, c = k - tap * cs;
                int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
                boff[q] = (int64_t)c * g.sbk + tap;
                if (CM == CV_DX) { dy = -dy; dx = -dx; }
                dyq[q] = dy;
                dxq[q] = dx;
                toff[q] = (int64_t)(dy * 11 + dx) * cs + c;
                kin[q] = k < ke;
            }
            int p = pa0;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int gm = m0 + rp + 16 * i;
                const int y = div11(p), x = p - 11 * y;
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    const bool ok = gm < g.M && kin[q] && (unsigned)(y + dyq[q]) < 11u && (unsigned)(x + dxq[q]) < 11u;
                    ra[2 * i + q] = ok ? g.A[(int64_t)gm * cs + toff[q]] : 0.f;
                }
                p += 16;
                if (p >= 121) p -= 121;
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int gn = n0 + rp + 16 * i;
#pragma unroll
                for (int q = 0; q < 2; q++)
                    rb[2 * i + q] = (gn < g.N && kin[q]) ? g.B[boff[q] + (int64_t)gn * g.sbn] : 0.f;
            }
        } else {
            if constexpr ((VEC & VA_K) != 0) {
                // A staged from va4 (the 16-B loads above)
            } else if (a_kc) {
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int gm = m0 + rp + 16 * i;
#pragma unroll
                    for (int q = 0; q < 2; q++) {
                        const int gk = k0 + kp + q;
                        ra[2 * i + q] = (gm < g.M && gk < ke) ? g.A[(int64_t)gm * g.sam + (int64_t)gk * g.sak] : 0.f;
                    }
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    const int idx = tid + 256 * i;
                    const int kk = idx >> 7, mm = idx & 127;
                    const int gm = m0 + mm, gk = k0 + kk;
                    ra[i] = (gm < g.M && gk < ke) ? g.A[(int64_t)gm * g.sam + (int64_t)gk * g.sak] : 0.f;
                }
            }
            if constexpr ((VEC & VB_K) != 0) {
                // B staged from vb4
            } else if constexpr (CM == CV_DW) {
                const int gn = n0 + (tid & 127);
                const int m1 = k0 + (tid >> 7);
                int p = (int)((uint32_t)m1 - div121((uint32_t)m1) * 121u);
                const int64_t toff = (int64_t)(dw_dy * 11 + dw_dx) * cs + dw_c;
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    const int gk = m1 + 2 * i;
                    const int y = div11(p), x = p - 11 * y;
                    const bool ok = gn < g.N && gk < ke && (unsigned)(y + dw_dy) < 11u && (unsigned)(x + dw_dx) < 11u;
                    rb[i] = ok ? g.B[(int64_t)gk * cs + toff] : 0.f;
                    p += 2;
                    if (p >= 121) p -= 121;
                }
            } else if (b_nc) {
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    const int idx = tid + 256 * i;
                    const int kk = idx >> 7, nn = idx & 127;
                    const int gn = n0 + nn, gk = k0 + kk;
                    rb[i] = (gn < g.N && gk < ke) ? g.B[(int64_t)gk * g.sbk + (int64_t)gn * g.sbn] : 0.f;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int gn = n0 + rp + 16 * i;
#pragma unroll
                    for (int q = 0; q < 2; q++) {
                        const int gk = k0 + kp + q;
                        rb[2 * i + q] = (gn < g.N && gk < ke) ? g.B[(int64_t)gk * g.sbk + (int64_t)gn * g.sbn] : 0.f;
                    }
                }
            }
        }
    };
    // one k pair -> hi pair and lo pair, each a 4-byte LDS store
    auto put2 = [&](__bf16 (*S)[TB][PK], int row, int kk, float v0, float v1) {
        const __bf16 h0 = (__bf16)v0, h1 = (__bf16)v1;
        const __bf16 l0 = (__bf16)(v0 - (float)h0), l1 = (__bf16)(v1 - (float)h1);
        *reinterpret_cast<uint32_t*>(&S[0][row][kk]) =
            (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
        *reinterpret_cast<uint32_t*>(&S[1][row][kk]) =
            (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
    };
    auto stash = [&]() {
        // 4 consecutive k of one row (the 16-B loads): 8-B hi and lo stores
        auto put4 = [&](__bf16 (*S)[TB][PK], const float4 v, int i) {
            const float f[4] = {v.x, v.y, v.z, v.w};
            bf16x4 hi, lo;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const __bf16 b = (__bf16)f[e];
                hi[e] = b;
                lo[e] = (__bf16)(f[e] - (float)b);
            }
            const int row = (tid >> 3) + 32 * i, kk = 4 * (tid & 7);
            *reinterpret_cast<bf16x4*>(&S[0][row][kk]) = hi;
            *reinterpret_cast<bf16x4*>(&S[1][row][kk]) = lo;
        };
        if constexpr (SPL) {
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int pc = tid + 256 * i, row = pc >> 2, kq = (pc & 3) * 8;
#pragma unroll
                for (int pl = 0; pl < 2; pl++) {
                    *reinterpret_cast<bf16x8*>(&As[pl][row][kq]) = sa[pl][i];
                    *reinterpret_cast<bf16x8*>(&Bs[pl][row][kq]) = sb[pl][i];
                }
            }
            return;
        }
        if constexpr ((VEC & VA_K) != 0) {
#pragma unroll
            for (int i = 0; i < 4; i++) put4(As, va4[i], i);
        } else if (a_kc) {
#pragma unroll
            for (int i = 0; i < 8; i++) put2(As, rp + 16 * i, kp, ra[2 * i], ra[2 * i + 1]);
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const int idx = tid + 256 * i;
                const int kk = idx >> 7, mm = idx & 127;
                const __bf16 hi = (__bf16)ra[i];
                As[0][mm][kk] = hi;
                As[1][mm][kk] = (__bf16)(ra[i] - (float)hi);
            }
        }
        if constexpr ((VEC & VB_K) != 0) {
#pragma unroll
            for (int i = 0; i < 4; i++) put4(Bs, vb4[i], i);
        } else if (!b_nc) {
#pragma unroll
            for (int i = 0; i < 8; i++) put2(Bs, rp + 16 * i, kp, rb[2 * i], rb[2 * i + 1]);
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const int idx = tid + 256 * i;
                const int kk = idx >> 7, nn = idx & 127;
                const __bf16 hi = (__bf16)rb[i];
                Bs[0][nn][kk] = hi;
                Bs[1][nn][kk] = (__bf16)(rb[i] - (float)hi);
            }
        }
    };
    if (kb < ke) fetch(kb);
    for (int k0 = kb; k0 < ke; k0 += BK) {
        stash();
        __syncthreads();
        if (k0 + BK < ke) fetch(k0 + BK);  // in flight during the MFMAs below
        const int h = lane >> 5;
#pragma unroll
        for (int s = 0; s < BK / 16; s++) {
            bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int ar = wm * 64 + i * 32 + (lane & 31), br = wn * 64 + i * 32 + (lane & 31);
                ah[i] = *reinterpret_cast<const bf16x8*>(&As[0][ar][16 * s + 8 * h]);
                al[i] = *reinterpret_cast<const bf16x8*>(&As[1][ar][16 * s + 8 * h]);
                bh[i] = *reinterpret_cast<const bf16x8*>(&Bs[0][br][16 * s + 8 * h]);
                bl[i] = *reinterpret_cast<const bf16x8*>(&Bs[1][br][16 * s + 8 * h]);
            }
#pragma unroll
            for (int mi = 0; mi < 2; mi++)
#pragma unroll
                for (int ni = 0; ni < 2; ni++) {
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mi], bh[ni], acc[mi][ni], 0, 0, 0);
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mi], bl[ni], acc[mi][ni], 0, 0, 0);
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[mi], bh[ni], acc[mi][ni], 0, 0, 0);
                }
        }
        __syncthreads();
    }
    const bool split = gridDim.z > 1;
#pragma unroll
    for (int ni = 0; ni < 2; ni++) {
        const int gn = n0 + wn * 64 + ni * 32 + (lane & 31);
        if (gn >= g.N) continue;
        const float bias = g.bias ? g.bias[gn] : 0.f;
#pragma unroll
        for (int mi = 0; mi < 2; mi++) {
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int gm = m0 + wm * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (gm >= g.M) continue;
                float* cp = g.C + (int64_t)gm * g.ldc + gn;
                if (split) {  // this K slice's partial, summed in slice order by splitk_reduce_kernel
                    g.ws[((int64_t)blockIdx.z * g.M + gm) * g.N + gn] = g.alpha * acc[mi][ni][r];
                    continue;
                }
                float v = g.alpha * acc[mi][ni][r] + bias;
                if (g.flags & EVX_GEMM_RELU) v = v > 0.f ? v : 0.f;
                if (g.mask) v = g.mask[(int64_t)gm * g.ldm + gn] ? v * g.mask_scale : 0.f;
                if (g.gate) v = g.gate[(int64_t)gm * g.ldg + gn] > 0.f ? v : 0.f;
                if (g.flags & EVX_GEMM_ACCUM) v += *cp;
                *cp = v;
            }
        }
    }
}

// Split-K reduction + epilogue: C = epi(sum_z ws[z][m][n]) with the slices added in slice order
// (deterministic: the same bits on every call), then bias, ReLU, dropout mask, gate, accumulate --
// the same sequence as the one-pass epilogue. Four consecutive columns per thread (16-B loads).
__global__ __launch_bounds__(256) void splitk_reduce_kernel(evx_gemm_desc g, int S) {
    const int64_t MN = (int64_t)g.M * g.N;
    const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i0 >= MN) return;
    float v[4];
    const bool vec = (i0 + 4 <= MN) && ((MN & 3) == 0);
    if (vec) {
        float4 a = *reinterpret_cast<const float4*>(g.ws + i0);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
#pragma unroll 8
        for (int z = 1; z < S; z++) {
            const float4 b = *reinterpret_cast<const float4*>(g.ws + (int64_t)z * MN + i0);
            v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
        }
    } else {
        for (int j = 0; j < 4; j++) {
            v[j] = 0.f;
            if (i0 + j < MN) {
                v[j] = g.ws[i0 + j];
                for (int z = 1; z < S; z++) v[j] += g.ws[(int64_t)z * MN + i0 + j];
            }
        }
    }
    for (int j = 0; j < 4; j++) {
        const int64_t i = i0 + j;
        if (i >= MN) break;
        const int64_t gm = i / g.N;
        const int gn = (int)(i - gm * g.N);
        float* cp = g.C + gm * g.ldc + gn;
        float x = v[j] + (g.bias ? g.bias[gn] : 0.f);
        if (g.flags & EVX_GEMM_RELU) x = x > 0.f ? x : 0.f;
        if (g.mask) x = g.mask[gm * g.ldm + gn] ? x * g.mask_scale : 0.f;
        if (g.gate) x = g.gate[gm * g.ldg + gn] > 0.f ? x : 0.f;
        if (g.flags & EVX_GEMM_ACCUM) x += *cp;
        *cp = x;
    }
}

// x3 GEMM with both f32 operands k-major ("TN": the weight gradients dW = dY^T X, K = the batch or
// pixel rows): C[m][n] = sum_k A[k][m] B[k][n], A[k][m] = g.A[k sak + m] (sam = 1), B[k][n] =
// g.B[k sbk + n] (sbn = 1) or, CONV (EVX_CONV_DW), B[k][n] = X[pixel k shifted by tap][c] for the
// tap-major column n = tap cs + c, stored at the reference's column c * 9 + tap. 128 x 128 tiles of
// 4 waves (2 x 2 of 64 x 64), K chunks of 64 rows staged in their memory order ([k][m] / [k][n])
// as bf16 hi and lo planes (split in registers from 16-B f32 loads, 8-B LDS stores) and read back
// by ds_read_b64_tr_b16, which hands each lane the 8 consecutive k of its column -- the generic
// kernel's one-element transposing staging took ~0.3 PF on these shapes. The next chunk's loads
// are in flight while the current one's MFMAs run. x3 products hi*hi + hi*lo + lo*hi, f32
// accumulation; gridDim.z splits K into the workspace ws[z][M][N] (splitk_reduce adds in order).
constexpr int T3K = 64, T3P = TB + 32;  // K chunk, LDS row pitch (bf16): 320-B rows, conflict-free tr reads
constexpr int TN3_LDS = 4 * T3K * T3P * 2;  // A hi, A lo, B hi, B lo: 80 KB (two workgroups per CU)
// AK (A k-contiguous, A[m][k] = g.A[m sam + k]): A staged as [m][k] rows (pitch T3K + 8: conflict-free
// 16-B fragment reads) -- the activation gradients dX = dY W of the fc layers
constexpr int T3AP = T3K + 8;
static_assert(2 * TB * T3AP <= 2 * T3K * T3P, "the AK A planes fit the [k][m] ones' space");
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
__device__ __forceinline__ bf16x8 tr_frag3(const __bf16* img, int lane_off, int k0, int c0) {
    const __bf16* p0 = img + k0 * T3P + c0 + lane_off;
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p0));
    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p0 + 4 * T3P));
    const s16x4_t v[2] = {lo, hi};
    return __builtin_bit_cast(bf16x8, v);
}
template <bool CONV, bool AK = false>
__global__ __launch_bounds__(256, 2) void tn3_kernel(evx_gemm_desc g, int klen, int cs) {
    extern __shared__ __attribute__((aligned(16))) char tsm[];
    auto img = reinterpret_cast<__bf16 (*)[T3K][T3P]>(tsm);  // [4][T3K][T3P]
    auto imga = reinterpret_cast<__bf16 (*)[TB][T3AP]>(tsm);  // AK: [2][TB][T3AP] over planes 0-1
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    const int wm = w >> 1, wn = w & 1;
    const int bx = (int)blockIdx.x, by = (int)blockIdx.y;
    const int m0 = by * TB, n0 = bx * TB;
    const int kb = blockIdx.z * klen, ke = min(g.K, kb + klen);
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;
    // staging: thread t moves 4 columns 4 (t & 31) .. + 3 of rows (t >> 5) + 8 j (j < 8) of each operand
    const int sc = 4 * (tid & 31), sr = tid >> 5;
    const int am = m0 + sc, bn = n0 + sc;
    // CONV: this thread's 4 columns share one tap (cs % 4 == 0): its pixel shift and channel
    int cdy = 0, cdx = 0, cc = 0;
    if constexpr (CONV) {
        const int tap = bn / cs;
        cc = bn - tap * cs;
        cdy = tap / 3 - 1;
        cdx = tap - (tap / 3) * 3 - 1;
    }
    float4 ra[8], rb[8];
    // AK: thread t moves k 4 (t & 15) .. + 3 of rows m0 + (t >> 4) + 16 j
    const int akk = 4 * (tid & 15), akm = tid >> 4;
    auto fetch = [&](int k0) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int k = k0 + sr + 8 * j;
            const bool kin = k < ke;
            if constexpr (AK) {
                const int m = m0 + akm + 16 * j, kk = k0 + akk;
                ra[j] = m < g.M && kk < ke ? *reinterpret_cast<const float4*>(g.A + (int64_t)m * g.sam + kk)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                ra[j] = kin && am < g.M ? *reinterpret_cast<const float4*>(g.A + (int64_t)k * g.sak + am)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            if constexpr (CONV) {
                const int q = (int)((uint32_t)k - div121((uint32_t)k) * 121u), y = div11(q), x = q - 11 * y;
                const bool ok = kin && bn < g.N && (unsigned)(y + cdy) < 11u && (unsigned)(x + cdx) < 11u;
                rb[j] = ok ? *reinterpret_cast<const float4*>(g.B + (int64_t)(k + cdy * 11 + cdx) * cs + cc)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                rb[j] = kin && bn < g.N ? *reinterpret_cast<const float4*>(g.B + (int64_t)k * g.sbk + bn) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    };
    auto split4 = [](float4 v, uint2& hv, uint2& lv) {
        const float f[4] = {v.x, v.y, v.z, v.w};
        __bf16 hi[4], lo[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            hi[e] = (__bf16)f[e];
            lo[e] = (__bf16)(f[e] - (float)hi[e]);
        }
        hv = __builtin_bit_cast(uint2, hi);
        lv = __builtin_bit_cast(uint2, lo);
    };
    auto put4 = [&](int pl, int row, float4 v) {  // 4 columns: hi into plane pl, lo into pl + 1 (8-B stores)
        uint2 hv, lv;
        split4(v, hv, lv);
        *reinterpret_cast<uint2*>(&img[pl][row][sc]) = hv;
        *reinterpret_cast<uint2*>(&img[pl + 1][row][sc]) = lv;
    };
    const int q4 = (lane >> 2) & 3, pq = lane & 3;
    const int lane_off = (8 * h + q4) * T3P + 16 * ((lane >> 4) & 1) + 4 * pq;
    if (kb < ke) fetch(kb);
    for (int k0 = kb; k0 < ke; k0 += T3K) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if constexpr (AK) {
                uint2 hv, lv;
                split4(ra[j], hv, lv);
                *reinterpret_cast<uint2*>(&imga[0][akm + 16 * j][akk]) = hv;
                *reinterpret_cast<uint2*>(&imga[1][akm + 16 * j][akk]) = lv;
            } else {
                put4(0, sr + 8 * j, ra[j]);
            }
            put4(2, sr + 8 * j, rb[j]);
        }
        __syncthreads();
        if (k0 + T3K < ke) fetch(k0 + T3K);
#pragma unroll
        for (int s = 0; s < T3K / 16; s++) {
            bf16x8 av[2][2], bv[2][2];  // [plane][tile]
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int p = 0; p < 2; p++) {
                    if constexpr (AK)
                        av[p][i] = *reinterpret_cast<const bf16x8*>(&imga[p][wm * 64 + i * 32 + (lane & 31)][s * 16 + 8 * h]);
                    else
                        av[p][i] = tr_frag3(&img[p][0][0], lane_off, s * 16, wm * 64 + i * 32);
                    bv[p][i] = tr_frag3(&img[2 + p][0][0], lane_off, s * 16, wn * 64 + i * 32);
                }
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[0][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[1][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1][i], bv[0][j], acc[i][j], 0, 0, 0);
                }
        }
        __syncthreads();
    }
    // raw sums: C itself (one K slice) or the slice's workspace part; CONV columns to c * 9 + tap
    float* out = gridDim.z == 1 ? g.C : g.ws + (int64_t)blockIdx.z * g.M * g.N;
    const int64_t ld = gridDim.z == 1 ? g.ldc : g.N;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int n = n0 + wn * 64 + j * 32 + (lane & 31);
        if (n >= g.N) continue;
        int col = n;
        if constexpr (CONV) {
            const int tap = n / cs;
            col = (n - tap * cs) * 9 + tap;
        }
        const bool epi = !CONV && gridDim.z == 1;  // one K pass: evx_gemm's epilogue here (else the reduction's)
        const float bv = epi && g.bias ? g.bias[n] : 0.f;
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m >= g.M) continue;
                float x = acc[i][j][r];
                if (epi) {
                    x += bv;
                    if (g.flags & EVX_GEMM_RELU) x = x > 0.f ? x : 0.f;
                    if (g.mask) x = g.mask[(int64_t)m * g.ldm + n] ? x * g.mask_scale : 0.f;
                    if (g.gate) x = g.gate[(int64_t)m * g.ldg + n] > 0.f ? x : 0.f;
                    if (g.flags & EVX_GEMM_ACCUM) x += out[(int64_t)m * ld + col];
                }
                out[(int64_t)m * ld + col] = x;
            }
    }
}

// splitk_reduce_kernel for many slices (S >= 8, M N a multiple of 4): a workgroup takes 64 float4
// of C, each wave sums a contiguous quarter of the slices (in slice order) and wave 0 adds the four
// quarter sums in order -- 4x the workgroups and a quarter of the dependent loads per thread of
// the one-thread-per-float4 form (the conv weight gradients: S ~ 100 slices of a 73 728-float C)
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(evx_gemm_desc g, int S) {
    __shared__ float4 part[3][64];
    const int64_t MN = (int64_t)g.M * g.N;
    const int q = (int)threadIdx.x >> 6, l = (int)threadIdx.x & 63;
    const int64_t i0 = ((int64_t)blockIdx.x * 64 + l) * 4;
    const bool live = i0 < MN;
    const int z0 = q * S / 4, z1 = (q + 1) * S / 4;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (live) {
        a = *reinterpret_cast<const float4*>(g.ws + (int64_t)z0 * MN + i0);
#pragma unroll 8  // 8 loads in flight; the adds stay in slice order (the same bits)
        for (int z = z0 + 1; z < z1; z++) {
            const float4 b = *reinterpret_cast<const float4*>(g.ws + (int64_t)z * MN + i0);
            a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        }
    }
    if (q) part[q - 1][l] = a;
    __syncthreads();
    if (q || !live) return;
    float v[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float4 b = part[k][l];
        v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
    }
    for (int j = 0; j < 4; j++) {
        const int64_t i = i0 + j;
        const int64_t gm = i / g.N;
        const int gn = (int)(i - gm * g.N);
        float* cp = g.C + gm * g.ldc + gn;
        float x = v[j] + (g.bias ? g.bias[gn] : 0.f);
        if (g.flags & EVX_GEMM_RELU) x = x > 0.f ? x : 0.f;
        if (g.mask) x = g.mask[gm * g.ldm + gn] ? x * g.mask_scale : 0.f;
        if (g.gate) x = g.gate[gm * g.ldg + gn] > 0.f ? x : 0.f;
        if (g.flags & EVX_GEMM_ACCUM) x += *cp;
        *cp = x;
    }
}

// ------------------------------------------------------------- column sums
// out[n] (+)= sum_m X[m*ld + n], deterministic: fixed-order partials then a fixed-order total.
// Partials: COLSUM_ROWS rows per chunk; a block covers 64 columns x 4 chunks (the 4 waves), so a
// narrow matrix (a conv layer's 32 channels) still fills its lanes. The total: one block per
// column, strided partial sums then a fixed LDS tree (was one thread per column walking every
// chunk: ~110 us for the 968 chunks of a 123 904-pixel conv layer).
constexpr int COLSUM_ROWS = 64;
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ X, int64_t ld, int M, int N,
                                                     float* __restrict__ part, int chunks) {
    const int n = blockIdx.x * 64 + (threadIdx.x & 63);
    const int c = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (n >= N || c >= chunks) return;
    const int rows = (M + chunks - 1) / chunks;
    const int r0 = c * rows, r1 = min(M, r0 + rows);
    float s = 0.f;
#pragma unroll 8  // 8 loads in flight; the adds in row order (the same bits)
    for (int m = r0; m < r1; m++) s += X[(int64_t)m * ld + n];
    part[(int64_t)c * N + n] = s;
}
__global__ __launch_bounds__(256) void colsum_finish(const float* __restrict__ part, int N, int chunks,
                                                     float* __restrict__ out, int accum) {
    __shared__ float red[256];
    const int n = blockIdx.x, t = threadIdx.x;
    float s = 0.f;
#pragma unroll 8
    for (int c = t; c < chunks; c += 256) s += part[(int64_t)c * N + n];
    red[t] = s;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (t < h) red[t] += red[t + h];
        __syncthreads();
    }
    if (t == 0) out[n] = accum ? out[n] + red[0] : red[0];
}

// --------------------------------------------------------------- TD loss
// DQNAgent.learn (agents/dqn_agent.py:143-151): q = Q(s).gather(a); y = r + gamma *
// max Q_tgt(s') * ~done; loss = mean((q - y)^2); dQ[i, a_i] = 2 (q - y) / B. With
// importance weights w (prioritized replay): loss = mean(w (q - y)^2), and |q - y| out.
// One row per thread over many blocks, each block's partial into the caller's workspace; a
// one-block launch per net then sums them in block order (deterministic; no module state, so
// launches on different streams with their own workspaces never meet).
__global__ __launch_bounds__(256) void td_loss_kernel(const float* __restrict__ Q, const float* __restrict__ Qt,
                                                      int A, const int32_t* __restrict__ act,
                                                      const float* __restrict__ rew, const uint8_t* __restrict__ done,
                                                      float gamma, int B, const float* __restrict__ w,
                                                      float* __restrict__ dQ, float* __restrict__ part,
                                                      float* __restrict__ td_abs, int ntd = 0,
                                                      float* __restrict__ zero = nullptr, int64_t nzero = 0) {
    __shared__ float red[256];
    if (zero && (int)blockIdx.x >= ntd) {  // the extra workgroups clear the gradient buffer for the backward
        if (blockIdx.y) return;
        const int64_t z0 = ((int64_t)blockIdx.x - ntd) * 256 + threadIdx.x, zs = ((int64_t)gridDim.x - ntd) * 256;
        for (int64_t k = z0; k < nzero; k += zs) zero[k] = 0.f;
        return;
    }
    const unsigned nb = zero ? (unsigned)ntd : gridDim.x;
    // grouped nets (evx_td_loss_zero_g): net blockIdx.y owns rows [y B, (y + 1) B) and loss_out[y]
    const unsigned gy = blockIdx.y;
    if (gy) {
        const size_t o = (size_t)gy * B;
        Q += o * A;
        Qt += o * A;
        act += o;
        rew += o;
        done += o;
        if (w) w += o;
        dQ += o * A;
        if (td_abs) td_abs += o;
    }
    const float nrm = (float)B;
    const int i = blockIdx.x * 256 + threadIdx.x;
    float pt = 0.f;
    if (i < B) {
        float mx = Qt[(int64_t)i * A];
        for (int j = 1; j < A; j++) mx = fmaxf(mx, Qt[(int64_t)i * A + j]);
        const float y = rew[i] + gamma * mx * (done[i] ? 0.f : 1.f);
        const int a = act[i];
        const float d = Q[(int64_t)i * A + a] - y;
        // prioritized replay: importance weights scale each squared error and its gradient
        const float wi = w ? w[i] : 1.f;
        pt = w ? wi * (d * d) : d * d;
        const float g = w ? wi * (2.f * d) : 2.f * d;
        for (int j = 0; j < A; j++) dQ[(int64_t)i * A + j] = (j == a) ? g / nrm : 0.f;
        if (td_abs) td_abs[i] = fabsf(d);
    }
    red[threadIdx.x] = pt;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[gy * nb + blockIdx.x] = red[0];
}
// loss[y] = (sum of net y's nb block partials) / B: strided partial sums, then a fixed LDS tree
__global__ __launch_bounds__(256) void td_finish_kernel(const float* __restrict__ part, int nb, int B,
                                                        float* __restrict__ loss_out) {
    __shared__ float red[256];
    const float* p = part + (size_t)blockIdx.x * nb;
    float t = 0.f;
    for (int k = threadIdx.x; k < nb; k += 256) t += p[k];
    red[threadIdx.x] = t;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) loss_out[blockIdx.x] = red[0] / (float)B;
}

// ------------------------------------------------- clip_grad_norm_ + Adam
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, int64_t n, float* __restrict__ part) {
    __shared__ float red[256];
    float s = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) s += g[i] * g[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}
__global__ __launch_bounds__(256) void sumsq_finish(const float* __restrict__ part, int nparts, float* __restrict__ norm) {
    __shared__ float red[256];
    float s = 0.f;
    for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) norm[0] = sqrtf(red[0]);
}

// torch.nn.utils.clip_grad_norm_ (coef = max_norm / (norm + 1e-6), clamped <= 1) fused
// with torch.optim.Adam's update (exp_avg.lerp_, exp_avg_sq.mul_.addcmul_, addcdiv_).
__global__ __launch_bounds__(256) void clip_adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                        const float* __restrict__ norm, float max_norm, float lr,
                                                        float beta1, float beta2, float eps, float step_size,
                                                        float bc2_sqrt, float weight_decay) {
    float coef = 1.f;
    if (norm && max_norm > 0.f) {
        coef = max_norm / (norm[0] + 1e-6f);
        coef = coef < 1.f ? coef : 1.f;
    }
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        float gi = g[i] * coef;
        if (weight_decay != 0.f) gi += weight_decay * p[i];
        const float mi = m[i] + (gi - m[i]) * (1.f - beta1);
        const float vi = v[i] * beta2 + (1.f - beta2) * gi * gi;
        m[i] = mi;
        v[i] = vi;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        p[i] = p[i] - step_size * (mi / denom);
        g[i] = gi;
    }
}

// ------------------------------------------------------------- dropout mask
// keep with probability 1-p (torch.nn.Dropout semantics; mask values 0/1)
__global__ __launch_bounds__(256) void dropout_mask_kernel(uint8_t* __restrict__ mask, int64_t n, float p,
                                                           uint64_t seed, uint64_t offset) {
    const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i4 >= n) return;
    const uint64_t c = (uint64_t)i4 / 4 + offset;
    const u4 r = philox((uint32_t)c, (uint32_t)(c >> 32), 0x5eedu, 0u, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
    for (int j = 0; j < 4 && i4 + j < n; j++) mask[i4 + j] = u01(rr[j]) >= p ? 1 : 0;
}

// ------------------------------------------------------------------- act
// DQNAgent.act (agents/dqn_agent.py:101-124): with probability epsilon a uniform
// random action, else argmax_a Q (first maximum, as np.argmax).
__global__ __launch_bounds__(256) void act_kernel(const float* __restrict__ Q, int n, int A, float epsilon,
                                                  uint64_t seed, uint64_t offset, int32_t* __restrict__ actions) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    int best = 0;
    float bv = Q[(int64_t)i * A];
    for (int j = 1; j < A; j++) {
        const float q = Q[(int64_t)i * A + j];
        if (q > bv) {
            bv = q;
            best = j;
        }
    }
    if (epsilon > 0.f) {
        const uint64_t c = (uint64_t)i + offset;
        const u4 r = philox((uint32_t)c, (uint32_t)(c >> 32), 0xac7u, 0u, (uint32_t)seed, (uint32_t)(seed >> 32));
        if (u01(r.x) <= epsilon) best = (int)((uint64_t)r.y * (uint64_t)A >> 32);
    }
    actions[i] = best;
}

// ---------------------------------------------------------------- replay
// Uniform replay ring (DQNAgent.memory, agents/dqn_agent.py:88-99) with compact
// observations; per-agent transitions share the env's team reward/done.
__global__ __launch_bounds__(256) void replay_push_kernel(evx_replay rp, const evx_obs* __restrict__ s,
                                                          const evx_obs* __restrict__ s2,
                                                          const evx_obs* __restrict__ s2_term, const int32_t* __restrict__ a,
                                                          const double* __restrict__ r_env,
                                                          const uint8_t* __restrict__ done_env, int n, int agents_per_env,
                                                          int64_t pos) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t slot = (pos + i) % rp.capacity;
    const int e = i / agents_per_env;
    rp.s[slot] = s[i];
    rp.s2[slot] = (s2_term && done_env[e]) ? s2_term[i] : s2[i];
    rp.a[slot] = a[i];
    rp.r[slot] = (float)r_env[e];
    rp.done[slot] = done_env[e];
}

// Sampling WITHOUT replacement, as DQNAgent.learn's random.sample(memory, B)
// (agents/dqn_agent.py:132): draw i of a batch is perm(i) for a keyed pseudo-random permutation
// perm of [0, n) -- a 6-round balanced Feistel network on the smallest even-width domain 2^w >= n,
// cycle-walked back into [0, n) (terminates: i's cycle under the domain permutation contains i
// itself; expected < 4 rounds of walking since 2^w < 4n). Round keys from Philox4x32-10 of the
// draw's (offset, stream) under the seed, so each learn step's batch is a fresh permutation and
// the B draws are distinct (B <= n). oracle/draw_oracle.c orc_replay_indices restates it.
__global__ __launch_bounds__(256) void replay_sample_kernel(evx_replay rp, int64_t base, int64_t size, int B, uint64_t seed,
                                                            uint64_t offset, evx_obs* __restrict__ s,
                                                            evx_obs* __restrict__ s2, int32_t* __restrict__ a,
                                                            float* __restrict__ r, uint8_t* __restrict__ done,
                                                            int64_t* __restrict__ idx_out, int nets = 1,
                                                            int joint = 0) {
    const int i0 = blockIdx.x * 256 + threadIdx.x;
    if (i0 >= B) return;
    // nets > 1 (evx_replay_sample_agents): agent blockIdx.y's own transitions -- the ring slots
    // == agent (mod nets) -- into rows [agent B, (agent + 1) B), a permutation keyed by the agent;
    // joint (evx_replay_sample_joint): draw i is shared by every agent (the same env-steps)
    const int g = (int)blockIdx.y;
    const int i = g * B + i0;
    const uint64_t n = nets > 1 ? (uint64_t)(size / nets) : (uint64_t)size;
    const perm_key pk = make_perm_key(n, seed, offset, joint ? 0u : (uint32_t)g);
    const uint64_t d = perm_apply(pk, (uint64_t)i0, n);
    int64_t j;
    if (nets > 1) {
        j = (int64_t)d * nets + g;
    } else {
        j = base + (int64_t)d;
        if (j >= rp.capacity) j -= rp.capacity;
    }
    s[i] = rp.s[j];
    s2[i] = rp.s2[j];
    a[i] = rp.a[j];
    r[i] = rp.r[j];
    done[i] = rp.done[j];
    if (idx_out) idx_out[i] = j;
}

__global__ __launch_bounds__(256) void gather_rows_kernel(const evx_obs* __restrict__ src,
                                                          const int64_t* __restrict__ idx, int n,
                                                          evx_obs* __restrict__ dst) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[i] = src[idx[i]];
}

// ------------------------------------------------------------ conv helpers
// DQNNetwork conv layers (agents/dqn_agent.py:22-24,48-50): 3x3, padding 1, on
// 11x11 maps, as im2col + GEMM. x: [B][C][11][11] (NCHW); cols: [B*121][C*9]
// with k = c*9 + ky*3 + kx (the order of a Conv2d weight [Cout][C][3][3]).
__global__ __launch_bounds__(256) void im2col_kernel(const float* __restrict__ x, int B, int C, int nhwc,
                                                     float* __restrict__ cols) {
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t total = (int64_t)B * 121 * C * 9;
    if (gid >= total) return;
    const int K = C * 9;
    const int64_t row = gid / K;
    const int k = (int)(gid - row * K);
    const int b = (int)(row / 121), pix = (int)(row - (int64_t)b * 121);
    const int y = pix / 11, xx = pix - y * 11;
    const int c = k / 9, r = k - c * 9, ky = r / 3, kx = r - ky * 3;
    const int iy = y + ky - 1, ix = xx + kx - 1;
    float v = 0.f;
    if (iy >= 0 && iy < 11 && ix >= 0 && ix < 11) {
        // nhwc: input given as the reference's (B, 11, 11, C) observation tensor (permute folded here)
        v = nhwc ? x[(((int64_t)b * 11 + iy) * 11 + ix) * C + c] : x[(((int64_t)b * C + c) * 11 + iy) * 11 + ix];
    }
    cols[gid] = v;
}

// dx[b][c][iy][ix] = sum over (pixel, tap) mapping to it of dcols (fixed order, no atomics)
__global__ __launch_bounds__(256) void col2im_kernel(const float* __restrict__ dcols, int B, int C,
                                                     float* __restrict__ dx) {
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t total = (int64_t)B * C * 121;
    if (gid >= total) return;
    const int b = (int)(gid / (C * 121));
    const int rem = (int)(gid - (int64_t)b * C * 121);
    const int c = rem / 121, pix = rem - c * 121, iy = pix / 11, ix = pix - iy * 11;
    const int K = C * 9;
    float s = 0.f;
    for (int ky = 0; ky < 3; ky++)
        for (int kx = 0; kx < 3; kx++) {
            const int y = iy - ky + 1, xx = ix - kx + 1;
            if (y < 0 || y >= 11 || xx < 0 || xx >= 11) continue;
            s += dcols[((int64_t)b * 121 + y * 11 + xx) * K + c * 9 + ky * 3 + kx];
        }
    dx[gid] = s;
}

// [B*121][C] (GEMM output, pixel-major) <-> [B][C][121] (NCHW): one workgroup per b, its 121 C
// values read contiguously into LDS (pixel rows padded to C + 1 words: the column reads of the
// pixel-major side hit distinct banks) and written back contiguously in the other order
__global__ __launch_bounds__(256) void pix2nchw_kernel(const float* __restrict__ src, int B, int C, int to_nchw,
                                                       float* __restrict__ dst) {
    extern __shared__ float tl[];  // [121][C + 1]
    const int n = 121 * C;
    const float* __restrict__ s = src + (size_t)blockIdx.x * n;
    float* __restrict__ d = dst + (size_t)blockIdx.x * n;
    for (int j = threadIdx.x; j < n; j += 256) {
        const float v = s[j];
        if (to_nchw) {  // s: pixel-major (p * C + c)
            const int p = j / C, c = j - p * C;
            tl[p * (C + 1) + c] = v;
        } else {  // s: NCHW (c * 121 + p)
            const int c = j / 121, p = j - c * 121;
            tl[p * (C + 1) + c] = v;
        }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += 256) {
        if (to_nchw) {  // d: NCHW
            const int c = j / 121, p = j - c * 121;
            d[j] = tl[p * (C + 1) + c];
        } else {  // d: pixel-major
            const int p = j / C, c = j - p * C;
            d[j] = tl[p * (C + 1) + c];
        }
    }
}

// the same permutation element-wise, one output element per thread (C beyond the LDS tile)
__global__ __launch_bounds__(256) void pix2nchw_flat_kernel(const float* __restrict__ src, int64_t total, int C,
                                                            int to_nchw, float* __restrict__ dst) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= total) return;
    const int64_t n = (int64_t)121 * C;
    const int64_t b = j / n;
    const int r = (int)(j - b * n);
    int p, c;
    if (to_nchw) {  // d: NCHW (c * 121 + p), s: pixel-major
        c = r / 121;
        p = r - c * 121;
    } else {  // d: pixel-major (p * C + c), s: NCHW
        p = r / C;
        c = r - p * C;
    }
    dst[j] = src[b * n + (to_nchw ? (int64_t)p * C + c : (int64_t)c * 121 + p)];
}

// NCHW [B][C][121] -> pixel-major [B][121 * C] bf16 hi / lo planes (evx_pix_split)
__global__ __launch_bounds__(256) void pix_split_kernel(const float* __restrict__ src, int B, int C,
                                                        __bf16* __restrict__ dst) {
    extern __shared__ float tl[];  // [121][C + 1]
    const int n = 121 * C;
    const float* __restrict__ s = src + (size_t)blockIdx.x * n;
    __bf16* __restrict__ d = dst + (size_t)blockIdx.x * n;
    const size_t lo = (size_t)B * n;
    for (int j = threadIdx.x; j < n; j += 256) {
        const int c = j / 121, p = j - c * 121;
        tl[p * (C + 1) + c] = s[j];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += 256) {
        const int p = j / C, c = j - p * C;
        const float v = tl[p * (C + 1) + c];
        const __bf16 hi = (__bf16)v;
        d[j] = hi;
        d[j + lo] = (__bf16)(v - (float)hi);
    }
}

// dy[i] = y[i] > 0 ? dy[i] : 0 (ReLU backward for outputs that do not come out of a GEMM)
__global__ __launch_bounds__(256) void relu_grad_kernel(float* __restrict__ dy, const float* __restrict__ y,
                                                        int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n && !(y[i] > 0.f)) dy[i] = 0.f;
}

}  // namespace evxq

// ===================================================================== C-ABI
namespace {
thread_local char q_err[256] = "";
int qfail(int code, const char* msg) {
    snprintf(q_err, sizeof(q_err), "%s", msg);
    return code;
}
int qlaunch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) return 0;
    snprintf(q_err, sizeof(q_err), "%s: %s", what, hipGetErrorString(e));
    return -5;
}
unsigned nblk(int64_t n) { return (unsigned)((n + 255) / 256); }
}  // namespace

extern "C" {

const char* evx_q_last_error(void) { return q_err; }

}  // extern "C"

namespace {
// K slices of a GEMM (1: no split). Split K only on the bf16 / x3 paths (the exact-f32 path is
// the parity path and stays one pass). Without an epilogue: grids under 256 tiles with K >= 512
// (dW = dY^T X). With one (bias / ReLU / mask / gate), when the contraction is long enough to pay
// for the reduction pass: the conv net's fc1 (K = 15 488) at a learn batch of 1024 is 32 tiles,
// 1.19 ms unsplit; at the act's 8192 rows 256 tiles, one 4-wave workgroup per CU. Each K slice
// keeps >= 256 (>= 1024 with an epilogue) of the contraction. The slices' partials go to the
// caller's workspace (ws, [S][M][N] f32), so S is also capped by ws_elems / (M N).
int gemm_slices(const evx_gemm_desc* g, int64_t ws_cap, int* klen_out) {
    const int TB = evxq::TB;
    const int tiles = ((g->M + TB - 1) / TB) * ((g->N + TB - 1) / TB);
    const bool epi = g->bias || g->mask || g->gate || (g->flags & EVX_GEMM_RELU);
    int S = 1;
    if (g->precision != EVX_PREC_F32 && tiles < (epi ? 257 : 256) && g->K >= (epi ? 4096 : 512)) {
        S = ((epi ? 1024 : 512) + tiles - 1) / tiles;
        const int kmin = epi ? 1024 : 256;
        if (S > g->K / kmin) S = g->K / kmin;
        if (S < 1) S = 1;
    }
    if (S > 1) {
        const int64_t mn = (int64_t)g->M * g->N;
        const int64_t fit = ws_cap / mn;
        if (S > fit) S = (int)fit;
        if (S < 2) S = 1;
    }
    int klen = (g->K + S - 1) / S;
    klen = (klen + evxq::BK - 1) / evxq::BK * evxq::BK;
    S = (g->K + klen - 1) / klen;
    if (klen_out) *klen_out = klen;
    return S;
}

}  // namespace
namespace evxq {
// 3x3 convolution (padding 1, 11x11 maps, x3) of one image per workgroup, forward or dX
// (agents/dqn_agent.py:22-24,48-50: conv1 6 -> 32, conv2 32 -> 64, conv3 64 -> 128 channels, each
// + bias, ReLU; the backward's dX = dY (*) flip(W) with the lower layer's ReLU gate). The image
// (the layer input, or dY for dX) is staged in LDS as bf16 hi / lo planes over a 13x13
// zero-bordered grid, CB <= 64 channels at a time (channels padded to CP, a multiple of 16), so
// each of the 9 taps reads its shifted A fragments straight from LDS -- no per-element bounds tests
// or global gathers per tap and K tile as in gemm128x3_kernel<CV_FWD / CV_DX>. Output pixels are 4
// row tiles of 32 (121 live), the NT = N / 32 column tiles are dealt to the 4 waves (wave w: column
// tile w % NT, NT row tiles); K = channel blocks x 9 taps x CB channels in 16-deep steps. B
// fragments come pre-split from conv_wpack_kernel (a contiguous 1-KB hi and lo block per wave and
// k-step, two k-steps ahead). x3 products (hi*hi + hi*lo + lo*hi), f32 accumulation. Epilogue:
// forward -- bias, ReLU; dX -- the gate (the lower layer's output > 0); pixel-major rows
// C[img * 121 + p][n].
// Weights packed per call (the caller's workspace, per stream tag): k-step ks = (b * 9 + tap) *
// (CB / 16) + j, fragment (nt, ks) lane l holds W[n = 32 nt + (l & 31)][c][tap] (forward: sbn, sbk
// the torch strides; dX: c the dY channel) for c = b CB + 16 j + 8 (l >> 5) + e, e < 8 (0 past the
// staged channels), as bf16 hi at wp[((nt * KS + ks) * 64 + l) * 8 + e], lo NT * KS * 512 further.
template <int CP>
__device__ __forceinline__ void conv_kstep(int ks, int h, int& tap, int& c0) {
    constexpr int CB = CP > 64 ? 64 : CP, KJ = CB / 16;
    const int b = ks / (9 * KJ), r = ks - b * 9 * KJ;
    tap = r / KJ;
    c0 = b * CB + (r - tap * KJ) * 16 + 8 * h;
}
template <int CP>
__global__ __launch_bounds__(256) void conv_wpack_kernel(const float* __restrict__ W, int64_t sbk, int64_t sbn, int cin,
                                                         int NT, __bf16* __restrict__ wp) {
    constexpr int KS = 9 * CP / 16;
    const int i = (int)(blockIdx.x * 256 + threadIdx.x);
    if (i >= NT * KS * 64) return;
    const int l = i & 63, f = i >> 6, ks = f % KS, nt = f / KS;
    const int n = nt * 32 + (l & 31);
    int tap, c0;
    conv_kstep<CP>(ks, l >> 5, tap, c0);
    bf16x8 hi, lo;
#pragma unroll
    for (int e = 0; e < 8; e++) {
        const float v = c0 + e < cin ? W[(int64_t)n * sbn + (int64_t)(c0 + e) * sbk + tap] : 0.f;
        const __bf16 h = (__bf16)v;
        hi[e] = h;
        lo[e] = (__bf16)(v - (float)h);
    }
    *reinterpret_cast<bf16x8*>(wp + (size_t)i * 8) = hi;
    *reinterpret_cast<bf16x8*>(wp + (size_t)(NT * KS * 64 + i) * 8) = lo;
}
template <int CP, int NT, bool DX>
__global__ __launch_bounds__(256, 2) void conv3x3_x3_kernel(evx_gemm_desc g, int cin, const __bf16* __restrict__ wp) {
    constexpr int CB = CP > 64 ? 64 : CP, NB = CP / CB;
    constexpr int XP = CB + 8;  // LDS row pitch (bf16): 16-B aligned rows, spread banks
    constexpr int KSB = 9 * CB / 16, KS = NB * KSB;
    __shared__ __attribute__((aligned(16))) __bf16 Xs[2][169][XP];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    const int img = blockIdx.x;
    const float* __restrict__ X = g.A + (size_t)img * 121 * cin;
    // stage channel block b: every (13x13 cell, channel) of both planes; border cells and padded
    // channels are 0
    auto stage = [&](int b) {
        if (CB == 16 && cin == 6) {  // conv1: one cell per thread, its 6 channels as 3 8-B loads, 10 zeros
            for (int q = tid; q < 169; q += 256) {
                const int y = q / 13 - 1, x = q - (q / 13) * 13 - 1;
                float f[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                if ((unsigned)y < 11u && (unsigned)x < 11u) {
                    const float2* s2 = reinterpret_cast<const float2*>(X + (y * 11 + x) * 6);
#pragma unroll
                    for (int e = 0; e < 3; e++) {
                        const float2 v = s2[e];
                        f[2 * e] = v.x;
                        f[2 * e + 1] = v.y;
                    }
                }
                bf16x8 h0, h1, l0, l1;
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    h0[e] = h1[e] = l0[e] = l1[e] = (__bf16)0.f;
                }
#pragma unroll
                for (int e = 0; e < 6; e++) {
                    const __bf16 h = (__bf16)f[e];
                    h0[e] = h;
                    l0[e] = (__bf16)(f[e] - (float)h);
                }
                *reinterpret_cast<bf16x8*>(&Xs[0][q][0]) = h0;
                *reinterpret_cast<bf16x8*>(&Xs[0][q][8]) = h1;
                *reinterpret_cast<bf16x8*>(&Xs[1][q][0]) = l0;
                *reinterpret_cast<bf16x8*>(&Xs[1][q][8]) = l1;
            }
            return;
        }
        if (CB >= 32 && (cin & 3) == 0) {  // 4 channels per thread and pass: 16-B loads, 8-B LDS stores
            constexpr int C4 = CB / 4;
            for (int i = tid; i < 169 * C4; i += 256) {
                const int q = i / C4, c = (i - q * C4) * 4;
                const int y = q / 13 - 1, x = q - (q / 13) * 13 - 1;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (b * CB + c < cin && (unsigned)y < 11u && (unsigned)x < 11u)
                    v = *reinterpret_cast<const float4*>(X + (y * 11 + x) * cin + b * CB + c);
                const float f[4] = {v.x, v.y, v.z, v.w};
                bf16x4 hi, lo;
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const __bf16 h = (__bf16)f[e];
                    hi[e] = h;
                    lo[e] = (__bf16)(f[e] - (float)h);
                }
                *reinterpret_cast<bf16x4*>(&Xs[0][q][c]) = hi;
                *reinterpret_cast<bf16x4*>(&Xs[1][q][c]) = lo;
            }
            return;
        }
        for (int i = tid; i < 169 * CB; i += 256) {
            const int q = i / CB, c = i - q * CB;
            const int y = q / 13 - 1, x = q - (q / 13) * 13 - 1;
            float v = 0.f;
            if (b * CB + c < cin && (unsigned)y < 11u && (unsigned)x < 11u) v = X[(y * 11 + x) * cin + b * CB + c];
            const __bf16 hi = (__bf16)v;
            Xs[0][q][c] = hi;
            Xs[1][q][c] = (__bf16)(v - (float)hi);
        }
    };
    stage(0);
    const int nt = w % NT, mt0 = (w / NT) * NT;  // this wave: column tile nt, row tiles mt0 .. mt0 + NT - 1
    const int n = nt * 32 + (lane & 31);         // the lane's output channel (B operand row)
    int base[NT];                                // LDS cell of the lane's A row at tap offset (0, 0)
#pragma unroll
    for (int k = 0; k < NT; k++) {
        int m = (mt0 + k) * 32 + (lane & 31);
        m = m < 121 ? m : 0;  // rows 121.. read pixel 0 (their outputs are not stored)
        const int y = (m * 187) >> 11, x = m - 11 * y;
        base[k] = (y + 1) * 13 + (x + 1);
    }
    f32x16 acc[NT];
#pragma unroll
    for (int k = 0; k < NT; k++)
#pragma unroll
        for (int r = 0; r < 16; r++) acc[k][r] = 0.f;
    const __bf16* __restrict__ wh = wp + ((size_t)nt * KS * 64 + lane) * 8;
    const __bf16* __restrict__ wl = wh + (size_t)NT * KS * 512;
    bf16x8 bh = *reinterpret_cast<const bf16x8*>(wh), bl = *reinterpret_cast<const bf16x8*>(wl);
    bf16x8 bh1 = bh, bl1 = bl;
    if (KS > 1) {
        bh1 = *reinterpret_cast<const bf16x8*>(wh + 512);
        bl1 = *reinterpret_cast<const bf16x8*>(wl + 512);
    }
    __syncthreads();
    for (int ks = 0; ks < KS; ks++) {
        if (NB > 1 && ks > 0 && ks % KSB == 0) {  // the next channel block
            __syncthreads();
            stage(ks / KSB);
            __syncthreads();
        }
        bf16x8 bh2 = bh1, bl2 = bl1;
        if (ks + 2 < KS) {
            bh2 = *reinterpret_cast<const bf16x8*>(wh + (size_t)(ks + 2) * 512);
            bl2 = *reinterpret_cast<const bf16x8*>(wl + (size_t)(ks + 2) * 512);
        }
        int tap, c0;
        conv_kstep<CP>(ks, h, tap, c0);
        c0 -= (ks / KSB) * CB;  // channel within the staged block
        const int toff = (DX ? -1 : 1) * ((tap / 3 - 1) * 13 + (tap % 3 - 1));
#pragma unroll
        for (int k = 0; k < NT; k++) {
            const int q = base[k] + toff;
            const bf16x8 ah = *reinterpret_cast<const bf16x8*>(&Xs[0][q][c0]);
            const bf16x8 al = *reinterpret_cast<const bf16x8*>(&Xs[1][q][c0]);
            acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[k], 0, 0, 0);
            acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[k], 0, 0, 0);
            acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[k], 0, 0, 0);
        }
        bh = bh1;
        bl = bl1;
        bh1 = bh2;
        bl1 = bl2;
    }
    const float bias = !DX && g.bias ? g.bias[n] : 0.f;
    const bool relu = !DX && (g.flags & EVX_GEMM_RELU) != 0;
    const bool osp = !DX && (g.flags & EVX_GEMM_OUT_SPLIT) != 0;  // bf16 hi / lo planes
    float* __restrict__ Y = g.C + (size_t)img * 121 * g.ldc + n;
    __bf16* __restrict__ Yh = reinterpret_cast<__bf16*>(g.C) + (size_t)img * 121 * g.ldc + n;
    const size_t ylo = (size_t)g.M * g.ldc;
    const float* __restrict__ gate = DX && g.gate ? g.gate + (size_t)img * 121 * g.ldg + n : nullptr;
#pragma unroll
    for (int k = 0; k < NT; k++)
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const int m = (mt0 + k) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (m >= 121) continue;
            float v = acc[k][r] + bias;
            if (relu) v = v > 0.f ? v : 0.f;
            if (gate) v = gate[(size_t)m * g.ldg] > 0.f ? v : 0.f;
            if (osp) {
                const __bf16 hi = (__bf16)v;
                Yh[(size_t)m * g.ldc] = hi;
                Yh[(size_t)m * g.ldc + ylo] = (__bf16)(v - (float)hi);
            } else {
                Y[(size_t)m * g.ldc] = v;
            }
        }
}
// The forward of conv2 over many images (the act's 8192, the learner's 1024): 512-thread
// workgroups (one per CU) walk the images with their share of the layer's packed weights held in
// VGPRs for the whole launch -- conv3x3_x3_kernel re-read every weight fragment from L2 per image
// (295 KB per conv3 image: 2.4 GB per 8192-image act). A workgroup owns NTW of the layer's NT
// 32-channel column tiles (column group cg; the CG = NT / NTW groups of an image run on one XCD,
// so its input is fetched into that L2 once); wave w takes column tile w % NTW, and the 8 / NTW
// waves of a column tile split the 4 row tiles and (KH > 1) the K steps, the K parts added through
// LDS in a fixed order; conv2 (NT 2, NTW 2, KH 1): one row tile and all 18 k-steps per wave (act
// 223 -> 139 us at 8192 images). (conv3 as NT 4, NTW 2, KH 4 -- a quarter of the 36 k-steps per
// wave -- measured slower than the per-image kernel: see conv_direct.) Row tiles RP at a time. The next image's input is loaded into registers while the current one is
// computed, then staged as bf16 hi / lo planes over the 13x13 zero-bordered grid (the layout,
// fragments, x3 products and epilogue of conv3x3_x3_kernel).
template <int CP, int NT, int NTW, int KH, int RP>
__global__ __launch_bounds__(512, 1) void conv3x3_wreg_kernel(evx_gemm_desc g, int cin, const __bf16* __restrict__ wp,
                                                              int nimg, int nslot) {
    static_assert(CP == 32 || CP == 64, "conv2 / conv3 inputs");
    constexpr int XP = CP + 8, KJ = CP / 16, KS = 9 * KJ, KW = KS / KH, WPT = 8 / NTW, RW = 4 * KH / WPT;
    constexpr int CG = NT / NTW;
    static_assert(KS % KH == 0 && WPT % KH == 0 && RW * (WPT / KH) == 4 && RW % RP == 0 && NT % NTW == 0, "split");
    constexpr int C4 = CP / 4, NI = 169 * C4, NPF = (NI + 511) / 512;  // float4 staging pieces per thread
    __shared__ __attribute__((aligned(16))) __bf16 Xs[2][169][XP];
    __shared__ __attribute__((aligned(16))) float Red[KH > 1 ? (KH - 1) * NTW * RP * 32 * 32 : 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    // workgroup -> (column group, image slot): the CG groups of a slot 8 workgroups apart (one XCD)
    const int b = (int)blockIdx.x;
    int cg, slot;
    if (CG > 1 && (gridDim.x & (8 * CG - 1)) == 0) {
        cg = (b >> 3) % CG;
        slot = (b & 7) + ((b >> 3) / CG) * 8;
    } else {
        cg = b % CG;
        slot = b / CG;
    }
    const int ctl = w % NTW, ct = cg * NTW + ctl, g2 = w / NTW, kh = g2 % KH, rt0 = (g2 / KH) * RW;
    const int n = ct * 32 + (lane & 31);
    bf16x8 wh[KW], wl[KW];
#pragma unroll
    for (int j = 0; j < KW; j++) {
        const size_t o = ((size_t)(ct * KS + kh * KW + j) * 64 + lane) * 8;
        wh[j] = *reinterpret_cast<const bf16x8*>(wp + o);
        wl[j] = *reinterpret_cast<const bf16x8*>(wp + o + (size_t)NT * KS * 512);
    }
    int base[RW];
#pragma unroll
    for (int k = 0; k < RW; k++) {
        int m = (rt0 + k) * 32 + (lane & 31);
        m = m < 121 ? m : 0;  // rows 121.. read pixel 0 (their outputs are not stored)
        const int y = (m * 187) >> 11, x = m - 11 * y;
        base[k] = (y + 1) * 13 + (x + 1);
    }
    auto opaque = [](int v) {  // hides the image index from loop strength reduction
        asm volatile("" : "+s"(v));
        return v;
    };
    auto opaque_v = [](int v) {  // per-thread staging offsets: recomputed per image, not held live
        asm volatile("" : "+v"(v));
        return v;
    };
    // 32-bit element offsets from a wave-uniform image base (64-bit pointers per piece and per output
    // row, strength-reduced across the image loop, took 80 VGPRs and spilled the weights)
    float4 pf[NPF];
    auto load = [&](int img) {
        const float* __restrict__ X = g.A + (size_t)opaque(img) * 121 * cin;
        const int tv = opaque_v(tid);
#pragma unroll
        for (int t = 0; t < NPF; t++) {
            const int i = tv + 512 * t, q = i / C4, c = (i - q * C4) * 4;
            const int y = q / 13 - 1, x = q - (q / 13) * 13 - 1;
            pf[t] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (i < NI && (unsigned)y < 11u && (unsigned)x < 11u)
                pf[t] = *reinterpret_cast<const float4*>(X + (uint32_t)((y * 11 + x) * cin + c));
        }
    };
    auto store = [&]() {
        const int tv = opaque_v(tid);
#pragma unroll
        for (int t = 0; t < NPF; t++) {
            const int i = tv + 512 * t, q = i / C4, c = (i - q * C4) * 4;
            if (i < NI) {
                const float f[4] = {pf[t].x, pf[t].y, pf[t].z, pf[t].w};
                bf16x4 hi, lo;
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const __bf16 v = (__bf16)f[e];
                    hi[e] = v;
                    lo[e] = (__bf16)(f[e] - (float)v);
                }
                *reinterpret_cast<bf16x4*>(&Xs[0][q][c]) = hi;
                *reinterpret_cast<bf16x4*>(&Xs[1][q][c]) = lo;
            }
        }
    };
    const float bias = g.bias ? g.bias[n] : 0.f;
    const bool relu = (g.flags & EVX_GEMM_RELU) != 0;
    const bool osp = (g.flags & EVX_GEMM_OUT_SPLIT) != 0;
    const size_t ylo = (size_t)g.M * g.ldc;
    const uint32_t ldc = (uint32_t)g.ldc;
    int img = slot;
    if (img < nimg) load(img);
    for (; img < nimg; img += nslot) {
        __syncthreads();  // the previous image's fragments and partials have been read
        store();
        __syncthreads();
        if (img + nslot < nimg) load(img + nslot);  // in flight during the MFMAs
        const size_t ib = (size_t)opaque(img) * 121 * g.ldc;
        float* __restrict__ Y = g.C + ib;
        __bf16* __restrict__ Yh = reinterpret_cast<__bf16*>(g.C) + ib;
        __bf16* __restrict__ Yl = Yh + ylo;
#pragma unroll
        for (int p0 = 0; p0 < RW; p0 += RP) {
            f32x16 acc[RP];
#pragma unroll
            for (int k = 0; k < RP; k++)
#pragma unroll
                for (int r = 0; r < 16; r++) acc[k][r] = 0.f;
            // the K part as a compile-time constant: each k-step's tap and channel offset fold into
            // the LDS reads' immediate offsets (a runtime part kept its addresses live and spilled)
            auto ksteps = [&](auto khc) {
                constexpr int KHC = decltype(khc)::value;
#pragma unroll
                for (int j = 0; j < KW; j++) {
                    asm volatile("" ::: "memory");  // one k-step's fragment reads at a time
                    const int ks = KHC * KW + j, tap = ks / KJ, cj = (ks - tap * KJ) * 16;
                    const int toff = (tap / 3 - 1) * 13 + (tap % 3 - 1);
#pragma unroll
                    for (int k = 0; k < RP; k++) {
                        const __bf16* x0 = &Xs[0][base[p0 + k]][8 * h] + toff * XP + cj;
                        const __bf16* x1 = &Xs[1][base[p0 + k]][8 * h] + toff * XP + cj;
                        const bf16x8 ah = *reinterpret_cast<const bf16x8*>(x0);
                        const bf16x8 al = *reinterpret_cast<const bf16x8*>(x1);
                        acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, wh[j], acc[k], 0, 0, 0);
                        acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, wl[j], acc[k], 0, 0, 0);
                        acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, wh[j], acc[k], 0, 0, 0);
                    }
                }
            };
            if constexpr (KH == 1) {
                ksteps(std::integral_constant<int, 0>());
            } else {
                switch (kh) {
                    case 0: ksteps(std::integral_constant<int, 0>()); break;
                    case 1: ksteps(std::integral_constant<int, 1 % KH>()); break;
                    case 2: ksteps(std::integral_constant<int, 2 % KH>()); break;
                    default: ksteps(std::integral_constant<int, 3 % KH>()); break;
                }
                // the other K parts' partials through LDS, added by part 0 in part order
                float* red = Red + (size_t)(kh - 1) * NTW * RP * 1024 + ctl * RP * 1024;
                if (kh > 0) {
#pragma unroll
                    for (int k = 0; k < RP; k++)
#pragma unroll
                        for (int r = 0; r < 16; r++)
                            red[(k * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 32 + (lane & 31)] = acc[k][r];
                }
                __syncthreads();
                if (kh == 0) {
#pragma unroll
                    for (int q = 0; q < KH - 1; q++) {
                        const float* rq = Red + (size_t)q * NTW * RP * 1024 + ctl * RP * 1024;
#pragma unroll
                        for (int k = 0; k < RP; k++)
#pragma unroll
                            for (int r = 0; r < 16; r++)
                                acc[k][r] += rq[(k * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 32 + (lane & 31)];
                    }
                }
                __syncthreads();  // Red is rewritten by the next pass
                if (kh != 0) continue;
            }
#pragma unroll
            for (int k = 0; k < RP; k++) {
                const int mb = opaque_v((rt0 + p0 + k) * 32 + 4 * h);  // output offsets not held live
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int m = mb + (r & 3) + 8 * (r >> 2);
                    if (m >= 121) continue;
                    const uint32_t o = (uint32_t)m * ldc + (uint32_t)n;
                    float v = acc[k][r] + bias;
                    if (relu) v = v > 0.f ? v : 0.f;
                    if (osp) {
                        const __bf16 hi = (__bf16)v;
                        Yh[o] = hi;
                        Yl[o] = (__bf16)(v - (float)hi);
                    } else {
                        Y[o] = v;
                    }
                }
            }
        }
    }
}
}  // namespace evxq
namespace {

// The LDS-staged conv kernels (conv3x3_x3_kernel) apply to plain calls -- forward: bias / ReLU
// epilogue and the torch weight layout; dX: the ReLU gate -- over cfg4's layer shapes; CP of the
// staged channels (0: not applicable). Their packed weights need conv_direct_ws floats of workspace.
static int conv_direct_cp(const evx_gemm_desc* g, int mode, int cs) {
    if (g->mask || (g->flags & EVX_GEMM_ACCUM) || g->alpha != 1.f || g->ldc != g->N || g->M % 121 != 0) return 0;
    if (mode == EVX_CONV_FWD) {
        if (g->gate || g->sbk != 9 || g->sbn != 9 * cs) return 0;
        if (cs <= 16 && g->N == 32) return 16;
        if (cs == 32 && g->N == 64) return 32;
        if (cs == 64 && g->N == 128) return 64;
    } else if (mode == EVX_CONV_DX) {
        if (g->bias || (g->flags & EVX_GEMM_RELU) || g->sbn != 9 || g->sbk != 9 * (int64_t)g->N) return 0;
        if (cs == 64 && g->N == 32) return 64;
        if (cs == 128 && g->N == 64) return 128;
    }
    return 0;
}
static int64_t conv_direct_ws(const evx_gemm_desc* g, int mode, int cs) {
    const int cp = conv_direct_cp(g, mode, cs);
    return cp ? (int64_t)(g->N / 32) * (9 * cp / 16) * 512 : 0;
}
template <int CP, int NT, bool DX>
static void conv_direct_launch(const evx_gemm_desc* g, int cs, __bf16* wp, hipStream_t st) {
    const unsigned pb = (unsigned)((NT * (9 * CP / 16) * 64 + 255) / 256);
    hipLaunchKernelGGL(evxq::conv_wpack_kernel<CP>, dim3(pb), dim3(256), 0, st, g->B, g->sbk, g->sbn, cs, NT, wp);
    hipLaunchKernelGGL((evxq::conv3x3_x3_kernel<CP, NT, DX>), dim3((unsigned)(g->M / 121)), dim3(256), 0, st, *g, cs,
                       (const __bf16*)wp);
}
// conv2 forward with the weights in registers (conv3x3_wreg_kernel): one workgroup per CU
template <int CP, int NT, int NTW, int KH, int RP>
static void conv_wreg_launch(const evx_gemm_desc* g, int cs, __bf16* wp, hipStream_t st) {
    const unsigned pb = (unsigned)((NT * (9 * CP / 16) * 64 + 255) / 256);
    hipLaunchKernelGGL(evxq::conv_wpack_kernel<CP>, dim3(pb), dim3(256), 0, st, g->B, g->sbk, g->sbn, cs, NT, wp);
    constexpr int CG = NT / NTW;
    const int nimg = (int)(g->M / 121);
    int nslot = std::min(nimg, evxh::cu_count() / CG);
    if (nslot >= 8) nslot &= ~7;  // whole XCD rounds (the column groups of a slot share one)
    hipLaunchKernelGGL((evxq::conv3x3_wreg_kernel<CP, NT, NTW, KH, RP>), dim3((unsigned)(nslot * CG)), dim3(512), 0, st,
                       *g, cs, (const __bf16*)wp, nimg, nslot);
}
static bool conv_direct(const evx_gemm_desc* g, int mode, int cs, hipStream_t st) {
    const int cp = conv_direct_cp(g, mode, cs);
    if (!cp || !g->ws || g->ws_elems < conv_direct_ws(g, mode, cs)) return false;
    __bf16* wp = reinterpret_cast<__bf16*>(g->ws);
    if (mode == EVX_CONV_FWD) {
        if (cp == 16) conv_direct_launch<16, 1, false>(g, cs, wp, st);
        else if (cp == 32) conv_wreg_launch<32, 2, 2, 1, 1>(g, cs, wp, st);
        // conv3 keeps the per-image kernel: with its 36 k-steps of weights split over four waves
        // (conv3x3_wreg_kernel<64, 4, 2, 4, 2>, 254 VGPRs) the K-part reductions and their barriers
        // per image cost more than the weight re-reads saved (act 654 -> ~1000 us, learn 88 -> 130 us)
        else conv_direct_launch<64, 4, false>(g, cs, wp, st);
    } else {
        if (cp == 64) conv_direct_launch<64, 1, true>(g, cs, wp, st);
        else conv_direct_launch<128, 2, true>(g, cs, wp, st);
    }
    return true;
}

// tn3_kernel's cases: x3, alpha 1, B n-contiguous (sbn 1) or the conv dW gather (channels a multiple
// of 4, no epilogue), A m- or k-contiguous, row strides and widths multiples of 4, 16-B aligned
// returns 0 (not this kernel's case), 1 (A k-major: A[k][m], sam 1) or 2 (A k-contiguous: A[m][k], sak 1;
// plain B only)
static int tn3_ok(const evx_gemm_desc* g, int cm, int cs) {
    if (g->precision != EVX_PREC_X3 || (g->flags & ~(EVX_GEMM_RELU | EVX_GEMM_ACCUM)) || g->alpha != 1.f) return 0;
    if (cm == evxq::CV_DW && (g->bias || g->mask || g->gate || g->flags)) return 0;
    auto al16 = [](const float* p) { return ((uintptr_t)p & 15) == 0; };
    if (!al16(g->A) || !al16(g->B) || g->K < 256) return 0;
    const bool bplain = cm == evxq::CV_NONE && g->sbn == 1 && (g->sbk & 3) == 0 && (g->N & 3) == 0;
    if (g->sam == 1 && (g->sak & 3) == 0 && (g->M & 3) == 0) {
        if (cm == evxq::CV_DW) return (cs & 3) == 0 && g->N == 9 * cs ? 1 : 0;
        return bplain ? 1 : 0;
    }
    if (g->sak == 1 && (g->sam & 3) == 0 && (g->K & 3) == 0 && bplain) return 2;
    return 0;
}
int gemm_launch(const evx_gemm_desc* g, int cm, int cs, void* stream) {
    if (!g || !g->A || !g->B || !g->C) return qfail(-22, "gemm: NULL operand");
    if (g->M <= 0 || g->N <= 0 || g->K <= 0) return 0;
    if (g->ws_elems < 0) return qfail(-22, "gemm: ws_elems < 0");
    const int TB = evxq::TB;
    int klen = 0;
    const int S = gemm_slices(g, g->ws ? g->ws_elems : 0, &klen);
    dim3 grid((unsigned)((g->N + TB - 1) / TB), (unsigned)((g->M + TB - 1) / TB), (unsigned)S);
    if (grid.y > 65535u) return qfail(-22, "gemm: M too large for one launch");
    hipStream_t st = (hipStream_t)stream;
    if ((cm == evxq::CV_FWD || cm == evxq::CV_DX) && S == 1 && conv_direct(g, cm, cs, st)) return qlaunch("conv3x3");
    if (g->flags & EVX_GEMM_OUT_SPLIT) return qfail(-22, "gemm: OUT_SPLIT needs the LDS-staged conv forward (and its workspace)");
    if (const int tk = tn3_ok(g, cm, cs)) {  // B k-major (weight gradients: fc and conv dW; activation gradients)
        {
            static std::atomic<uint64_t> attr_done;
            const void* ks[3] = {(const void*)evxq::tn3_kernel<false>, (const void*)evxq::tn3_kernel<true>,
                                 (const void*)evxq::tn3_kernel<false, true>};
            evxh::max_lds_once(attr_done, ks, 3, evxq::TN3_LDS);
        }
        const dim3 tg = grid;
        if (tk == 2)
            hipLaunchKernelGGL((evxq::tn3_kernel<false, true>), tg, dim3(256), evxq::TN3_LDS, st, *g, klen, cs);
        else if (cm == evxq::CV_DW)
            hipLaunchKernelGGL(evxq::tn3_kernel<true>, tg, dim3(256), evxq::TN3_LDS, st, *g, klen, cs);
        else
            hipLaunchKernelGGL(evxq::tn3_kernel<false>, tg, dim3(256), evxq::TN3_LDS, st, *g, klen, cs);
    } else
    if (g->flags & EVX_GEMM_SPLIT_AB) {
        if (cm != evxq::CV_NONE || g->precision != EVX_PREC_X3 || g->sak != 1 || g->sbk != 1 || (g->K & 7) ||
            (g->sam & 7) || (g->sbn & 7))
            return qfail(-22, "gemm: SPLIT_AB needs x3, k-contiguous operands, K and row strides multiples of 8");
        hipLaunchKernelGGL((evxq::gemm128x3_kernel<evxq::CV_NONE, true>), grid, dim3(256), 0, st, *g, klen, 0);
    } else
    if (cm == evxq::CV_FWD)
        hipLaunchKernelGGL(evxq::gemm128x3_kernel<evxq::CV_FWD>, grid, dim3(256), 0, st, *g, klen, cs);
    else if (cm == evxq::CV_DX)
        hipLaunchKernelGGL(evxq::gemm128x3_kernel<evxq::CV_DX>, grid, dim3(256), 0, st, *g, klen, cs);
    else if (cm == evxq::CV_DW)
        hipLaunchKernelGGL(evxq::gemm128x3_kernel<evxq::CV_DW>, grid, dim3(256), 0, st, *g, klen, cs);
    else if (g->precision == EVX_PREC_BF16)
        hipLaunchKernelGGL(evxq::gemm128_kernel<__bf16>, grid, dim3(256), 0, st, *g, klen);
    else if (g->precision == EVX_PREC_X3) {
        // k-contiguous f32 operands staged from 16-B loads (the fc layers' forward: A and B; dX: A)
        auto al16 = [](const float* p) { return ((uintptr_t)p & 15) == 0; };
        const bool ak = g->sak == 1 && (g->sam & 3) == 0 && (g->K & 3) == 0 && al16(g->A);
        const bool bk = g->sbk == 1 && (g->sbn & 3) == 0 && (g->K & 3) == 0 && al16(g->B);
        if (ak && bk)
            hipLaunchKernelGGL((evxq::gemm128x3_kernel<evxq::CV_NONE, false, evxq::VA_K | evxq::VB_K>), grid, dim3(256), 0,
                               st, *g, klen, 0);
        else if (ak)
            hipLaunchKernelGGL((evxq::gemm128x3_kernel<evxq::CV_NONE, false, evxq::VA_K>), grid, dim3(256), 0, st, *g,
                               klen, 0);
        else if (bk)
            hipLaunchKernelGGL((evxq::gemm128x3_kernel<evxq::CV_NONE, false, evxq::VB_K>), grid, dim3(256), 0, st, *g,
                               klen, 0);
        else
            hipLaunchKernelGGL(evxq::gemm128x3_kernel<evxq::CV_NONE>, grid, dim3(256), 0, st, *g, klen, 0);
    }
    else
        hipLaunchKernelGGL(evxq::gemm128_kernel<float>, grid, dim3(256), 0, st, *g, klen);
    if (S > 1) {  // the slices' partials summed in slice order, then the epilogue
        const int e = qlaunch("gemm");
        if (e) return e;
        const int64_t MN = (int64_t)g->M * g->N;
        if (S >= 8 && (MN & 3) == 0)
            hipLaunchKernelGGL(evxq::splitk_reduce4_kernel, dim3((unsigned)((MN / 4 + 63) / 64)), dim3(256), 0, st, *g, S);
        else
            hipLaunchKernelGGL(evxq::splitk_reduce_kernel, dim3(nblk((MN + 3) / 4)), dim3(256), 0, st, *g, S);
    }
    return qlaunch("gemm");
}
}  // namespace

extern "C" {

int evx_gemm(const evx_gemm_desc* g, void* stream) { return gemm_launch(g, evxq::CV_NONE, 0, stream); }

int64_t evx_gemm_ws_elems(const evx_gemm_desc* g) {
    if (!g || g->M <= 0 || g->N <= 0 || g->K <= 0) return 0;
    const int S = gemm_slices(g, INT64_MAX, nullptr);
    return S > 1 ? (int64_t)S * g->M * g->N : 0;
}

int64_t evx_conv3x3_ws_elems(const evx_gemm_desc* g, int32_t mode, int32_t cs) {
    if (!g || g->M <= 0 || g->N <= 0 || g->K <= 0 || cs <= 0) return 0;
    if (g->precision == EVX_PREC_X3) {
        const int64_t w = conv_direct_ws(g, mode, cs);
        if (w > 0) return w;
    }
    return evx_gemm_ws_elems(g);
}

int evx_conv3x3_gemm(const evx_gemm_desc* g, int32_t mode, int32_t cs, void* stream) {
    if (!g) return qfail(-22, "conv3x3: NULL descriptor");
    if (g->precision != EVX_PREC_X3) return qfail(-22, "conv3x3: implicit-GEMM convolution is x3 only");
    if (mode < EVX_CONV_FWD || mode > EVX_CONV_DW) return qfail(-22, "conv3x3: bad mode");
    if (cs <= 0) return qfail(-22, "conv3x3: channels <= 0");
    const int64_t pix = mode == EVX_CONV_DW ? g->K : g->M;  // rows of the pixel-major activations
    if (pix % 121 || pix >= (1LL << 26)) return qfail(-22, "conv3x3: pixel count not 121*B (< 2^26)");
    if ((mode == EVX_CONV_DW ? g->N : g->K) != 9 * cs) return qfail(-22, "conv3x3: 3x3 taps x channels mismatch");
    if (mode == EVX_CONV_DW && (g->sam != 1 || g->sak != g->M))
        return qfail(-22, "conv3x3 dW: A must be dY [pixels][M]");
    return gemm_launch(g, mode, cs, stream);
}

int evx_colsum(const float* X, int64_t ld, int32_t M, int32_t N, float* out, int32_t accum, float* scratch,
               int32_t scratch_elems, void* stream) {
    if (M <= 0 || N <= 0) return 0;
    int chunks = (M + evxq::COLSUM_ROWS - 1) / evxq::COLSUM_ROWS;
    if ((int64_t)chunks * N > scratch_elems) chunks = scratch_elems / N;
    if (chunks < 1) return qfail(-22, "colsum: scratch too small");
    hipLaunchKernelGGL(evxq::colsum_kernel, dim3((unsigned)((N + 63) / 64), (unsigned)((chunks + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, X, ld, M, N, scratch, chunks);
    hipLaunchKernelGGL(evxq::colsum_finish, dim3((unsigned)N), dim3(256), 0, (hipStream_t)stream, scratch, N, chunks,
                       out, accum);
    return qlaunch("colsum");
}

int64_t evx_td_loss_ws_floats(int32_t B, int32_t nets) {
    if (B <= 0 || nets < 1) return 0;
    return (int64_t)((B + 255) / 256) * nets;
}

static int td_launch(const float* Q, const float* Qt, int32_t A, const int32_t* act, const float* rew,
                     const uint8_t* done, float gamma, int32_t B, int32_t nets, const float* w, float* dQ, float* loss,
                     float* td_abs, float* zero, int64_t nzero, float* ws, int64_t ws_floats, void* stream,
                     const char* what) {
    if (B <= 0) return 0;
    if (nets < 1 || nets > 65535) return qfail(-22, "td_loss: nets must be 1..65535");
    if (!Q || !Qt || !act || !rew || !done || !dQ || !loss) return qfail(-22, "td_loss: NULL argument");
    const int ntd = (B + 255) / 256;
    if (!ws || ws_floats < (int64_t)ntd * nets) return qfail(-22, "td_loss: workspace smaller than evx_td_loss_ws_floats");
    const int nz = zero && nzero > 0 ? (int)std::min<int64_t>((nzero + 256 * 16 - 1) / (256 * 16), 512) : 0;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(evxq::td_loss_kernel, dim3(ntd + nz, nets), dim3(256), 0, st, Q, Qt, A, act, rew, done, gamma, B,
                       w, dQ, ws, td_abs, ntd, nz ? zero : nullptr, nzero);
    hipLaunchKernelGGL(evxq::td_finish_kernel, dim3(nets), dim3(256), 0, st, (const float*)ws, ntd, B, loss);
    return qlaunch(what);
}

int evx_td_loss_w(const float* Q, const float* Qt, int32_t A, const int32_t* act, const float* rew,
                  const uint8_t* done, float gamma, int32_t B, const float* w, float* dQ, float* loss, float* td_abs,
                  float* ws, int64_t ws_floats, void* stream) {
    return td_launch(Q, Qt, A, act, rew, done, gamma, B, 1, w, dQ, loss, td_abs, nullptr, 0, ws, ws_floats, stream,
                     "td_loss");
}

int evx_td_loss_zero(const float* Q, const float* Qt, int32_t A, const int32_t* act, const float* rew,
                     const uint8_t* done, float gamma, int32_t B, const float* w, float* dQ, float* loss, float* td_abs,
                     float* zero, int64_t nzero, float* ws, int64_t ws_floats, void* stream) {
    return td_launch(Q, Qt, A, act, rew, done, gamma, B, 1, w, dQ, loss, td_abs, zero, nzero, ws, ws_floats, stream,
                     "td_loss_zero");
}

int evx_td_loss_zero_g(const float* Q, const float* Qt, int32_t A, const int32_t* act, const float* rew,
                       const uint8_t* done, float gamma, int32_t B, int32_t nets, const float* w, float* dQ, float* loss,
                       float* td_abs, float* zero, int64_t nzero, float* ws, int64_t ws_floats, void* stream) {
    return td_launch(Q, Qt, A, act, rew, done, gamma, B, nets, w, dQ, loss, td_abs, zero, nzero, ws, ws_floats, stream,
                     "td_loss_zero_g");
}

int evx_td_loss(const float* Q, const float* Qt, int32_t A, const int32_t* act, const float* rew, const uint8_t* done,
                float gamma, int32_t B, float* dQ, float* loss, float* ws, int64_t ws_floats, void* stream) {
    return evx_td_loss_w(Q, Qt, A, act, rew, done, gamma, B, nullptr, dQ, loss, nullptr, ws, ws_floats, stream);
}

int evx_sumsq_norm(const float* g, int64_t n, float* scratch, int32_t scratch_elems, float* norm, void* stream) {
    int parts = (int)((n + 4095) / 4096);
    if (parts > scratch_elems) parts = scratch_elems;
    if (parts > 2048) parts = 2048;
    if (parts < 1) parts = 1;
    hipLaunchKernelGGL(evxq::sumsq_kernel, dim3(parts), dim3(256), 0, (hipStream_t)stream, g, n, scratch);
    hipLaunchKernelGGL(evxq::sumsq_finish, dim3(1), dim3(256), 0, (hipStream_t)stream, scratch, parts, norm);
    return qlaunch("sumsq");
}

int evx_clip_adam(float* p, float* g, float* m, float* v, int64_t n, const float* norm, float max_norm,
                  const evx_adam* h, void* stream) {
    if (!h) return qfail(-22, "adam: NULL hyper-parameters");
    if (n <= 0) return 0;
    const double bc1 = 1.0 - pow((double)h->beta1, (double)h->step);
    const double bc2 = 1.0 - pow((double)h->beta2, (double)h->step);
    const float step_size = (float)(h->lr / bc1);
    const float bc2_sqrt = (float)sqrt(bc2);
    unsigned blocks = nblk(n);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(evxq::clip_adam_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, norm,
                       max_norm, h->lr, h->beta1, h->beta2, h->eps, step_size, bc2_sqrt, h->weight_decay);
    return qlaunch("clip_adam");
}

int evx_dropout_mask(uint8_t* mask, int64_t n, float p, uint64_t seed, uint64_t offset, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(evxq::dropout_mask_kernel, dim3(nblk((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, mask, n,
                       p, seed, offset);
    return qlaunch("dropout_mask");
}

int evx_act(const float* Q, int32_t n, int32_t A, float epsilon, uint64_t seed, uint64_t offset, int32_t* actions,
            void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(evxq::act_kernel, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, Q, n, A, epsilon, seed,
                       offset, actions);
    return qlaunch("act");
}

int evx_replay_push(const evx_replay* rp, const evx_obs* s, const evx_obs* s2, const int32_t* a, const double* r_env,
                    const uint8_t* done_env, int32_t n, int32_t agents_per_env, int64_t pos, void* stream) {
    if (!rp || rp->capacity <= 0) return qfail(-22, "replay: bad ring");
    if (n <= 0) return 0;
    hipLaunchKernelGGL(evxq::replay_push_kernel, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, *rp, s, s2,
                       (const evx_obs*)nullptr, a, r_env, done_env, n, agents_per_env, pos);
    return qlaunch("replay_push");
}

int evx_replay_push_term(const evx_replay* rp, const evx_obs* s, const evx_obs* s2, const evx_obs* s2_term,
                         const int32_t* a, const double* r_env, const uint8_t* done_env, int32_t n,
                         int32_t agents_per_env, int64_t pos, void* stream) {
    if (!rp || rp->capacity <= 0) return qfail(-22, "replay: bad ring");
    if (n <= 0) return 0;
    hipLaunchKernelGGL(evxq::replay_push_kernel, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, *rp, s, s2, s2_term,
                       a, r_env, done_env, n, agents_per_env, pos);
    return qlaunch("replay_push_term");
}

int evx_replay_sample(const evx_replay* rp, int64_t size, int32_t B, uint64_t seed, uint64_t offset, evx_obs* s,
                      evx_obs* s2, int32_t* a, float* r, uint8_t* done, int64_t* idx_out, void* stream) {
    if (!rp || size <= 0) return qfail(-22, "replay: empty");
    if (B <= 0) return 0;
    if (size > rp->capacity) return qfail(-22, "replay: size > capacity");
    if (B > size) return qfail(-22, "replay: sample larger than population (random.sample)");
    hipLaunchKernelGGL(evxq::replay_sample_kernel, dim3(nblk(B)), dim3(256), 0, (hipStream_t)stream, *rp, (int64_t)0,
                       size, B, seed, offset, s, s2, a, r, done, idx_out);
    return qlaunch("replay_sample");
}

int evx_replay_sample_agents(const evx_replay* rp, int64_t size, int32_t B, int32_t nets, uint64_t seed,
                             uint64_t offset, evx_obs* s, evx_obs* s2, int32_t* a, float* r, uint8_t* done,
                             void* stream) {
    if (!rp || !s || !s2 || !a || !r || !done) return qfail(-22, "replay_sample_agents: NULL argument");
    if (B <= 0) return 0;
    if (nets < 1 || nets > 65535) return qfail(-22, "replay_sample_agents: nets must be 1..65535");
    if (rp->capacity % nets) return qfail(-22, "replay_sample_agents: capacity must be a multiple of nets");
    if (size < nets || size > rp->capacity || size % nets)
        return qfail(-22, "replay_sample_agents: size must be a positive multiple of nets within the capacity");
    if (B > size / nets) return qfail(-22, "replay_sample_agents: sample larger than an agent's population");
    hipLaunchKernelGGL(evxq::replay_sample_kernel, dim3(nblk(B), nets), dim3(256), 0, (hipStream_t)stream, *rp, (int64_t)0,
                       size, B, seed, offset, s, s2, a, r, done, nullptr, (int)nets);
    return qlaunch("replay_sample_agents");
}

int evx_replay_sample_joint(const evx_replay* rp, int64_t size, int32_t B, int32_t nets, uint64_t seed,
                            uint64_t offset, evx_obs* s, evx_obs* s2, int32_t* a, float* r, uint8_t* done,
                            void* stream) {
    if (!rp || !s || !s2 || !a || !r || !done) return qfail(-22, "replay_sample_joint: NULL argument");
    if (B <= 0) return 0;
    if (nets < 1 || nets > 65535) return qfail(-22, "replay_sample_joint: nets must be 1..65535");
    if (rp->capacity % nets) return qfail(-22, "replay_sample_joint: capacity must be a multiple of nets");
    if (size < nets || size > rp->capacity || size % nets)
        return qfail(-22, "replay_sample_joint: size must be a positive multiple of nets within the capacity");
    if (B > size / nets) return qfail(-22, "replay_sample_joint: sample larger than the population");
    hipLaunchKernelGGL(evxq::replay_sample_kernel, dim3(nblk(B), nets), dim3(256), 0, (hipStream_t)stream, *rp, (int64_t)0,
                       size, B, seed, offset, s, s2, a, r, done, nullptr, (int)nets, 1);
    return qlaunch("replay_sample_joint");
}

int evx_replay_sample_window(const evx_replay* rp, int64_t base, int64_t count, int32_t B, uint64_t seed,
                             uint64_t offset, evx_obs* s, evx_obs* s2, int32_t* a, float* r, uint8_t* done,
                             int64_t* idx_out, void* stream) {
    if (!rp || count <= 0) return qfail(-22, "replay: empty window");
    if (count > rp->capacity || base < 0 || base >= rp->capacity) return qfail(-22, "replay: bad window");
    if (B <= 0) return 0;
    if (B > count) return qfail(-22, "replay: sample larger than the window (random.sample)");
    hipLaunchKernelGGL(evxq::replay_sample_kernel, dim3(nblk(B)), dim3(256), 0, (hipStream_t)stream, *rp, base, count,
                       B, seed, offset, s, s2, a, r, done, idx_out);
    return qlaunch("replay_sample_window");
}

int evx_gather_obs(const evx_obs* src, const int64_t* idx, int32_t n, evx_obs* dst, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(evxq::gather_rows_kernel, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, src, idx, n, dst);
    return qlaunch("gather_obs");
}

int evx_im2col3x3(const float* x, int32_t B, int32_t C, int32_t nhwc, float* cols, void* stream) {
    const int64_t total = (int64_t)B * 121 * C * 9;
    if (total <= 0) return 0;
    hipLaunchKernelGGL(evxq::im2col_kernel, dim3(nblk(total)), dim3(256), 0, (hipStream_t)stream, x, B, C, nhwc, cols);
    return qlaunch("im2col");
}

int evx_col2im3x3(const float* dcols, int32_t B, int32_t C, float* dx, void* stream) {
    const int64_t total = (int64_t)B * C * 121;
    if (total <= 0) return 0;
    hipLaunchKernelGGL(evxq::col2im_kernel, dim3(nblk(total)), dim3(256), 0, (hipStream_t)stream, dcols, B, C, dx);
    return qlaunch("col2im");
}

int evx_relu_grad(float* dy, const float* y, int64_t n, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(evxq::relu_grad_kernel, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, dy, y, n);
    return qlaunch("relu_grad");
}

int evx_pix_split(const float* src, int32_t B, int32_t C, uint16_t* dst, void* stream) {
    if (B <= 0 || C <= 0) return 0;
    const size_t lds = (size_t)121 * (C + 1) * 4;
    if (lds > 64 * 1024) return qfail(-22, "pix_split: C > 134 channels");
    hipLaunchKernelGGL(evxq::pix_split_kernel, dim3((unsigned)B), dim3(256), lds, (hipStream_t)stream, src, B, C,
                       reinterpret_cast<__bf16*>(dst));
    return qlaunch("pix_split");
}

int evx_pix_nchw(const float* src, int32_t B, int32_t C, int32_t to_nchw, float* dst, void* stream) {
    const int64_t total = (int64_t)B * C * 121;
    if (total <= 0) return 0;
    const size_t lds = (size_t)121 * (C + 1) * 4;
    if (lds > 64 * 1024) {  // the LDS tile holds C <= 134: element-wise beyond
        hipLaunchKernelGGL(evxq::pix2nchw_flat_kernel, dim3(nblk(total)), dim3(256), 0, (hipStream_t)stream, src, total,
                           C, to_nchw, dst);
        return qlaunch("pix_nchw");
    }
    hipLaunchKernelGGL(evxq::pix2nchw_kernel, dim3((unsigned)B), dim3(256), lds, (hipStream_t)stream, src, B, C, to_nchw,
                       dst);
    return qlaunch("pix_nchw");
}

}  // extern "C"
