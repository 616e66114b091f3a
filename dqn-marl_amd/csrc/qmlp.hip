// MI355X (gfx950) fast path of the MLP Q-network (726 -> 512 -> 256 -> 5) on bf16 MFMA.
//
// Reference: Louvre_Evacuation/agents/dqn_agent.py DQNNetwork.forward (:40-61, the
// fc stack; the MLP variant of SURVEY §8a A19 feeds it the flattened 11x11x6
// patch) and DQNAgent.act (:101-124). The observation tensor of
// EvacuationEnv._get_state (envs/evacuation_env.py:84-120) is never materialised:
// fc1's A operand is generated from the 32-B compact observation straight into
// the LDS tile the MFMAs read (the expanded input would be 190 MB per act step).
//
//   qfc1_kernel : H1 = dropout(relu(X W1^T + b1)) -> bf16 [N][512]; X optionally
//                 written out as bf16 [N][736] (the learner's dW1 operand)
//   qfc23_kernel: H2 = relu(H1 W2^T + b2) (optionally saved, f32), Q = H2 W3^T + b3,
//                 optionally the epsilon-greedy action (evx_act's rule and RNG)
//
// Tiles: a workgroup owns 64 rows; its 4 waves split the output columns. Weights
// (L2-resident, bf16, K padded to a multiple of 32) go from global memory straight
// into the MFMA B-operand registers, one K-chunk ahead; A chunks are double
// buffered in LDS, one barrier per chunk. v_mfma_f32_32x32x16_bf16 operand map:
// lane l supplies A[row l&31][k 8(l>>5)..+7] and B[k 8(l>>5)..+7][col l&31];
// C/D: col = l&31, row = (r&3) + 8(r>>2) + 4(l>>5).
//
// Dropout keep bits are a counter-based hash of (seed, stream, row pair, col), 16 bits
// per element; the backward pass reads the mask back as [H1 > 0] instead of storing it.
//
// X3 (f32-accurate) mode, the reference's fp32 arithmetic on the bf16 matrix cores: an f32
// operand v is carried as hi = bf16(v) and lo = bf16(v - hi) (16 significant bits) and a
// product as hi*hi + hi*lo + lo*hi (relative error ~2^-16 per product, f32 accumulation);
// operands that are exactly 0/1 (occupancy, barrier, exit) have no lo part. fc1's K grows
// to 640: the compact 512 (hi of the danger feature) plus one slot per cell for the danger's
// lo residual (k = 512 + c), which multiplies the danger column's hi weight. Split
// activations (H1, dZ2, dZ1) are stored as two bf16 planes [2][rows][cols].
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "evacx.h"
#include "evx_host.h"

namespace evxm {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int HID = 512, HID2 = 256, NACT = 5, K1 = 726, NCELL = 121;
// fc1's compact K: 4 features per cell (occ, danger, barrier, exit = the reference's
// channels 1-4), 128 cells (>= 121 zero). Channel 0 is identically 0 (space / max(space)
// with max = inf) and channel 5 is the constant centre one-hot, folded into the bias:
// b1c = b1 + bf16(W1[:, CENTRE_COL]). 726 -> 512 contraction length, same products.
constexpr int K1P = 512, KC1 = 32, NKC1 = K1P / KC1;
constexpr int K1X = 640, NKC1X = K1X / KC1;  // X3: + the danger residual slot of every cell
constexpr int CENTRE_COL = 60 * 6 + 5;
// the flat parameter buffer (state_dict order: fc1.weight, fc1.bias, fc2.weight, fc2.bias, fc3.*)
constexpr int NPAR = HID * K1 + HID + HID2 * HID + HID2 + NACT * HID2 + NACT;
constexpr int OB1 = HID * K1, OW2 = OB1 + HID, OB2 = OW2 + HID2 * HID, OW3 = OB2 + HID2, OB3 = OW3 + NACT * HID2;
constexpr int RM = 64;  // rows per workgroup (fc23, backward)
// reference column (of the 726) of compact feature k < 4 * NCELL
__host__ __device__ __forceinline__ int ref_col(int k) { return (k >> 2) * 6 + (k & 3) + 1; }
// X3: reference column of x column k < 640 (the danger residual of cell c at 512 + c adds
// into the danger column of c), -1 for padding
__host__ __device__ __forceinline__ int ref_col3(int k) {
    return k < 4 * NCELL ? ref_col(k) : (k >= K1P && k < K1P + NCELL) ? (k - K1P) * 6 + 2 : -1;
}
// f32 -> (hi, lo) bf16 pair of the X3 mode; v - hi is exact in f32
__device__ __forceinline__ void split2(float v, __bf16& hi, __bf16& lo) {
    hi = (__bf16)v;
    lo = (__bf16)(v - (float)hi);
}

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}
// dropout keep test: Bernoulli(1 - p) per (row, col) of one mask stream
__device__ __forceinline__ uint32_t drop_row(uint32_t seed, uint32_t stream, uint32_t row) {
    return fmix32(seed ^ fmix32(stream * 0x632be5abu + 0x9e3779b9u) ^ (row * 0x9e3779b1u));
}
// one 32-bit hash per (row pair, column): the low half decides the even row, the high
// half the odd row; keep iff the 16-bit uniform >= thresh16 = floor(p * 65536)
__device__ __forceinline__ uint32_t drop_pair(uint32_t pairh, uint32_t col) {
    return fmix32(pairh ^ (col * 0x85ebca77u + 0x27d4eb2fu));
}

// Philox4x32-10, as evx_act (qnet.hip) uses it for epsilon-greedy
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
__device__ __forceinline__ float u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }

// Weights in MFMA B-operand order: the block of (32-column tile t, K-chunk kc,
// 16-wide step s) holds lane l's 8 values (column 32t + (l&31), k = kc*KC + 16s +
// 8(l>>5) .. +7) at l*8, so a wave's operand load is one contiguous 1-KB read.
__host__ __device__ __forceinline__ size_t w1_tile(int t, int kc, int s, int nkc = NKC1) {
    return ((size_t)(t * nkc + kc) * 2 + s) * 512;
}
__host__ __device__ __forceinline__ size_t w2_tile(int t, int kc, int s) {
    return ((size_t)(t * (HID / 32) + kc) * 2 + s) * 512;
}
// fc1's occupancy columns (reference channel 1 of cells 0..127, >= 121 zero), K = 128
// in 4 chunks of 32
__host__ __device__ __forceinline__ size_t w1o_tile(int t, int kc, int s) { return ((size_t)(t * 4 + kc) * 2 + s) * 512; }
// fc2.weight^T for the backward (columns = fc2 inputs, K = fc2 outputs)
__host__ __device__ __forceinline__ size_t w2t_tile(int t, int kc, int s) {
    return ((size_t)(t * (HID2 / 32) + kc) * 2 + s) * 512;
}

struct Fwd {
    int N;
    const evx_obs* obs;
    // layout (EvacuationEnv._get_state inputs)
    const uint8_t* cellinfo;
    const float* danger;
    const uint32_t* feat;  // evx_layout.obs_feat: static per-cell features, padded grid per fire step
    const uint32_t* const* feats;  // layout set: obs_feat of layout evx_obs.layout (NULL: feat)
    int L, W, ox0, oy0, OX, OY, exit_x, exit_y, t_max;
    // parameters
    const __bf16* w1;  // [512][512] compact K, w1_tile order
    const float* b1;   // b1c: fc1.bias with the centre channel folded in
    const __bf16* w2;  // [256][512] in w2_tile order
    const float* b2;
    const float* w3;   // [5][256]
    const float* b3;
    // dropout on fc1's output
    uint32_t drop_seed, drop_stream, drop_thresh;  // thresh: floor(p * 65536) on 16-bit uniforms
    uint32_t drop_row0;  // global row of row 0 in the hash (even): masks keyed by global agent id
    float drop_scale;
    // outputs
    __bf16* h1;  // [N][512]
    __bf16* x;   // [N][512] compact K, or null
    float* h2;   // [N][256] or null
    float* q;    // [N][5] or null
    int32_t* actions;
    float epsilon;
    uint64_t act_seed, act_offset;
    // act fast path (qact_kernel): fc1's pre-activation at zero occupancy per window centre
    // at fire step stat_fs ([(L+2)(W+2)][512] f32, bias included), and fc1's occupancy
    // columns in w1o_tile order; null = the full path only
    const float* stat;
    const __bf16* w1o;
    int stat_fs;
    int stat_x0, stat_nx;  // the table's centres: x in [stat_x0, stat_x0 + stat_nx), every y
    // qfc1_kernel raw mode: f32 pre-activation (acc + bias, no ReLU / dropout) [N][512]
    float* raw;
    // X3 mode: danger residual features (evx_layout.obs_feat_lo / obs_feats_lo), lo weight
    // copies (w1 then spans K1X), the lo plane of h1
    const uint16_t* feat_lo;
    const uint16_t* const* feats_lo;
    const __bf16* w1l;
    const __bf16* w2l;
    __bf16* h1l;
    // explicit dropout keep mask [N][512] (replaces the hash when set)
    const uint8_t* drop_mask;
    // X3 act fast path: fc1's occupancy columns lo (w1o_tile order; hi in w1o)
    const __bf16* w1ol;
    // act row permutation (evx_act_perm): batch row i reads / writes row
    // perm[i / rpe] * rpe + i % rpe (dropout rows and epsilon draws keep the original row)
    const int32_t* perm;
    int rpe;
    // grouped act (evx_qmlp_act_g): gn nets interleaved in the shared row buffers -- batch row i
    // of net g reads / writes row i * gn + g (0: not interleaved)
    int gn, g;
    // fc1_tile<.., XIN>: the rows' x3 compact inputs [N][640] bf16 (X as x_expand_kernel writes it) in
    // place of generating them from the observations (evx_qmlp_stat_x: the act table's static rows)
    const __bf16* xin;
    // x_expand_kernel: the act table rows' X (evx_qmlp_params.stat_xin, rows as a.stat's), or NULL
    const __bf16* xtab;
    // persistent x3 act (evx_qmlp_fwd_out.act_ws, or NULL): [0] tiles left to the 64-row kernel,
    // [1] qact3h_rest_kernel's finished workgroups, [2 ..] those tiles
    int* rest_ws;
};
__device__ __forceinline__ int orow(const Fwd& a, int row) {
    int r = row;
    if (a.perm) {
        // rows_per_env a power of two (the trainer's R): a shift instead of a 32-bit division
        const int s = (a.rpe & (a.rpe - 1)) == 0 ? row >> (__builtin_ffs(a.rpe) - 1) : row / a.rpe;
        r = a.perm[s] * a.rpe + (row - s * a.rpe);
    }
    return a.gn ? r * a.gn + a.g : r;
}
// dropout hash row of batch row `row` (+ drop_row0): the data row, except in a grouped act,
// where it is the net's own batch row (row pairs stay hash pairs)
__device__ __forceinline__ int krow(const Fwd& a, int row) { return a.gn ? row : orow(a, row); }

template <typename T>
__device__ __forceinline__ T* adv(T* p, size_t n) { return p ? p + n : p; }
// Grouped launches (evx_qmlp_*_g, SURVEY §8f F3: independent nets per robot): every per-net
// buffer is an array [nets][one net's buffer], so net g's view is net 0's pointers advanced by
// g x the one-net size. x3 operand layout. Blocked problems (the learner) own rows
// [g N, (g + 1) N) of the row buffers; an interleaved one (the act, gn > 0) shares them. The
// dropout rows of net g are keyed g N + row.
__device__ __forceinline__ Fwd fwd_net(const Fwd& a0, int g) {
    Fwd a = a0;
    const size_t G = (size_t)g, N = (size_t)a.N;
    a.w1 += G * HID * K1X;
    a.w1l = adv(a.w1l, G * HID * K1P);
    a.w2 += G * HID2 * HID;
    a.w2l = adv(a.w2l, G * HID2 * HID);
    a.b1 += G * HID;
    a.b2 += G * NPAR;
    a.w3 += G * NPAR;
    a.b3 += G * NPAR;
    a.w1o = adv(a.w1o, G * HID * 128);
    a.w1ol = adv(a.w1ol, G * HID * 128);
    a.drop_row0 += (uint32_t)(G * N);
    if (a.gn) {
        a.g = g;
        return a;
    }
    a.obs += G * N;
    a.h1 = adv(a.h1, G * 2 * N * HID);
    a.h1l = a.h1 ? a.h1 + N * HID : nullptr;
    a.x = adv(a.x, G * N * K1X);
    a.h2 = adv(a.h2, G * N * HID2);
    a.q = adv(a.q, G * N * NACT);
    a.actions = adv(a.actions, G * N);
    a.drop_mask = adv(a.drop_mask, G * N * HID);
    return a;
}

// One row's window in the static feature map (evx_layout.obs_feat): base index of
// window cell (0, 0) = map cell (cx - 5, cy - 5) at the row's fire step. Rows past N
// and out-of-range centres are clamped into the map (their outputs are not stored).
__device__ __forceinline__ int feat_base(const Fwd& a, const evx_obs& ob) {
    const int PX = a.L + 2 + 2 * EVX_FEAT_PAD, PY = a.W + 2 + 2 * EVX_FEAT_PAD;
    const int cx = min(max(ob.cx, 0), a.L + 1), cy = min(max(ob.cy, 0), a.W + 1);
    const int fs = min(max(ob.fire_step, 0), a.t_max);
    return (fs * PX + cx + EVX_FEAT_PAD - 5) * PY + cy + EVX_FEAT_PAD - 5;
}
// map offset of window cell c = 11 i + j (c < 128; (c * 373) >> 12 == c / 11 there)
__device__ __forceinline__ int feat_off(const Fwd& a, int c) {
    const int i = (c * 373) >> 12;
    return c + i * (a.W + 2 + 2 * EVX_FEAT_PAD - 11);
}
// _get_state of window cell c (envs/evacuation_env.py:84-120, as obs_expand_kernel
// evaluates it) as fc1's 4 compact bf16 features, two per word: (occ | danger << 16,
// barrier | exit << 16), from the cell's static feature word and the occupancy bits;
// cells >= 121 are K padding (0). Branch-free.
__device__ __forceinline__ uint2 cell_feat(const evx_obs& ob, int c, uint32_t v) {
    const uint32_t one = 0x3f80u;  // bf16(1.0)
    const int q = c >> 5;          // no dynamic index into ob.occ (it would live in scratch)
    const uint32_t ow = q == 0 ? ob.occ[0] : q == 1 ? ob.occ[1] : q == 2 ? ob.occ[2] : ob.occ[3];
    const uint32_t occ = ((ow >> (c & 31)) & 1u) * one;
    uint32_t w0 = occ | (v << 16);
    uint32_t w1 = ((v >> 16) & 1u) * one | (((v >> 17) & 1u) * one) << 16;
    w0 = c < NCELL ? w0 : 0u;
    w1 = c < NCELL ? w1 : 0u;
    return make_uint2(w0, w1);
}

// ------------------------------------------------------------------ fc1
// Workgroup tile: 32*MT rows x 32*NTW*NWV columns; wave w owns all rows and
// columns [32*NTW*w, +32*NTW) of it, so every B fragment (global, L2-resident, one
// 1-KB block per wave load) feeds MT MFMAs. K in 16 chunks of 32 (8 cells): each
// thread expands 2 (or 4) cells of one row per chunk from their static feature
// words (loaded two chunks ahead) into a double-buffered LDS A tile, one barrier per
// chunk. Returns after a barrier with the A buffers free.
// X3: 4 more chunks of 32 cells' danger residuals (8 or 16 per thread), and every
// compact chunk's fragments meet the lo weights too (the features are exact in bf16
// except the danger, whose lo rides in the extra chunks).
// Column tile nt of a wave starts at ncol0 + nt * nstride.
// KU: K-loop unroll (0: the compiler's choice; the x3 act passes 2 -- fully unrolled, the
// per-chunk feature offsets were hoisted into ~70 live VGPRs and spilled)
// XIN (x3): the A rows read from a.xin (16-B pieces of X at the positions the generator writes them)
template <int MT, int NTW, int NWV, bool X3 = false, int KU = 0, bool XIN = false>
__device__ __forceinline__ void fc1_tile(const Fwd& a, int m0, int ncol0, bool want_x, char* smem,
                                         f32x16 (&acc)[MT][NTW], int nstride = 32) {
    static_assert(!XIN || X3, "X input: the x3 layout");
    constexpr int NT = 64 * NWV, RT = 32 * MT;
    constexpr int CPT = 8 * RT / NT, TPR = 8 / CPT;  // cells per thread and chunk, threads per row
    static_assert(CPT == 2 || CPT == 4, "generator: 16-B A stores");
    constexpr int NKC = X3 ? NKC1X : NKC1, KX = X3 ? K1X : K1P;
    constexpr int LPT = 32 / TPR;  // X3 residual chunks: cells per thread
    constexpr int APAD = KC1 + 8;
    auto As = reinterpret_cast<__bf16 (*)[RT][APAD]>(smem);
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
    const int gr = tid / TPR, gc = (tid % TPR) * CPT, gl = (tid % TPR) * LPT;
    const bool rowok = m0 + gr < a.N;
    evx_obs ob;
    if (XIN || !rowok) {
        ob = evx_obs{{0u, 0u, 0u, 0u}, 0, 0, 0, 0};
    } else {
        ob = a.obs[orow(a, m0 + gr)];
    }
    const bool wx = a.x && rowok && want_x;
    const int fbase = feat_base(a, ob);
    const uint32_t* fb = (a.feats ? a.feats[ob.layout] : a.feat) + fbase;
    const uint16_t* flb = nullptr;
    if constexpr (X3) flb = (a.feats_lo ? a.feats_lo[ob.layout] : a.feat_lo) + fbase;
    uint32_t fv[CPT];
    uint32_t lv[X3 ? LPT / 2 : 1];  // residual bf16 pairs
    constexpr int XP = CPT / 2;  // XIN: 16-B pieces per thread and chunk (CPT / 2 compact = LPT / 8 residual)
    static_assert(!XIN || LPT / 8 == XP, "XIN: the compact and residual pieces per thread agree");
    uint4 xr[XP];
    const __bf16* xrow = XIN ? a.xin + (size_t)(m0 + gr) * K1X : nullptr;
    auto reads = [&](int kc) {
        if constexpr (XIN) {
            const int c0 = kc < NKC1 ? kc * KC1 + gc * 4 : kc * KC1 + gl;
#pragma unroll
            for (int t = 0; t < XP; t++) xr[t] = rowok ? *reinterpret_cast<const uint4*>(xrow + c0 + 8 * t) : make_uint4(0u, 0u, 0u, 0u);
        } else if (!X3 || kc < NKC1) {
#pragma unroll
            for (int t = 0; t < CPT; t++) fv[t] = fb[feat_off(a, kc * 8 + gc + t)];
        } else if constexpr (X3) {
#pragma unroll
            for (int t = 0; t < LPT; t += 2) {  // cells 32 (kc - 16) + gl + t, t + 1 (< 128: inside the padded map)
                const int c0 = (kc - NKC1) * 32 + gl + t;
                const uint32_t l0 = c0 < NCELL ? (uint32_t)flb[feat_off(a, c0)] : 0u;
                const uint32_t l1 = c0 + 1 < NCELL ? (uint32_t)flb[feat_off(a, c0 + 1)] : 0u;
                lv[t >> 1] = l0 | (l1 << 16);
            }
        }
    };
    auto stash = [&](int buf, int kc) {
        if constexpr (XIN) {
            const int c0 = kc < NKC1 ? gc * 4 : gl;
#pragma unroll
            for (int t = 0; t < XP; t++) *reinterpret_cast<uint4*>(&As[buf][gr][c0 + 8 * t]) = xr[t];
        } else if (!X3 || kc < NKC1) {
#pragma unroll
            for (int t = 0; t < CPT; t += 2) {
                const uint2 f0 = cell_feat(ob, kc * 8 + gc + t, fv[t]), f1 = cell_feat(ob, kc * 8 + gc + t + 1, fv[t + 1]);
                const uint4 v = make_uint4(f0.x, f0.y, f1.x, f1.y);
                *reinterpret_cast<uint4*>(&As[buf][gr][(gc + t) * 4]) = v;
                if (wx) *reinterpret_cast<uint4*>(a.x + (size_t)(m0 + gr) * KX + kc * KC1 + (gc + t) * 4) = v;
            }
        } else if constexpr (X3) {
#pragma unroll
            for (int t = 0; t < LPT; t += 8) {
                const uint4 v = make_uint4(lv[t / 2], lv[t / 2 + 1], lv[t / 2 + 2], lv[t / 2 + 3]);
                *reinterpret_cast<uint4*>(&As[buf][gr][gl + t]) = v;
                if (wx) *reinterpret_cast<uint4*>(a.x + (size_t)(m0 + gr) * KX + kc * KC1 + gl + t) = v;
            }
        }
    };
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
        for (int j = 0; j < NTW; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;
    // B fragments two K chunks ahead (bc: this chunk, bn: the next, bf: the one after);
    // X3: the lo fragments of the compact chunks alongside (lc, ln, lf)
    constexpr int NL = X3 ? NTW : 1;
    // (the lo fragments one chunk ahead only: register budget of the X3 act kernel)
    bf16x8 bc[NTW][2], bn[NTW][2], bf[NTW][2];
    bf16x8 lc[NL][2], ln[NL][2];
    auto loadB = [&](int kc, bf16x8 (&b)[NTW][2]) {
#pragma unroll
        for (int nt = 0; nt < NTW; nt++) {
            const int n = ncol0 + nt * nstride;
#pragma unroll
            for (int s = 0; s < 2; s++)
                b[nt][s] = *reinterpret_cast<const bf16x8*>(a.w1 + w1_tile(n >> 5, kc, s, NKC) + lane * 8);
        }
    };
    auto loadL = [&](int kc, bf16x8 (&l)[NL][2]) {
        if constexpr (X3) {
            if (kc < NKC1) {
#pragma unroll
                for (int nt = 0; nt < NTW; nt++)
#pragma unroll
                    for (int s = 0; s < 2; s++)
                        l[nt][s] = *reinterpret_cast<const bf16x8*>(a.w1l + w1_tile((ncol0 + nt * nstride) >> 5, kc, s) + lane * 8);
            }
        }
    };
    // X3: hi fragments one chunk ahead as well (bf unused)
    constexpr int AH = X3 ? 1 : 2;
    reads(0);
    stash(0, 0);
    reads(1);
    loadB(0, bc);
    if constexpr (AH == 2) loadB(1, bn);
    loadL(0, lc);
    __syncthreads();
    auto kstep = [&](int kc) {
        const int buf = kc & 1;
        if (kc + AH < NKC) loadB(kc + AH, AH == 2 ? bf : bn);
        if (kc + 1 < NKC) loadL(kc + 1, ln);
#pragma unroll
        for (int s = 0; s < 2; s++)
#pragma unroll
            for (int mt = 0; mt < MT; mt++) {
                const bf16x8 av = *reinterpret_cast<const bf16x8*>(&As[buf][mt * 32 + (lane & 31)][s * 16 + 8 * h]);
#pragma unroll
                for (int nt = 0; nt < NTW; nt++) {
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bc[nt][s], acc[mt][nt], 0, 0, 0);
                    if constexpr (X3) {
                        if (kc < NKC1)
                            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, lc[nt][s], acc[mt][nt], 0, 0, 0);
                    }
                }
            }
        if (kc + 1 < NKC) {
            stash(buf ^ 1, kc + 1);
            if (kc + 2 < NKC) reads(kc + 2);
#pragma unroll
            for (int nt = 0; nt < NTW; nt++) {
                bc[nt][0] = bn[nt][0];
                bc[nt][1] = bn[nt][1];
                if constexpr (AH == 2) {
                    bn[nt][0] = bf[nt][0];
                    bn[nt][1] = bf[nt][1];
                }
                if constexpr (X3) {
                    lc[nt][0] = ln[nt][0];
                    lc[nt][1] = ln[nt][1];
                }
            }
        }
        __syncthreads();
    };
    if constexpr (KU == 2) {
#pragma unroll 2
        for (int kc = 0; kc < NKC; kc++) kstep(kc);
    } else {
        for (int kc = 0; kc < NKC; kc++) kstep(kc);
    }
}

// fc1 epilogue of one 32-row slab: bias (centre channel folded in), ReLU, dropout
// (one hash per row pair), bf16 into dst[row within slab][column within tile]
// (X3: hi into dst, lo into dstl). An explicit keep mask (a.drop_mask) replaces the hash.
// MODE 0: no dropout, 1: the hash, 2: an explicit keep mask (a.drop_mask: the reference's
// captured torch masks, tests). One straight-line body per mode: a per-element branch on the
// mode inside the unrolled loops split it into many blocks and cost the act kernel ~100 VGPRs
// of spills.
// phs (MODE 1, or NULL): the row-pair hashes of the slab's 16 pairs, precomputed (the act: the
// same hashes serve both column halves, and computing them here hoisted 32 row lookups into
// registers)
template <int NTW, int LD, bool X3, int MODE>
__device__ __forceinline__ void fc1_slab_m(const Fwd& a, const f32x16 (&accm)[NTW], const float (&bias)[NTW],
                                           int row0, int col0, int cl0, __bf16 (*dst)[LD], __bf16 (*dstl)[LD],
                                           const uint32_t* phs = nullptr) {
    const int lane = threadIdx.x & 63, h = lane >> 5;
#pragma unroll
    for (int r = 0; r < 16; r += 2) {  // rows rl, rl + 1: one dropout hash per pair
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
        // rows rl, rl + 1 (rl even) stay a pair under the act permutation (rpe even)
        uint32_t ph = 0u;
        uint2 ph3[2];  // MODE 3 (a row-permuted act): rows rl, rl + 1's pair hashes and halves
        if constexpr (MODE == 3) {
            const uint2* p3 = reinterpret_cast<const uint2*>(phs);
            ph3[0] = p3[rl];
            ph3[1] = p3[rl + 1];
        }
        if constexpr (MODE == 1)
            ph = phs ? phs[rl >> 1]
                     : drop_row(a.drop_seed, a.drop_stream, (a.drop_row0 + (uint32_t)krow(a, row0 + rl)) >> 1);
#pragma unroll
        for (int nt = 0; nt < NTW; nt++) {
            const int cl = cl0 + nt * 32 + (lane & 31);
            float v0 = accm[nt][r] + bias[nt], v1 = accm[nt][r + 1] + bias[nt];
            v0 = v0 > 0.f ? v0 : 0.f;
            v1 = v1 > 0.f ? v1 : 0.f;
            if constexpr (MODE == 2) {
                const int r0 = row0 + rl, c = col0 + cl;
                const bool k0 = r0 < a.N && a.drop_mask[(size_t)r0 * HID + c];
                const bool k1 = r0 + 1 < a.N && a.drop_mask[(size_t)(r0 + 1) * HID + c];
                v0 = k0 ? v0 * a.drop_scale : 0.f;
                v1 = k1 ? v1 * a.drop_scale : 0.f;
            } else if constexpr (MODE == 1) {
                const uint32_t hh = drop_pair(ph, (uint32_t)(col0 + cl));
                v0 = (hh & 0xffffu) >= a.drop_thresh ? v0 * a.drop_scale : 0.f;
                v1 = (hh >> 16) >= a.drop_thresh ? v1 * a.drop_scale : 0.f;
            } else if constexpr (MODE == 3) {  // rows from different pairs: each its own pair's half
                const uint32_t c = (uint32_t)(col0 + cl);
                const uint32_t h0 = drop_pair(ph3[0].x, c), h1 = drop_pair(ph3[1].x, c);
                v0 = (ph3[0].y ? h0 >> 16 : h0 & 0xffffu) >= a.drop_thresh ? v0 * a.drop_scale : 0.f;
                v1 = (ph3[1].y ? h1 >> 16 : h1 & 0xffffu) >= a.drop_thresh ? v1 * a.drop_scale : 0.f;
            }
            if constexpr (X3) {
                split2(v0, dst[rl][cl], dstl[rl][cl]);
                split2(v1, dst[rl + 1][cl], dstl[rl + 1][cl]);
            } else {
                dst[rl][cl] = (__bf16)v0;
                dst[rl + 1][cl] = (__bf16)v1;
            }
        }
    }
}
// fc1 epilogue of one 32-row slab: bias (centre channel folded in), ReLU, dropout
// (one hash per row pair), bf16 into dst[row within slab][column within tile]
// (X3: hi into dst, lo into dstl). An explicit keep mask (a.drop_mask) replaces the hash.
template <int NTW, int LD, bool X3 = false>
__device__ __forceinline__ void fc1_slab(const Fwd& a, const f32x16 (&accm)[NTW], const float (&bias)[NTW],
                                         int row0, int col0, int cl0, __bf16 (*dst)[LD], __bf16 (*dstl)[LD] = nullptr) {
    if (a.drop_mask) fc1_slab_m<NTW, LD, X3, 2>(a, accm, bias, row0, col0, cl0, dst, dstl);
    else if (a.drop_thresh) fc1_slab_m<NTW, LD, X3, 1>(a, accm, bias, row0, col0, cl0, dst, dstl);
    else fc1_slab_m<NTW, LD, X3, 0>(a, accm, bias, row0, col0, cl0, dst, dstl);
}

// H1 = dropout(relu(X W1^T + b1)) -> bf16 [N][512] (and X when a.x). Act batches:
// <4, 2, 8> (128 rows x all 512 columns: every row expanded once); learner batches
// <2, 1, 4> (64 x 128). H1 is staged per 32-row slab through LDS so it leaves in
// 16-B row segments.
// GR (grouped, blocked): blockIdx.z = net * np + problem, net g's view of the problem
template <int MT, int NTW, int NWV, bool X3 = false, bool GR = false, bool XIN = false>
__global__ __launch_bounds__(64 * NWV, NWV == 8 ? 1 : 2) void qfc1_kernel(Fwd a0, Fwd a1, int np) {
    Fwd ag;
    if constexpr (GR) ag = fwd_net((int)blockIdx.z % np ? a1 : a0, (int)blockIdx.z / np);
    const Fwd& a = GR ? ag : (blockIdx.z ? a1 : a0);  // two independent problems in one launch (online / target)
    constexpr int NT = 64 * NWV, RT = 32 * MT, NW = 32 * NTW * NWV;
    constexpr int APAD = KC1 + 8, CPAD = NW + 8;
    constexpr int ABYTES = 2 * RT * APAD * 2, CBYTES = (X3 ? 2 : 1) * 32 * CPAD * 2;
    __shared__ __attribute__((aligned(16))) char smem[ABYTES > CBYTES ? ABYTES : CBYTES];
    auto Cs = reinterpret_cast<__bf16 (*)[CPAD]>(smem);
    auto Cl = reinterpret_cast<__bf16 (*)[CPAD]>(smem + 32 * CPAD * 2);  // X3: lo plane
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int m0 = blockIdx.x * RT;
    const int ncol0 = blockIdx.y * NW + w * (32 * NTW);
    f32x16 acc[MT][NTW];
    fc1_tile<MT, NTW, NWV, X3, 0, XIN>(a, m0, ncol0, blockIdx.y == 0, smem, acc);
    float bias[NTW];
#pragma unroll
    for (int nt = 0; nt < NTW; nt++) bias[nt] = a.b1[ncol0 + nt * 32 + (lane & 31)];
    if (a.raw) {  // pre-activation table (evx_qmlp_stat): acc + bias as f32, 128-B row segments
#pragma unroll
        for (int mt = 0; mt < MT; mt++)
#pragma unroll
            for (int nt = 0; nt < NTW; nt++)
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int row = m0 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    if (row < a.N) a.raw[(size_t)row * HID + ncol0 + nt * 32 + (lane & 31)] = acc[mt][nt][r] + bias[nt];
                }
        return;
    }
#pragma unroll
    for (int mt = 0; mt < MT; mt++) {
        if (mt) __syncthreads();  // the previous slab has been stored
        fc1_slab<NTW, CPAD, X3>(a, acc[mt], bias, m0 + mt * 32, blockIdx.y * NW, w * (32 * NTW), Cs, Cl);
        __syncthreads();
        constexpr int SEG = NW / 8;  // 16-B segments per row
        for (int i = tid; i < (X3 ? 2 : 1) * 32 * SEG; i += NT) {
            const int pl = i >= 32 * SEG, ii = i - pl * 32 * SEG;
            const int rl = ii / SEG, cc = (ii - rl * SEG) * 8;
            const int row = m0 + mt * 32 + rl;
            if (row < a.N)
                *reinterpret_cast<uint4*>((pl ? a.h1l : a.h1) + (size_t)row * HID + blockIdx.y * NW + cc) =
                    *reinterpret_cast<const uint4*>(pl ? &Cl[rl][cc] : &Cs[rl][cc]);
        }
    }
}

// fc3 + DQNAgent.act's epsilon-greedy (agents/dqn_agent.py:101-124) for one row: 4
// consecutive threads (part = tid & 3) hold quarter dot products of H2 row `hrow`
// (LDS, f32) with W3 (LDS); the sums are combined by two xor shuffles
__device__ __forceinline__ void fc3_act(const Fwd& a, const float* hrow, const float (*W3s)[HID2], int row,
                                        bool rowok) {
    const int part = threadIdx.x & 3;
    float qv[NACT];
#pragma unroll
    for (int t = 0; t < NACT; t++) qv[t] = 0.f;
    // part p takes columns p, p + 4, ...: with a row pitch of 4 (mod 32) words the 32 lanes
    // of a half-wave (8 rows x 4 parts) read 32 distinct banks, and W3s is one bank per part
#pragma unroll 4  // fully unrolled, its 64 + 320 LDS loads were hoisted together (act kernel spills)
    for (int j = 0; j < HID2 / 4; j++) {
        const int n = part + 4 * j;
        const float hv = hrow[n];
#pragma unroll
        for (int t = 0; t < NACT; t++) qv[t] += hv * W3s[t][n];
    }
#pragma unroll
    for (int t = 0; t < NACT; t++) {
        qv[t] += __shfl_xor(qv[t], 1, 64);
        qv[t] += __shfl_xor(qv[t], 2, 64);
    }
    if (part == 0 && rowok) {
#pragma unroll
        for (int t = 0; t < NACT; t++) qv[t] += a.b3[t];
        if (a.q) {
#pragma unroll
            for (int t = 0; t < NACT; t++) a.q[(size_t)row * NACT + t] = qv[t];
        }
        if (a.actions) {  // DQNAgent.act: epsilon-greedy over argmax (first maximum)
            int best = 0;
            float bv = qv[0];
#pragma unroll
            for (int t = 1; t < NACT; t++)
                if (qv[t] > bv) {
                    bv = qv[t];
                    best = t;
                }
            if (a.epsilon > 0.f) {
                const uint64_t c = (uint64_t)row + a.act_offset;
                const u4 r = philox((uint32_t)c, (uint32_t)(c >> 32), 0xac7u, 0u, (uint32_t)a.act_seed,
                                    (uint32_t)(a.act_seed >> 32));
                if (u01(r.x) <= a.epsilon) best = (int)((uint64_t)r.y * (uint64_t)NACT >> 32);
            }
            a.actions[row] = best;
        }
    }
}

// ------------------------------------------------------------ fused act
constexpr int A3_HP = 256 + 8;  // x3 act: H1 half-plane / H2 plane row pitch (bf16), 528 B
// X3 fc2 -> fc3 of a 64-row tile of 4 waves. fc2 runs with swapped operands (A = W2 fragments,
// B = H1 rows), so wave w's acc[mt][nt] is an H2^T tile: lane l holds tile row (batch row)
// 32 mt + (l & 31), register r column n = 64 w + 32 nt + (r & 3) + 8 (r >> 2) + 4 (l >> 5).
// fc3t_x3: H2 = relu(acc + b2) (to a.h2 in 16-B row pieces when set: the learner's backward),
// split into bf16 hi / lo in registers, and Q^T = W3 . H2^T on the matrix cores straight from
// the accumulators (x3: hi*hi + hi*lo + lo*hi): registers 8 kb .. 8 kb + 7 of a tile are the B
// operand of the 16 columns n = 64 w + 32 nt + 16 kb + 4 (l >> 5) + {0..3, 8..11} (a fixed
// permutation of K, which the A operand -- W3's 5 rows padded to 32, split in registers --
// follows). The 4 waves' partial Q^T over their 64 columns meet in LDS (red: [4][5][64] f32)
// and are added in wave order; DQNAgent.act's epsilon-greedy follows (q_out). Used by
// qfc23<X3> and qact3h alike (act and forward give the same Q bit for bit). act_rows: Q and
// actions go to orow (act), else to the batch row. (Storing H2 and 4-thread f32 dot products
// in fc3_act cost ~13k cycles per act tile.)
__device__ __forceinline__ void q_out(const Fwd& a, float (&qv)[NACT], int row) {
#pragma unroll
    for (int t = 0; t < NACT; t++) qv[t] += a.b3[t];
    if (a.q) {
#pragma unroll
        for (int t = 0; t < NACT; t++) a.q[(size_t)row * NACT + t] = qv[t];
    }
    if (a.actions) {  // DQNAgent.act: epsilon-greedy over argmax (first maximum)
        int best = 0;
        float bv = qv[0];
#pragma unroll
        for (int t = 1; t < NACT; t++)
            if (qv[t] > bv) {
                bv = qv[t];
                best = t;
            }
        if (a.epsilon > 0.f) {
            const uint64_t c = (uint64_t)row + a.act_offset;
            const u4 r = philox((uint32_t)c, (uint32_t)(c >> 32), 0xac7u, 0u, (uint32_t)a.act_seed,
                                (uint32_t)(a.act_seed >> 32));
            if (u01(r.x) <= a.epsilon) best = (int)((uint64_t)r.y * (uint64_t)NACT >> 32);
        }
        a.actions[row] = best;
    }
}
// MT: 32-row slabs of the tile (2: 64 rows; 1: qfc23's 32-row tiles for small batches)
template <int MT = 2>
__device__ __forceinline__ void fc3t_x3(const Fwd& a, const f32x16 (&acc)[MT][2], const float (*W3s)[HID2],
                                        float* red, int m0, bool act_rows) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, j = lane & 31;
    const int t = lane & 31;  // A row: action (< NACT) or padding
    f32x16 qp[MT];
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
#pragma unroll
        for (int r = 0; r < 16; r++) qp[mt][r] = 0.f;
#pragma unroll
    for (int nt = 0; nt < 2; nt++) {
        const int nb = w * 64 + nt * 32 + 4 * h;  // + (r & 3) + 8 (r >> 2)
        float b2v[16];
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const float4 bv = *reinterpret_cast<const float4*>(&a.b2[nb + 8 * g]);
            b2v[4 * g] = bv.x;
            b2v[4 * g + 1] = bv.y;
            b2v[4 * g + 2] = bv.z;
            b2v[4 * g + 3] = bv.w;
        }
        bf16x8 wh[2], wl[2];  // W3 in the K order of k-blocks 0 and 1 of this column tile
#pragma unroll
        for (int kb = 0; kb < 2; kb++) {
            float u[8];
            if (t < NACT) {
                const float4 u0 = *reinterpret_cast<const float4*>(&W3s[t][nb + 16 * kb]);
                const float4 u1 = *reinterpret_cast<const float4*>(&W3s[t][nb + 16 * kb + 8]);
                u[0] = u0.x; u[1] = u0.y; u[2] = u0.z; u[3] = u0.w;
                u[4] = u1.x; u[5] = u1.y; u[6] = u1.z; u[7] = u1.w;
            } else {
#pragma unroll
                for (int e = 0; e < 8; e++) u[e] = 0.f;
            }
#pragma unroll
            for (int e = 0; e < 8; e++) {
                __bf16 hi, lo;
                split2(u[e], hi, lo);
                wh[kb][e] = hi;
                wl[kb][e] = lo;
            }
        }
#pragma unroll
        for (int mt = 0; mt < MT; mt++) {
            const int row = m0 + mt * 32 + j;
            float v[16];
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const float x = acc[mt][nt][r] + b2v[r];
                v[r] = x > 0.f ? x : 0.f;
            }
            if (a.h2 && row < a.N) {
#pragma unroll
                for (int g = 0; g < 4; g++)
                    *reinterpret_cast<float4*>(&a.h2[(size_t)row * HID2 + nb + 8 * g]) =
                        make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
            }
#pragma unroll
            for (int kb = 0; kb < 2; kb++) {
                bf16x8 bh, bl;
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    __bf16 hi, lo;
                    split2(v[8 * kb + e], hi, lo);
                    bh[e] = hi;
                    bl[e] = lo;
                }
                qp[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh[kb], bh, qp[mt], 0, 0, 0);
                qp[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh[kb], bl, qp[mt], 0, 0, 0);
                qp[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl[kb], bh, qp[mt], 0, 0, 0);
            }
        }
    }
    // qp[mt] = this wave's Q^T partial: lane l holds tile row 32 mt + (l & 31), actions
    // 4 (l >> 5) + r (r < 4; valid below NACT)
    auto R = reinterpret_cast<float (*)[NACT][32 * MT]>(red);  // [4][NACT][32 MT]
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int act = 4 * h + r;
            if (act < NACT) R[w][act][mt * 32 + j] = qp[mt][r];
        }
    __syncthreads();
    if (tid < 32 * MT) {
        const int rt = m0 + tid;
        if (rt < a.N) {
            float qv[NACT];
#pragma unroll
            for (int k = 0; k < NACT; k++) qv[k] = ((R[0][k][tid] + R[1][k][tid]) + R[2][k][tid]) + R[3][k][tid];
            q_out(a, qv, act_rows ? orow(a, rt) : rt);
        }
    }
}

// fc3t_x3 for qact3p_kernel's 8 waves, in two parts. fc3p_partials: wave (column group cg, row half
// at r0) holds the H2^T tiles of fc2 columns 64 cg .. + 63 for rows r0 .. r0 + 63 (acc[mt][nt] as
// fc3t_x3's); H2 = relu(acc + b2) (b2 from LDS), and its Q^T partials (x3 MFMAs against W3, as
// fc3t_x3) go to red [4][NACT][128] by column group. fc3p_rows (after a barrier): thread t < 128 adds
// row t's partials in column-group order -- as fc3t_x3 adds its 4 waves' (the same bits) -- and runs
// DQNAgent.act's epsilon-greedy (q_out).
__device__ __forceinline__ void fc3p_partials(const f32x16 (&acc)[2][2], const float (*W3s)[HID2], const float* b2s,
                                              float* red, int cg, int r0, int lane) {
    const int h = lane >> 5, j = lane & 31;
    const int t = lane & 31;
    f32x16 qp[2];
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int r = 0; r < 16; r++) qp[mt][r] = 0.f;
#pragma unroll
    for (int nt = 0; nt < 2; nt++) {
        const int nb = cg * 64 + nt * 32 + 4 * h;  // + (r & 3) + 8 (r >> 2)
        float b2v[16];
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const float4 bv = *reinterpret_cast<const float4*>(&b2s[nb + 8 * g]);
            b2v[4 * g] = bv.x;
            b2v[4 * g + 1] = bv.y;
            b2v[4 * g + 2] = bv.z;
            b2v[4 * g + 3] = bv.w;
        }
        bf16x8 wh[2], wl[2];
#pragma unroll
        for (int kb = 0; kb < 2; kb++) {
            float u[8];
            if (t < NACT) {
                const float4 u0 = *reinterpret_cast<const float4*>(&W3s[t][nb + 16 * kb]);
                const float4 u1 = *reinterpret_cast<const float4*>(&W3s[t][nb + 16 * kb + 8]);
                u[0] = u0.x; u[1] = u0.y; u[2] = u0.z; u[3] = u0.w;
                u[4] = u1.x; u[5] = u1.y; u[6] = u1.z; u[7] = u1.w;
            } else {
#pragma unroll
                for (int e = 0; e < 8; e++) u[e] = 0.f;
            }
#pragma unroll
            for (int e = 0; e < 8; e++) {
                __bf16 hi, lo;
                split2(u[e], hi, lo);
                wh[kb][e] = hi;
                wl[kb][e] = lo;
            }
        }
#pragma unroll
        for (int mt = 0; mt < 2; mt++) {
            float v[16];
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const float x = acc[mt][nt][r] + b2v[r];
                v[r] = x > 0.f ? x : 0.f;
            }
#pragma unroll
            for (int kb = 0; kb < 2; kb++) {
                bf16x8 bh, bl;
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    __bf16 hi, lo;
                    split2(v[8 * kb + e], hi, lo);
                    bh[e] = hi;
                    bl[e] = lo;
                }
                qp[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh[kb], bh, qp[mt], 0, 0, 0);
                qp[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh[kb], bl, qp[mt], 0, 0, 0);
                qp[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl[kb], bh, qp[mt], 0, 0, 0);
            }
        }
    }
    auto R = reinterpret_cast<float (*)[NACT][128]>(red);  // [4][NACT][128]
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int act = 4 * h + r;
            if (act < NACT) R[cg][act][r0 + mt * 32 + j] = qp[mt][r];
        }
}
// rows spread over waves 0..3 (32 each, lanes 0..31: one wave per SIMD) -- q_out's epsilon draw is a
// 10-round Philox per row, and two waves carrying all 128 rows held the next slot back
// rowS: the tile rows' output rows (orow), recorded when the rows were set up
__device__ __forceinline__ void fc3p_rows(const Fwd& a, const float* red, int m0, const int* rowS) {
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    auto R = reinterpret_cast<const float (*)[NACT][128]>(red);
    if (w < 4 && l < 32) {
        const int r = 32 * w + l, rt = m0 + r;
        if (rt < a.N) {
            float qv[NACT];
#pragma unroll
            for (int k = 0; k < NACT; k++) qv[k] = ((R[0][k][r] + R[1][k][r]) + R[2][k][r]) + R[3][k][r];
            q_out(a, qv, rowS[r]);
        }
    }
}

// DQNAgent.act for 128 rows per workgroup (8 waves) in one launch: fc1 as
// qfc1_kernel<4, 2, 8>, H1 kept in LDS (bf16, never written to HBM), fc2 with wave w
// on columns [32w, 32w + 32) over all 128 rows (A fragments from the H1 tile, W2
// fragments from L2), H2 (f32) back into the same LDS, fc3 + epsilon-greedy as
// qfc23_kernel. Dynamic LDS: ACT_LDS bytes.
//
// Fast path (a.stat set, every row of the tile at fire step stat_fs -- every env older
// than 180 steps: the fire never resets): fc1's inputs other than the occupancy bits
// depend only on the window centre and the fire step, so fc1 = stat[centre] (the
// pre-activation at zero occupancy, bias included, rebuilt by evx_qmlp_stat after each
// weight update) + the occupancy columns times the 121 bits: the accumulators start
// from the table and K shrinks from 512 to 128, with the A fragments made in registers
// from the bits (no LDS staging, no barriers). Same products, f32 sums in another order
// (Q within f32 rounding of the full path).
constexpr int ACT_HP = HID + 8;                                  // H1 row pitch (bf16)
constexpr int ACT_H2P = HID2 + 4;                                // H2 row pitch (f32; fc3_act banks)
constexpr int ACT_HBYTES = 128 * ACT_HP * 2;                     // 133,120 = 128 * 260 * 4
static_assert(ACT_HBYTES >= 128 * ACT_H2P * 4, "H2 overlays the H1 tile");
constexpr int ACT_LDS = ACT_HBYTES + NACT * HID2 * 4 + 128 * 4;  // + W3 + window centres
__global__ __launch_bounds__(512, 1) void qact_kernel(Fwd a) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    auto H1s = reinterpret_cast<__bf16 (*)[ACT_HP]>(dsm);
    auto H2s = reinterpret_cast<float (*)[ACT_H2P]>(dsm);
    auto W3s = reinterpret_cast<float (*)[HID2]>(dsm + ACT_HBYTES);
    int* posS = reinterpret_cast<int*>(dsm + ACT_HBYTES + NACT * HID2 * 4);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    const int m0 = blockIdx.x * 128;
    for (int i = tid; i < NACT * HID2; i += 512) W3s[i / HID2][i % HID2] = a.w3[i];
    bool fast = false;
    if (a.stat) {  // tile-uniform: every row at the table's fire step, centre inside the map
        bool ok = true;
        if (tid < 128) {
            int pos = 0;
            if (m0 + tid < a.N) {
                const evx_obs ob = a.obs[orow(a, m0 + tid)];
                ok = min(max(ob.fire_step, 0), a.t_max) == a.stat_fs && ob.cx >= a.stat_x0 &&
                     ob.cx < a.stat_x0 + a.stat_nx && ob.cy >= 0 && ob.cy <= a.W + 1;
                pos = ok ? (ob.cx - a.stat_x0) * (a.W + 2) + ob.cy : 0;
            }
            posS[tid] = pos;
        }
        fast = __syncthreads_and(ok);  // also publishes posS
    }
    if (fast) {  // fc1 = stat[centre] + occupancy columns x bits -> H1 tile
        f32x16 acc[4][2];
        const int col0 = w * 64 + (lane & 31);
#pragma unroll
        for (int mt = 0; mt < 4; mt++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int rl = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const float* srow = a.stat + (size_t)posS[rl] * HID + col0;
                acc[mt][0][r] = srow[0];
                acc[mt][1][r] = srow[32];
            }
        uint32_t occ[4][4];
#pragma unroll
        for (int mt = 0; mt < 4; mt++) {
            const int row = m0 + mt * 32 + (lane & 31);
            uint4 o = make_uint4(0u, 0u, 0u, 0u);
            if (row < a.N) o = *reinterpret_cast<const uint4*>(&a.obs[orow(a, row)].occ[0]);
            occ[mt][0] = o.x;
            occ[mt][1] = o.y;
            occ[mt][2] = o.z;
            occ[mt][3] = o.w;
        }
        const uint32_t one = 0x3f80u;
#pragma unroll
        for (int ks = 0; ks < 8; ks++) {  // k-step: cells 16 ks + 8 h .. + 7 of the 128
            bf16x8 b[2];
#pragma unroll
            for (int nt = 0; nt < 2; nt++)
                b[nt] = *reinterpret_cast<const bf16x8*>(a.w1o + w1o_tile(w * 2 + nt, ks >> 1, ks & 1) + lane * 8);
            const int c0 = ks * 16 + 8 * h;  // multiple of 8: the 8 bits sit in one word
#pragma unroll
            for (int mt = 0; mt < 4; mt++) {
                const uint32_t wd = (c0 >> 5) == 0 ? occ[mt][0] : (c0 >> 5) == 1 ? occ[mt][1]
                                  : (c0 >> 5) == 2 ? occ[mt][2] : occ[mt][3];
                const uint32_t bits = (wd >> (c0 & 31)) & 0xffu;
                uint32_t av4[4];
#pragma unroll
                for (int j = 0; j < 4; j++)
                    av4[j] = ((bits >> (2 * j)) & 1u) * one | (((bits >> (2 * j + 1)) & 1u) * one) << 16;
                const bf16x8 av = __builtin_bit_cast(bf16x8, av4);
#pragma unroll
                for (int nt = 0; nt < 2; nt++)
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, b[nt], acc[mt][nt], 0, 0, 0);
            }
        }
        const float zero[2] = {0.f, 0.f};  // the table holds the bias
#pragma unroll
        for (int mt = 0; mt < 4; mt++)
            fc1_slab<2, ACT_HP>(a, acc[mt], zero, m0 + mt * 32, 0, w * 64,
                                reinterpret_cast<__bf16 (*)[ACT_HP]>(&H1s[mt * 32][0]));
    } else {  // fc1 -> H1 tile
        f32x16 acc[4][2];
        fc1_tile<4, 2, 8>(a, m0, w * 64, false, dsm, acc);  // ends with a barrier: A buffers free
        float bias[2];
#pragma unroll
        for (int nt = 0; nt < 2; nt++) bias[nt] = a.b1[w * 64 + nt * 32 + (lane & 31)];
#pragma unroll
        for (int mt = 0; mt < 4; mt++)
            fc1_slab<2, ACT_HP>(a, acc[mt], bias, m0 + mt * 32, 0, w * 64,
                                reinterpret_cast<__bf16 (*)[ACT_HP]>(&H1s[mt * 32][0]));
    }
    __syncthreads();
    // fc2: wave w -> columns [32w, 32w + 32), all 128 rows; K = 512 as 16 chunks x 2 steps
    f32x16 acc2[4];
#pragma unroll
    for (int mt = 0; mt < 4; mt++)
#pragma unroll
        for (int r = 0; r < 16; r++) acc2[mt][r] = 0.f;
    bf16x8 bc[2], bn[2];
#pragma unroll
    for (int s = 0; s < 2; s++) bc[s] = *reinterpret_cast<const bf16x8*>(a.w2 + w2_tile(w, 0, s) + lane * 8);
    for (int kc = 0; kc < HID / 32; kc++) {
        if (kc + 1 < HID / 32) {
#pragma unroll
            for (int s = 0; s < 2; s++)
                bn[s] = *reinterpret_cast<const bf16x8*>(a.w2 + w2_tile(w, kc + 1, s) + lane * 8);
        }
#pragma unroll
        for (int s = 0; s < 2; s++)
#pragma unroll
            for (int mt = 0; mt < 4; mt++) {
                const bf16x8 av =
                    *reinterpret_cast<const bf16x8*>(&H1s[mt * 32 + (lane & 31)][kc * 32 + s * 16 + 8 * h]);
                acc2[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bc[s], acc2[mt], 0, 0, 0);
            }
        bc[0] = bn[0];
        bc[1] = bn[1];
    }
    __syncthreads();  // every wave is done with H1: H2 reuses the space
    {
        const int col = w * 32 + (lane & 31);
        const float bias = a.b2[col];
#pragma unroll
        for (int mt = 0; mt < 4; mt++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const float v = acc2[mt][r] + bias;
                H2s[mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h][col] = v > 0.f ? v : 0.f;
            }
    }
    __syncthreads();
    const int row = tid >> 2;
    fc3_act(a, &H2s[row][0], W3s, orow(a, m0 + row), m0 + row < a.N);
}

// X3 (f32-accurate) act: H1 goes through LDS in two column halves (hi + lo planes of a whole
// 512-column tile would not fit beside a second workgroup). fc1 runs once over all 512 columns
// (the observations are expanded once per half on the full path); half hh's tiles go into the
// two LDS planes, then fc2 accumulates over that half of its K (3 MFMAs per fragment pair:
// hi*hi, hi*lo, lo*hi). The A staging of fc1, the H1 half planes and finally H2 share one
// LDS region.
// the occupancy-fragment table (table path: byte of 8 cell bits -> the 8 bf16 A values, 0 or
// 1.0, of one MFMA k-step; one ds_read_b128 instead of ~25 VALU)
constexpr int ACT3_OCC = 256 * 16;
// diagnostic build (-DEVX_ACT_STAMPS, tools/act_stamps.py): wave 0's s_memtime at the phase
// boundaries of every workgroup (evx_diag_act_stamps, qact3h_kernel)
#ifdef EVX_ACT_STAMPS
constexpr int ACT_NST = 12;
__device__ long long g_act_st[8192 * ACT_NST];
#define ACT_ST(i)                                                                                   \
    do {                                                                                            \
        if (threadIdx.x == 0 && blockIdx.x < 8192)                                                  \
            g_act_st[blockIdx.x * ACT_NST + (i)] = (long long)__builtin_amdgcn_s_memtime();         \
    } while (0)
#else
#define ACT_ST(i)
#endif
// The x3 act on 64-row tiles of 4 waves (256 threads, ACT3H_LDS = 77 KB): two independent
// workgroups per CU, so one's epilogues, barriers, table loads and fc3 run under the other's
// MFMAs (a 128-row, 8-wave form serialised them: ~1/3 MFMA-busy, 747 vs 658 us per 524288
// rows). Same arithmetic per row as the x3 forward (qfc1 + qfc23): wave w owns columns
// [64 w, 64 w + 64) of each fc1 half and of fc2 (2 column tiles), both 32-row slabs.
constexpr int A3H_HBYTES = 2 * 64 * A3_HP * 2;  // 67,584: both H1 half planes of 64 rows
static_assert(A3H_HBYTES >= 2 * 64 * (KC1 + 8) * 2, "fc1 A staging overlays the H1 planes");
constexpr int ACT3H_LDS = A3H_HBYTES + NACT * HID2 * 4 + 64 * 4 + 64 * 8 + ACT3_OCC;  // posS, phS (DM 3: [64] uint2)
// SAVE: the learner's online forward (evx_qmlp_forward2 at B >= 32768 with the online net's act
// table): the tables' tiles start fc1 from it like the act, each half's H1 planes go to a.h1 /
// a.h1l for the backward, H2 to a.h2 and Q to a.q by batch row; X is written by x_expand_kernel.
// One 64-row tile [m0, m0 + 64) on the workgroup's 4 waves (256 threads), LDS at dsm (ACT3H_LDS
// bytes): the body of qact3h_kernel, and the fallback of the persistent act (qact3p_kernel) for
// tiles that cannot take the table path.
template <int DM = 1, bool SAVE = false>
__device__ __forceinline__ void act3h_tile(const Fwd& a, char* dsm, const int m0) {
    auto Hh = reinterpret_cast<__bf16 (*)[A3_HP]>(dsm);
    auto Hl = reinterpret_cast<__bf16 (*)[A3_HP]>(dsm + 64 * A3_HP * 2);
    auto W3s = reinterpret_cast<float (*)[HID2]>(dsm + A3H_HBYTES);
    int* posS = reinterpret_cast<int*>(dsm + A3H_HBYTES + NACT * HID2 * 4);
    uint32_t* phS = reinterpret_cast<uint32_t*>(dsm + A3H_HBYTES + NACT * HID2 * 4 + 64 * 4);
    uint4* occT = reinterpret_cast<uint4*>(dsm + A3H_HBYTES + NACT * HID2 * 4 + 64 * 4 + 64 * 8);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    ACT_ST(0);
    for (int i = tid; i < NACT * HID2; i += 256) W3s[i / HID2][i % HID2] = a.w3[i];
    if (DM == 1 && tid >= 224) {  // the tile's 32 row-pair dropout hashes (published by the barriers below)
        const int r2 = m0 + 2 * (tid - 224);
        phS[tid - 224] = r2 < a.N ? drop_row(a.drop_seed, a.drop_stream, (a.drop_row0 + (uint32_t)krow(a, r2)) >> 1) : 0u;
    }
    bool fast = false;
    if (a.stat) {  // tile-uniform: every row at the table's fire step, centre inside the map
        bool ok = true;
        if (tid < 64) {
            int pos = 0;
            if (m0 + tid < a.N) {
                const evx_obs ob = a.obs[orow(a, m0 + tid)];
                ok = min(max(ob.fire_step, 0), a.t_max) == a.stat_fs && ob.cx >= a.stat_x0 &&
                     ob.cx < a.stat_x0 + a.stat_nx && ob.cy >= 0 && ob.cy <= a.W + 1;
                pos = ok ? (ob.cx - a.stat_x0) * (a.W + 2) + ob.cy : 0;
            }
            posS[tid] = pos;
        }
        {  // the occupancy-fragment table (published by the same barrier)
            const uint32_t bits = (uint32_t)tid, one = 0x3f80u;
            uint32_t v[4];
#pragma unroll
            for (int j = 0; j < 4; j++) v[j] = ((bits >> (2 * j)) & 1u) * one | (((bits >> (2 * j + 1)) & 1u) * one) << 16;
            occT[bits] = make_uint4(v[0], v[1], v[2], v[3]);
        }
        fast = __syncthreads_and(ok);  // also publishes posS
    }
    ACT_ST(1);
    f32x16 acc2[2][2];
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc2[mt][nt][r] = 0.f;
#pragma unroll
    for (int hh = 0; hh < 2; hh++) {
        f32x16 acc[2][2];
        const int col0 = hh * 256 + w * 64;  // the wave's column tiles: col0, col0 + 32
        if (fast) {
            // fc1 = table[centre] (f32: static features x W1 + b1, x3-accurate) + the occupancy
            // columns x bits (K = 128 cells; bits exact in bf16: hi and lo weights, 2 MFMAs)
            uint32_t occ[2][4];
#pragma unroll
            for (int mt = 0; mt < 2; mt++) {
                const int row = m0 + mt * 32 + (lane & 31);
                uint4 o = make_uint4(0u, 0u, 0u, 0u);
                if (row < a.N) o = *reinterpret_cast<const uint4*>(&a.obs[orow(a, row)].occ[0]);
                occ[mt][0] = o.x;
                occ[mt][1] = o.y;
                occ[mt][2] = o.z;
                occ[mt][3] = o.w;
            }
            const uint32_t cofs = (uint32_t)(col0 + (lane & 31));
#pragma unroll
            for (int mt = 0; mt < 2; mt++)
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int rl = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const uint32_t o = (uint32_t)posS[rl] * (uint32_t)HID + cofs;
                    acc[mt][0][r] = a.stat[o];
                    acc[mt][1][r] = a.stat[o + 32];
                }
#pragma unroll 2
            for (int ks = 0; ks < 8; ks++) {  // k-step: cells 16 ks + 8 h .. + 7 of the 128
                bf16x8 bh[2], bl[2];
#pragma unroll
                for (int nt = 0; nt < 2; nt++) {
                    const size_t o = w1o_tile((col0 >> 5) + nt, ks >> 1, ks & 1) + lane * 8;
                    bh[nt] = *reinterpret_cast<const bf16x8*>(a.w1o + o);
                    bl[nt] = *reinterpret_cast<const bf16x8*>(a.w1ol + o);
                }
                const int c0 = ks * 16 + 8 * h;  // multiple of 8: the 8 bits sit in one word
#pragma unroll
                for (int mt = 0; mt < 2; mt++) {
                    const uint32_t wd = (c0 >> 5) == 0 ? occ[mt][0] : (c0 >> 5) == 1 ? occ[mt][1]
                                      : (c0 >> 5) == 2 ? occ[mt][2] : occ[mt][3];
                    const bf16x8 av = __builtin_bit_cast(bf16x8, occT[(wd >> (c0 & 31)) & 0xffu]);
#pragma unroll
                    for (int nt = 0; nt < 2; nt++) {
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bh[nt], acc[mt][nt], 0, 0, 0);
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bl[nt], acc[mt][nt], 0, 0, 0);
                    }
                }
            }
        } else {
            fc1_tile<2, 2, 4, true, 2>(a, m0, col0, false, dsm, acc);  // ends with a barrier: A buffers free
        }
        ACT_ST(2 + 4 * hh);
        float bias[2];
#pragma unroll
        for (int nt = 0; nt < 2; nt++) bias[nt] = fast ? 0.f : a.b1[col0 + nt * 32 + (lane & 31)];  // the table holds the bias
#pragma unroll
        for (int mt = 0; mt < 2; mt++)
            fc1_slab_m<2, A3_HP, true, DM>(a, acc[mt], bias, m0 + mt * 32, hh * 256, w * 64,
                                           reinterpret_cast<__bf16 (*)[A3_HP]>(&Hh[mt * 32][0]),
                                           reinterpret_cast<__bf16 (*)[A3_HP]>(&Hl[mt * 32][0]),
                                           phS + mt * 16);
        ACT_ST(3 + 4 * hh);
        __syncthreads();
        ACT_ST(4 + 4 * hh);
        if constexpr (SAVE) {  // this half's H1 planes for the backward: rows m0 .., columns 256 hh ..
            for (int i = tid; i < 2 * 64 * 32; i += 256) {
                const int pl = i >> 11, rl = (i >> 5) & 63, pc = i & 31;
                if (m0 + rl < a.N) {
                    const uint4 v = *reinterpret_cast<const uint4*>(pl ? &Hl[rl][pc * 8] : &Hh[rl][pc * 8]);
                    *reinterpret_cast<uint4*>((pl ? a.h1l : a.h1) + (size_t)(m0 + rl) * HID + hh * 256 + pc * 8) = v;
                }
            }
        }
        // fc2 over K = [256 hh, 256 hh + 256): wave w -> columns [64 w, 64 w + 64)
        bf16x8 bc[2][2], bn[2][2], lc[2][2], ln[2][2];  // [nt][s]
        auto loadB = [&](int kc, bf16x8 (&b)[2][2], bf16x8 (&l)[2][2]) {
#pragma unroll
            for (int nt = 0; nt < 2; nt++)
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    const size_t o = w2_tile(w * 2 + nt, hh * 8 + kc, s) + lane * 8;
                    b[nt][s] = *reinterpret_cast<const bf16x8*>(a.w2 + o);
                    l[nt][s] = *reinterpret_cast<const bf16x8*>(a.w2l + o);
                }
        };
        loadB(0, bc, lc);
        for (int kc = 0; kc < 8; kc++) {
            if (kc + 1 < 8) loadB(kc + 1, bn, ln);
#pragma unroll
            for (int s = 0; s < 2; s++)
#pragma unroll
                for (int mt = 0; mt < 2; mt++) {
                    const int rr = mt * 32 + (lane & 31), kk = kc * 32 + s * 16 + 8 * h;
                    const bf16x8 ah = *reinterpret_cast<const bf16x8*>(&Hh[rr][kk]);
                    const bf16x8 al = *reinterpret_cast<const bf16x8*>(&Hl[rr][kk]);
#pragma unroll
                    for (int nt = 0; nt < 2; nt++) {  // H2^T tiles (fc3t_x3): W2 as A, H1 rows as B
                        acc2[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bc[nt][s], ah, acc2[mt][nt], 0, 0, 0);
                        acc2[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lc[nt][s], ah, acc2[mt][nt], 0, 0, 0);
                        acc2[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bc[nt][s], al, acc2[mt][nt], 0, 0, 0);
                    }
                }
#pragma unroll
            for (int nt = 0; nt < 2; nt++)
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    bc[nt][s] = bn[nt][s];
                    lc[nt][s] = ln[nt][s];
                }
        }
        ACT_ST(5 + 4 * hh);
        __syncthreads();  // every wave is done with this half: the next half / H2 reuse the planes
    }
    ACT_ST(10);
    fc3t_x3(a, acc2, W3s, reinterpret_cast<float*>(dsm), m0, !SAVE);
    ACT_ST(11);
}
template <bool GR = false, int DM = 1, bool SAVE = false>
__global__ __launch_bounds__(256, 2) void qact3h_kernel(Fwd a0) {
    Fwd ag;
    if constexpr (GR) ag = fwd_net(a0, (int)blockIdx.y);
    const Fwd& a = GR ? ag : a0;
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    act3h_tile<DM, SAVE>(a, dsm, (int)blockIdx.x * 64);
}

// ------------------------------------------------------------ persistent x3 act
// DQNAgent.act (agents/dqn_agent.py:101-124), f32-accurate, for 128-row tiles on one 8-wave
// workgroup per CU (two waves per SIMD, up to 256 registers each), workgroup b looping over tiles b,
// b + grid, ...: fc1's occupancy weights and fc2's weights (hi + lo) are streamed from L2 once per
// 128 rows instead of once per 64 (act3h_tile moved ~14 KB of weights and table per row), and the
// fc1 epilogue runs under fc2's MFMAs instead of beside another workgroup's. fc1 -> H1 -> fc2 goes
// in quarters of fc1's 512 columns:
//   slot q (0..3): fc1 of quarter q (the table row of every row's window centre + the occupancy
//     columns x bits; layout of the waves below), then fc2's accumulation over quarter q - 1's
//     128 K from one LDS buffer with quarter q's epilogue (ReLU, dropout, hi / lo split) writing
//     the other buffer between its MFMAs; one barrier per slot;
//   then fc2 over quarter 3 and fc3 + epsilon-greedy (fc3p_partials / fc3p_rows), in the next
//   tile's slot 0.
// The table loads of quarter q + 1 are issued in slot q after the weight loads that fc1 waits on
// (vmcnt counts loads in issue order). Per element the same products in the same order as
// act3h_tile: Q and actions are bit-identical to the 64-row kernel (tests/test_qmlp_x3_gpu.py).
// H1 of a quarter is stored transposed, H1^T [128 k][128 rows] bf16 per plane (256-B rows, 8-B
// pieces XOR-swizzled by h1t_swz): the epilogue writes 4 consecutive rows of a column per
// ds_write_b64 (16 lanes = 16 k rows: distinct banks), and fc2 reads its B operand (rows x 8 k) with
// ds_read_b64_tr_b16 (4 k rows x 64 B per 32 lanes: distinct banks). A tile with a row off the table
// path (fire step < the table's, or a centre outside it) runs act3h_tile on its two halves.
typedef const __attribute__((address_space(1))) char gbyte;  // global-memory views (explicit: the
typedef const __attribute__((address_space(1))) float gfloat;  // bases pass through asm, which would
typedef const __attribute__((address_space(1))) bf16x8 gbf16x8;  // leave generic pointers -> flat loads)
constexpr int A3P_PL = 128 * 128;                      // bf16 elements of one H1^T plane
constexpr int A3P_HB = 2 * 2 * A3P_PL * 2;             // 2 buffers x (hi, lo) planes: 131,072 B
constexpr int A3P_W3 = A3P_HB;                         // W3, f32 [5][256]
constexpr int A3P_RED = A3P_W3 + NACT * HID2 * 4;      // fc3t_x3's partials [4][5][128] f32
constexpr int A3P_POS = A3P_RED + 4 * NACT * 128 * 4;  // table row of each tile row [2][128] (this / next tile)
constexpr int A3P_PH = A3P_POS + 2 * 128 * 4;          // row-pair dropout hashes [2][64]
constexpr int A3P_OCC = A3P_PH + 2 * 64 * 4;           // occupancy-fragment table [256] uint4
constexpr int A3P_B2 = A3P_OCC + 256 * 16;             // fc2.bias f32 [256]
constexpr int A3P_ROW = A3P_B2 + HID2 * 4;             // each tile row's output row (orow) [2][128]
constexpr int ACT3P_LDS = A3P_ROW + 2 * 128 * 4;       // 154,112 B: one workgroup per CU
static_assert(ACT3P_LDS <= 160 * 1024 && ACT3H_LDS <= A3P_HB, "LDS: the fallback tile lives in the H1 buffers");
// H1^T row k: XOR on the dword index of its 8-B pieces -- bits 4-5 <- k & 3 (the 4 k rows of a
// transposed read in distinct 16-bank blocks), bits 1-3 <- (k >> 1) & 7 (with bit 4 = k & 1: the 16
// consecutive k rows of a ds_write_b64 lane group in distinct bank pairs)
__device__ __forceinline__ int h1t_swz(int k) { return ((k & 3) << 4) | (((k >> 1) & 7) << 1); }
// bf16 offset of rows r .. r + 3 (r a multiple of 4) in H1^T row k
__device__ __forceinline__ int h1t_off(int k, int r) { return k * 128 + 2 * ((r >> 1) ^ h1t_swz(k)); }

// diagnostic build (-DEVX_ACT_STAMPS, tools/act3p_stamps.py): wave 0's s_memtime at the slot
// boundaries of every tile of every workgroup (evx_diag_act3p_stamps)
#ifdef EVX_ACT_STAMPS
constexpr int A3P_NST = 16, A3P_MAXIT = 32;
__device__ long long g_act3p_st[256 * A3P_MAXIT * A3P_NST];
#define A3P_ST(i)                                                                                        \
    do {                                                                                                 \
        if (threadIdx.x == 0 && blockIdx.x < 256 && it_ < A3P_MAXIT)                                     \
            g_act3p_st[((int)blockIdx.x * A3P_MAXIT + it_) * A3P_NST + (i)] = (long long)__builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define A3P_ST(i)
#endif
// The tiles off the table path (a row below the table's fire step, or a centre outside it), which
// qact3p_kernel skips: workgroup b checks rows [1024 b, 1024 b + 1024) (4 per thread, one round of
// loads, the same test as qact3p_kernel) and runs act3h_tile on both halves of each such 128-row tile.
// A launch with no such tile costs one round of observation loads (512 workgroups at cfg3).
// With a.rest_ws (the tiles qact3p_kernel listed): halves 2 k, 2 k + 1 of listed tile k go to workgroups
// b, b + grid, ...; a launch with no listed tile costs one load per workgroup (no atomic), else the
// last workgroup to read the count zeroes it for the next act. One workgroup per CU (one wave per SIMD): the tile
// loop's body fits the 512 registers of a lone wave (at two per SIMD it spilled ~330 VGPRs to scratch).
template <int DM>
__global__ __launch_bounds__(256, 1) void qact3h_rest_kernel(Fwd a) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    __shared__ int bad[8];
    const int tid = threadIdx.x, m0 = (int)blockIdx.x * 1024;
    int* const ws = a.rest_ws;
    int nh = 16, h0 = 0, hs = 1;  // halves h0, h0 + hs, ... below nh
    if (ws) {
        if (tid == 0) {
            const int n = __hip_atomic_load(ws, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bad[0] = n;
            // n > 0 (every workgroup sees the same count): the last to have read it zeroes both counters
            // (acq_rel: the count is read before this workgroup counts as done); n = 0: both are zero
            if (n > 0 && __hip_atomic_fetch_add(ws + 1, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                             (int)gridDim.x - 1) {
                __hip_atomic_store(ws, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(ws + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        nh = 2 * min(max(bad[0], 0), (a.N + 127) / 128);  // (bounded by the list's length)
        h0 = (int)blockIdx.x;
        hs = (int)gridDim.x;
    } else {
        if (tid < 8) bad[tid] = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int r = tid + 256 * j;
            if (m0 + r < a.N) {
                const evx_obs ob = a.obs[orow(a, m0 + r)];
                const bool ok = min(max(ob.fire_step, 0), a.t_max) == a.stat_fs && ob.cx >= a.stat_x0 &&
                                ob.cx < a.stat_x0 + a.stat_nx && ob.cy >= 0 && ob.cy <= a.W + 1;
                if (!ok) bad[r >> 7] = 1;
            }
        }
        __syncthreads();
    }
    for (int hf = h0; hf < nh; hf += hs) {  // 64-row halves (one call site: the body is inlined once); uniform
        int mh;
        if (ws) {
            mh = ws[2 + (hf >> 1)] * 128 + 64 * (hf & 1);
        } else {
            if (!bad[hf >> 1] || m0 + 64 * hf >= a.N) continue;
            mh = m0 + 64 * hf;
        }
        // the arguments re-read per half through an opaque pointer: nothing derived from them is
        // hoisted out of the loop (hoisted, ~320 VGPRs of addresses were live across it and spilled)
        const Fwd* ap = &a;
        asm volatile("" : "+s"(ap));
        const Fwd ak = *ap;
        act3h_tile<DM, false>(ak, dsm, mh);
        __syncthreads();
    }
}

// 8 waves (two per SIMD): wave w owns fc1 columns 128 q + 32 (w & 3) and fc2 columns 64 (w & 3) ..
// + 63 for the tile's rows 64 (w >> 2) .. + 63, so the two waves of a SIMD (w, w + 4) stream the same
// weight fragments and cover each other's waits. Tiles are pipelined: the next tile's rows are
// checked and its table rows (quarter 0) loaded during this tile's slots 2 and 3, and fc2 over this
// tile's quarter 3 runs in the next tile's slot 0 beside that tile's first epilogue (then fc3).
template <int DM>
__global__ __launch_bounds__(512, 2) void qact3p_kernel(Fwd a, int ntiles) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    __bf16* H = reinterpret_cast<__bf16*>(dsm);  // [buffer][plane][A3P_PL]
    __bf16* const H1b = H + 2 * A3P_PL;          // buffer 1 (odd quarters)
    auto W3s = reinterpret_cast<float (*)[HID2]>(dsm + A3P_W3);
    float* red = reinterpret_cast<float*>(dsm + A3P_RED);
    int* posS = reinterpret_cast<int*>(dsm + A3P_POS);
    uint32_t* phS = reinterpret_cast<uint32_t*>(dsm + A3P_PH);
    const uint4* occT = reinterpret_cast<const uint4*>(dsm + A3P_OCC);
    float* b2s = reinterpret_cast<float*>(dsm + A3P_B2);
    int* rowS = reinterpret_cast<int*>(dsm + A3P_ROW);
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: weight offsets stay scalar
    const int c = w & 3, rh = w >> 2;                        // column group, row half
    const int r0 = 64 * rh;                                  // the wave's first tile row
    for (int i = tid; i < NACT * HID2; i += 512) W3s[i / HID2][i % HID2] = a.w3[i];
    if (tid < HID2) b2s[tid] = a.b2[tid];
    if (tid < 256) {  // byte of 8 cell bits -> the 8 bf16 A values (0 or 1.0) of one occupancy k-step
        const uint32_t bits = (uint32_t)tid, one = 0x3f80u;
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = ((bits >> (2 * j)) & 1u) * one | (((bits >> (2 * j + 1)) & 1u) * one) << 16;
        reinterpret_cast<uint4*>(dsm + A3P_OCC)[tid] = make_uint4(v[0], v[1], v[2], v[3]);
    }
    const gbyte *w2p = (const gbyte*)a.w2, *w2lp = (const gbyte*)a.w2l;
    const gbyte *w1op = (const gbyte*)a.w1o, *w1olp = (const gbyte*)a.w1ol, *statp = (const gbyte*)a.stat;
    // tile-uniform table path of tile tt's row tid (< 128): every row at the table's fire step with its
    // centre inside the table; its table row into posS[buf], the row-pair hashes into phS[buf]
    // pre: row tid's observation and output row, loaded (else loaded here); the output rows go to rowS[buf]
    auto setup_rows = [&](int tt, int buf, bool& ok, const evx_obs* pre, int prow) {
        ok = true;
        const int mm = tt * 128;
        if (tid < 128) {
            int pos = 0;
            if (mm + tid < a.N) {
                const int orw = pre ? prow : orow(a, mm + tid);
                rowS[buf * 128 + tid] = orw;
                const evx_obs ob = pre ? *pre : a.obs[orw];
                ok = min(max(ob.fire_step, 0), a.t_max) == a.stat_fs && ob.cx >= a.stat_x0 &&
                     ob.cx < a.stat_x0 + a.stat_nx && ob.cy >= 0 && ob.cy <= a.W + 1;
                pos = ok ? (ob.cx - a.stat_x0) * (a.W + 2) + ob.cy : 0;
            }
            posS[buf * 128 + tid] = pos;
        } else if (DM == 1 && tid < 192) {
            const int r2 = mm + 2 * (tid - 128);
            phS[buf * 64 + tid - 128] =
                r2 < a.N ? drop_row(a.drop_seed, a.drop_stream, (a.drop_row0 + (uint32_t)krow(a, r2)) >> 1) : 0u;
        }
    };
    int it_ = -1;
    (void)it_;
    int tile = blockIdx.x, cur = 0, pm0 = 0, pcur = 0;
    bool ready = false;  // tile is set up in buffer cur (posS / phS), its occupancy and quarter-0 table loaded
    bool pend = false;   // the previous tile (rows pm0 ..) still owes fc2 over its quarter 3 and fc3
    f32x16 acc2[2][2];
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc2[mt][nt][r] = 0.f;
    f32x16 tab[2], acc1[2];
    uint32_t occ[2][4];
    bf16x8 wb[2][2], wl[2][2];  // fc2 weight fragments: ring of 2, one k-step ahead
    bf16x8 bh[3], bl[3];        // fc1's occupancy weight fragments: ring of 3, two k-steps ahead
    while (true) {
        it_++;
        A3P_ST(0);
        // the lane index, opaque per iteration: the per-lane offsets derived from it are formed inside
        // it (hoisted out of the tile loop, a few hundred of them were live across it and spilled)
        int lane = tid & 63;
        asm volatile("" : "+v"(lane));
        const int h = lane >> 5, j32 = lane & 31;
        const uint32_t l16 = (uint32_t)lane * 16u;  // a lane's 16 B of a 1-KB operand fragment
        // fc2's transposed B reads: lane l takes k rows 8 h + (l >> 2 & 3) (+ 4) of a k-step, rows
        // r0 + 32 mt + 16 (l >> 4 & 1) + 4 (l & 3) .. + 3 (tr_frag's addressing on the swizzled image)
        const int kq = 8 * h + ((lane >> 2) & 3), rq = r0 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
        auto trf = [&](const __bf16* plane, int ks, int mt) -> bf16x8 {
            const __bf16* b = plane + ks * 16 * 128;
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b + h1t_off(kq, 32 * mt + rq)));
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b + h1t_off(kq + 4, 32 * mt + rq)));
            const s16x4 v[2] = {lo, hi};
            return __builtin_bit_cast(bf16x8, v);
        };
        auto load_occ = [&](int mm) {
#pragma unroll
            for (int mt = 0; mt < 2; mt++) {
                const int row = mm + r0 + mt * 32 + j32;
                uint4 o = make_uint4(0u, 0u, 0u, 0u);
                if (row < a.N) o = *reinterpret_cast<const uint4*>(&a.obs[orow(a, row)].occ[0]);
                occ[mt][0] = o.x;
                occ[mt][1] = o.y;
                occ[mt][2] = o.z;
                occ[mt][3] = o.w;
            }
        };
        // table rows of quarter q (rows of posS[buf]): register r of tile mt is row r0 + 32 mt + (r & 3) +
        // 8 (r >> 2) + 4 h
        auto load_tab = [&](int buf, int q) {
            const uint32_t cofs = (uint32_t)(128 * q + 32 * c + j32) * 4u;  // + the row's table offset
#pragma unroll
            for (int mt = 0; mt < 2; mt++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const int4 p4 = *reinterpret_cast<const int4*>(&posS[buf * 128 + r0 + 32 * mt + 8 * g + 4 * h]);
                    const int pp[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
                    for (int i = 0; i < 4; i++)  // 32-bit byte offsets from the uniform base
                        tab[mt][4 * g + i] = *(const gfloat*)(statp + ((uint32_t)pp[i] * (uint32_t)(HID * 4) + cofs));
                }
        };
        auto load_w2 = [&](int q, int ks, int slot) {
#pragma unroll
            for (int nt = 0; nt < 2; nt++) {  // uniform base + (fragment offset + the lane's 16 B)
                const uint32_t o = (uint32_t)w2_tile(c * 2 + nt, 4 * q + (ks >> 1), ks & 1) * 2u + l16;
                wb[slot][nt] = *(const gbf16x8*)(w2p + o);
                wl[slot][nt] = *(const gbf16x8*)(w2lp + o);
            }
        };
        // fc1 of quarter q: acc1 = tab + occupancy columns x bits (ks ascending, hi then lo per
        // fragment, as act3h_tile); at ks 5, behind every fc1 weight load (tab was read at ks 0), the
        // table loads of the quarter after (tbuf, tq; tq < 0: none)
        // fc1 weight fragments of k-step ks of quarter q (column tile 4 q + c) into ring slot ks % 3
        auto ldw = [&](int q, int ks) {
            const uint32_t o = (uint32_t)w1o_tile(4 * q + c, ks >> 1, ks & 1) * 2u + l16;
            bh[ks % 3] = *(const gbf16x8*)(w1op + o);
            bl[ks % 3] = *(const gbf16x8*)(w1olp + o);
        };
        // (its first two k-steps' fragments were loaded by the phase before: fc2q's last k-steps)
        auto fc1q = [&](int q, int tbuf, int tq) {
#pragma unroll
            for (int ks = 0; ks < 8; ks++) {
                if (ks + 2 < 8) ldw(q, ks + 2);
                if (ks == 5 && tq >= 0) load_tab(tbuf, tq);
                const int c0 = ks * 16 + 8 * h;  // cells c0 .. c0 + 7, in word ks >> 1
#pragma unroll
                for (int mt = 0; mt < 2; mt++) {
                    const bf16x8 av = __builtin_bit_cast(bf16x8, occT[(occ[mt][ks >> 1] >> (c0 & 31)) & 0xffu]);
                    acc1[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bh[ks % 3], ks == 0 ? tab[mt] : acc1[mt], 0, 0, 0);
                    acc1[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bl[ks % 3], acc1[mt], 0, 0, 0);
                }
            }
        };
        // quarter q's epilogue for rows r0 + 32 mt + 8 g + 4 h .. + 3 of the lane's column -> H1^T (buffer Hb)
        auto epi = [&](int q, __bf16* Hb, int mt, int g) {
            const int k = 32 * c + j32, rb = r0 + 32 * mt + 8 * g + 4 * h;
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const float x = acc1[mt][4 * g + i];
                v[i] = x > 0.f ? x : 0.f;
            }
            if constexpr (DM == 1) {
                const uint2 ph = *reinterpret_cast<const uint2*>(&phS[cur * 64 + (rb >> 1)]);
                const uint32_t col = (uint32_t)(128 * q + k);
                const uint32_t h0 = drop_pair(ph.x, col), h1 = drop_pair(ph.y, col);
                v[0] = (h0 & 0xffffu) >= a.drop_thresh ? v[0] * a.drop_scale : 0.f;
                v[1] = (h0 >> 16) >= a.drop_thresh ? v[1] * a.drop_scale : 0.f;
                v[2] = (h1 & 0xffffu) >= a.drop_thresh ? v[2] * a.drop_scale : 0.f;
                v[3] = (h1 >> 16) >= a.drop_thresh ? v[3] * a.drop_scale : 0.f;
            }
            __bf16 hi[4], lo[4];
#pragma unroll
            for (int i = 0; i < 4; i++) split2(v[i], hi[i], lo[i]);
            const int o = h1t_off(k, rb);
            *reinterpret_cast<uint2*>(Hb + o) = __builtin_bit_cast(uint2, hi);
            *reinterpret_cast<uint2*>(Hb + A3P_PL + o) = __builtin_bit_cast(uint2, lo);
        };
        // fc2 over quarter qq's K from buffer Hb (k-step ks: fc2 K 128 qq + 16 ks; kc, s order as
        // act3h_tile); EPI: quarter eq's epilogue into buffer He, one row group per k-step; the last
        // k-step loads the first fragments of quarter (qq + 1) & 3 (the next tile's 0 after 3)
        // wq >= 0: the next fc1's quarter -- its first two k-steps' weight fragments (k-steps 5, 6)
        auto fc2q = [&](int qq, const __bf16* Hb, auto epi_on, int eq, __bf16* He, int wq) {
#pragma unroll
            for (int ks = 0; ks < 8; ks++) {
                if (ks + 1 < 8) load_w2(qq, ks + 1, (ks + 1) & 1);
                else load_w2((qq + 1) & 3, 0, 0);
                if (ks == 5 && wq >= 0) ldw(wq, 0);
                if (ks == 6 && wq >= 0) ldw(wq, 1);
                const int sl = ks & 1;
#pragma unroll
                for (int mt = 0; mt < 2; mt++) {
                    const bf16x8 ah = trf(Hb, ks, mt), al = trf(Hb + A3P_PL, ks, mt);
#pragma unroll
                    for (int nt = 0; nt < 2; nt++) {  // H2^T tiles (fc3t_x3): W2 as A, H1 rows as B
                        acc2[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wb[sl][nt], ah, acc2[mt][nt], 0, 0, 0);
                        acc2[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl[sl][nt], ah, acc2[mt][nt], 0, 0, 0);
                        acc2[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wb[sl][nt], al, acc2[mt][nt], 0, 0, 0);
                    }
                }
                if constexpr (decltype(epi_on)::value) epi(eq, He, ks >> 2, ks & 3);
            }
        };
        auto fc3_prev = [&]() {  // the previous tile's fc3 partials, then a fresh fc2 sum
            fc3p_partials(acc2, W3s, b2s, red, c, r0, lane);
#pragma unroll
            for (int mt = 0; mt < 2; mt++)
#pragma unroll
                for (int nt = 0; nt < 2; nt++)
#pragma unroll
                    for (int r = 0; r < 16; r++) acc2[mt][nt][r] = 0.f;
        };
        if (!ready) {  // no tile set up ahead (the first, or the one after a skipped tile)
            if (pend) {
                fc2q(3, H1b, std::false_type{}, 0, H, -1);
                fc3_prev();
                __syncthreads();
                fc3p_rows(a, red, pm0, rowS + pcur * 128);
                pend = false;
            }
            bool fast = false;
            for (; tile < ntiles; tile += gridDim.x) {
                __syncthreads();  // the last readers of posS / phS / H1 / the partials are done
                bool ok;
                setup_rows(tile, cur, ok, nullptr, 0);
                fast = __syncthreads_and(ok);
                if (fast) break;  // else qact3h_rest_kernel's: listed for it
                if (tid == 0 && a.rest_ws) {  // (a count past ntiles: a workspace not zeroed -- nothing written)
                    const int k = atomicAdd(a.rest_ws, 1);
                    if (k >= 0 && k < ntiles) a.rest_ws[2 + k] = tile;
                }
            }
            if (!fast) break;
            load_occ(tile * 128);
            load_tab(cur, 0);
            load_w2(0, 0, 0);
            ldw(0, 0);
            ldw(0, 1);
        }
        const int m0 = tile * 128;
        A3P_ST(1);
        // slot 0: fc1 of quarter 0; fc2 over the previous tile's quarter 3 with this epilogue beside it
        fc1q(0, cur, 1);
        A3P_ST(2);
        if (pend) {
            fc2q(3, H1b, std::true_type{}, 0, H, 1);
        } else {
            ldw(1, 0);
            ldw(1, 1);
#pragma unroll
            for (int mt = 0; mt < 2; mt++)
#pragma unroll
                for (int g = 0; g < 4; g++) epi(0, H, mt, g);
        }
        if (pend) fc3_prev();  // the previous tile's fc3 partials (its fc2 sum is complete)
        A3P_ST(3);
        __syncthreads();
        if (pend) fc3p_rows(a, red, pm0, rowS + pcur * 128);  // its rows: Q, epsilon-greedy
        A3P_ST(4);
        // slot 1
        fc1q(1, cur, 2);
        A3P_ST(5);
        fc2q(0, H, std::true_type{}, 1, H1b, 2);
        A3P_ST(6);
        __syncthreads();
        A3P_ST(7);
        // slot 2, and the next tile's rows checked (posS / phS of the other buffer; its observations
        // loaded at the slot's start)
        const int nt2 = tile + (int)gridDim.x;
        evx_obs obn{{0u, 0u, 0u, 0u}, 0, 0, 0, 0};
        int orn = 0;
        if (tid < 128 && nt2 < ntiles && nt2 * 128 + tid < a.N) {
            orn = orow(a, nt2 * 128 + tid);
            obn = a.obs[orn];
        }
        fc1q(2, cur, 3);
        A3P_ST(8);
        fc2q(1, H1b, std::true_type{}, 2, H, 3);
        bool okn = true;
        if (nt2 < ntiles) setup_rows(nt2, cur ^ 1, okn, &obn, orn);
        A3P_ST(9);
        const bool fast_next = __syncthreads_and(okn) && nt2 < ntiles;
        A3P_ST(10);
        // slot 3: the next tile's quarter-0 table rows (fc1q's ks 5) and occupancy after fc1
        fc1q(3, cur ^ 1, fast_next ? 0 : -1);
        if (fast_next) load_occ(nt2 * 128);
        A3P_ST(11);
        fc2q(2, H, std::true_type{}, 3, H1b, fast_next ? 0 : -1);
        A3P_ST(12);
        __syncthreads();
        A3P_ST(13);
        pend = true;
        pm0 = m0;
        pcur = cur;
        tile = nt2;
        ready = fast_next;
        if (fast_next) cur ^= 1;
    }
}

// X (the x3 compact input of every batch row, [N][640] bf16: per cell (occ | danger hi, barrier |
// exit), then the 128 cells' danger residuals) for the backward's dW1 when the online forward runs
// through the act kernel's table path -- what qfc1_kernel's staging writes as it goes (fc1_tile's
// stash). 80 16-B pieces per row (0..63: two cells' features, 64..79: eight residuals), 20 threads
// per row, each with 4 pieces t, t + 20, t + 40, t + 60: one observation load, then 4 independent
// gathers in flight (one piece per thread left the launch bound by its dependent load chain).
__global__ __launch_bounds__(256) void x_expand_kernel(Fwd a) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int row = (int)(i / 20), t = (int)(i - (int64_t)row * 20);
    if (row >= a.N) return;
    const evx_obs ob = a.obs[orow(a, row)];
    if (a.xtab && a.stat && min(max(ob.fire_step, 0), a.t_max) == a.stat_fs && ob.cx >= a.stat_x0 &&
        ob.cx < a.stat_x0 + a.stat_nx && ob.cy >= 0 && ob.cy <= a.W + 1) {
        // a table row: its static inputs are the table row's X (occupancy 0); the occupancy bits of
        // cells 2q, 2q + 1 go into the low halves of words 0 and 2 of piece q < 64 (cell_feat's encoding)
        const __bf16* src = a.xtab + (size_t)((ob.cx - a.stat_x0) * (a.W + 2) + ob.cy) * K1X;
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = *reinterpret_cast<const uint4*>(src + 8 * (t + 20 * k));
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int q = t + 20 * k;
            if (q < 64) {
                const int c0 = 2 * q, w = c0 >> 5;  // cells c0, c0 + 1 share an occupancy word
                const uint32_t ow = w == 0 ? ob.occ[0] : w == 1 ? ob.occ[1] : w == 2 ? ob.occ[2] : ob.occ[3];
                v[k].x |= c0 < NCELL ? ((ow >> (c0 & 31)) & 1u) * 0x3f80u : 0u;
                v[k].z |= c0 + 1 < NCELL ? ((ow >> ((c0 + 1) & 31)) & 1u) * 0x3f80u : 0u;
            }
            *reinterpret_cast<uint4*>(a.x + (size_t)row * K1X + 8 * q) = v[k];
        }
        return;
    }
    const int fbase = feat_base(a, ob);
    const uint32_t* fb = (a.feats ? a.feats[ob.layout] : a.feat) + fbase;
    const uint16_t* flb = (a.feats_lo ? a.feats_lo[ob.layout] : a.feat_lo) + fbase;
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int q = t + 20 * k;
        if (q < 64) {
            const uint2 f0 = cell_feat(ob, 2 * q, fb[feat_off(a, 2 * q)]);
            const uint2 f1 = cell_feat(ob, 2 * q + 1, fb[feat_off(a, 2 * q + 1)]);
            v[k] = make_uint4(f0.x, f0.y, f1.x, f1.y);
        } else {
            uint32_t w[4];
#pragma unroll
            for (int u = 0; u < 8; u += 2) {
                const int c0 = 8 * (q - 64) + u;
                const uint32_t l0 = c0 < NCELL ? (uint32_t)flb[feat_off(a, c0)] : 0u;
                const uint32_t l1 = c0 + 1 < NCELL ? (uint32_t)flb[feat_off(a, c0 + 1)] : 0u;
                w[u >> 1] = l0 | (l1 << 16);
            }
            v[k] = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) *reinterpret_cast<uint4*>(a.x + (size_t)row * K1X + 8 * (t + 20 * k)) = v[k];
}

// The learner's online (SAVE) and target forwards through the act table in one launch of 2 x the
// 64-row tiles (blockIdx.y = net), for batches whose separate launches would each fill at most one
// round of workgroups (evx_qmlp_forward2 at 8192 <= B < 32768: cfg5's B = 8192 -- one round for both
// nets instead of qfc1 + qfc23; at B = 32768 the paired form measured no faster than two launches).
template <int DM>
__global__ __launch_bounds__(256, 2) void qfwd2_kernel(Fwd a0, Fwd a1) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    if (blockIdx.y == 0) act3h_tile<DM, true>(a0, dsm, (int)blockIdx.x * 64);
    else act3h_tile<DM, false>(a1, dsm, (int)blockIdx.x * 64);
}

// ------------------------------------------------------------ fc2 + fc3
// X3: A = H1 hi / lo planes, B = fc2.weight hi / lo (3 MFMAs per fragment pair)
// MT = 1 (x3 only): 32-row tiles, twice the workgroups of a small batch (the LDS stages keep
// their 64-row shape; rows 32.. are not staged)
template <bool X3 = false, bool GR = false, int MT = 2>
__global__ __launch_bounds__(256, 2) void qfc23_kernel(Fwd a0, Fwd a1, int np) {
    static_assert(MT == 2 || X3, "32-row tiles: the x3 epilogue only");
    Fwd ag;
    if constexpr (GR) ag = fwd_net((int)blockIdx.z % np ? a1 : a0, (int)blockIdx.z / np);
    const Fwd& a = GR ? ag : (blockIdx.z ? a1 : a0);
    // A stages (row pitch 40 bf16 = 20 words: conflict-free ds_read_b128), then H2 in the same
    // bytes (pitch 4 mod 32 words: fc3_act reads conflict-free)
    constexpr int AP = 40, NPL = X3 ? 2 : 1;
    constexpr int SMB = X3 ? NPL * 2 * RM * AP * 2 : RM * (HID2 + 4) * 4;  // X3: A stages, then fc3t_x3's partials
    static_assert(NPL * 2 * RM * AP * 2 <= SMB && 4 * NACT * 64 * 4 <= SMB, "A stages / H2 / partials fit");
    __shared__ __attribute__((aligned(16))) char sm23[SMB];
    auto As = reinterpret_cast<__bf16 (*)[NPL][RM][AP]>(sm23);  // [buf][plane][row][k]
    auto Hs = reinterpret_cast<float (*)[HID2 + 4]>(sm23);
    __shared__ float W3s[NACT][HID2];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    const int m0 = blockIdx.x * (32 * MT);
    for (int i = tid; i < NACT * HID2; i += 256) W3s[i / HID2][i % HID2] = a.w3[i];
    const int gr = tid >> 2, go = (tid & 3) * 8;
    const bool stg = gr < 32 * MT;  // this thread stages A row gr
    const bool rowok = stg && m0 + gr < a.N;
    f32x16 acc[MT][2];
#pragma unroll
    for (int i = 0; i < MT; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;
    bf16x8 bc[NPL][2][2], bn[NPL][2][2];  // [plane][column tile][step]
    auto loadB = [&](int kc, bf16x8 (&b)[NPL][2][2]) {
#pragma unroll
        for (int nt = 0; nt < 2; nt++) {
            const int n = w * 64 + nt * 32;
#pragma unroll
            for (int s = 0; s < 2; s++) {  // tiled: one contiguous 1-KB block per wave load
                b[0][nt][s] = *reinterpret_cast<const bf16x8*>(a.w2 + w2_tile(n >> 5, kc, s) + lane * 8);
                if constexpr (X3) b[NPL - 1][nt][s] = *reinterpret_cast<const bf16x8*>(a.w2l + w2_tile(n >> 5, kc, s) + lane * 8);
            }
        }
    };
    auto loadA = [&](int kc, int pl) -> bf16x8 {
        bf16x8 v;
        if (rowok) {
            v = *reinterpret_cast<const bf16x8*>((pl ? a.h1l : a.h1) + (size_t)(m0 + gr) * HID + kc * 32 + go);
        } else {
#pragma unroll
            for (int t = 0; t < 8; t++) v[t] = (__bf16)0.f;
        }
        return v;
    };
    constexpr int NKC = HID / 32;
    if (stg) {
#pragma unroll
        for (int pl = 0; pl < NPL; pl++) *reinterpret_cast<bf16x8*>(&As[0][pl][gr][go]) = loadA(0, pl);
    }
    loadB(0, bc);
    __syncthreads();
    for (int kc = 0; kc < NKC; kc++) {
        const int buf = kc & 1;
        bf16x8 an[NPL];
        if (kc + 1 < NKC) {
#pragma unroll
            for (int pl = 0; pl < NPL; pl++) an[pl] = loadA(kc + 1, pl);
            loadB(kc + 1, bn);
        }
#pragma unroll
        for (int mt = 0; mt < MT; mt++)
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const bf16x8 av = *reinterpret_cast<const bf16x8*>(&As[buf][0][mt * 32 + (lane & 31)][s * 16 + 8 * h]);
                if constexpr (X3) {  // H2^T tiles (fc3t_x3): W2 as A, H1 rows as B
                    const bf16x8 al =
                        *reinterpret_cast<const bf16x8*>(&As[buf][NPL - 1][mt * 32 + (lane & 31)][s * 16 + 8 * h]);
#pragma unroll
                    for (int nt = 0; nt < 2; nt++) {
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bc[0][nt][s], av, acc[mt][nt], 0, 0, 0);
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bc[NPL - 1][nt][s], av, acc[mt][nt], 0, 0, 0);
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bc[0][nt][s], al, acc[mt][nt], 0, 0, 0);
                    }
                } else {
#pragma unroll
                    for (int nt = 0; nt < 2; nt++)
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bc[0][nt][s], acc[mt][nt], 0, 0, 0);
                }
            }
        if (kc + 1 < NKC) {
            if (stg) {
#pragma unroll
                for (int pl = 0; pl < NPL; pl++) *reinterpret_cast<bf16x8*>(&As[buf ^ 1][pl][gr][go]) = an[pl];
            }
#pragma unroll
            for (int pl = 0; pl < NPL; pl++)
#pragma unroll
                for (int nt = 0; nt < 2; nt++) {
                    bc[pl][nt][0] = bn[pl][nt][0];
                    bc[pl][nt][1] = bn[pl][nt][1];
                }
        }
        __syncthreads();
    }
    if constexpr (X3) {
        fc3t_x3<MT>(a, acc, W3s, reinterpret_cast<float*>(sm23), m0, false);  // the A stages are free
        return;
    } else {
    // H2 = relu(acc + b2) -> LDS (and HBM for the learner)
#pragma unroll
    for (int nt = 0; nt < 2; nt++) {
        const int col = w * 64 + nt * 32 + (lane & 31);
        const float bias = a.b2[col];
#pragma unroll
        for (int mt = 0; mt < 2; mt++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int rr = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                float v = acc[mt][nt][r] + bias;
                v = v > 0.f ? v : 0.f;
                Hs[rr][col] = v;
                if (a.h2 && m0 + rr < a.N) a.h2[(size_t)(m0 + rr) * HID2 + col] = v;
            }
    }
    __syncthreads();
    fc3_act(a, &Hs[gr][0], W3s, m0 + gr, rowok);
    }
}

// f32 parameters -> bf16 copies: W1 (compact K, w1_tile order) + the folded fc1 bias,
// W2 (w2_tile order), W2^T (w2t_tile order, the backward's operand)
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ w1, const float* __restrict__ b1,
                                                   const float* __restrict__ w2, __bf16* __restrict__ w1b,
                                                   float* __restrict__ b1c, __bf16* __restrict__ w2b,
                                                   __bf16* __restrict__ w2t, __bf16* __restrict__ w1o) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (w1o && i < HID * 128) {  // occupancy columns, w1o_tile order
        const int j = i & 7, l = (i >> 3) & 63, blk = i >> 9;
        const int s = blk & 1, kc = (blk >> 1) & 3, t = blk >> 3;
        const int n = t * 32 + (l & 31), c = kc * 32 + s * 16 + 8 * (l >> 5) + j;
        w1o[i] = (__bf16)(c < NCELL ? w1[n * K1 + c * 6 + 1] : 0.f);
    }
    if (i < HID * K1P) {  // destination index -> (tile, chunk, step, lane, j)
        const int j = i & 7, l = (i >> 3) & 63, blk = i >> 9;
        const int s = blk & 1, kc = (blk >> 1) % NKC1, t = blk / (2 * NKC1);
        const int n = t * 32 + (l & 31), k = kc * KC1 + s * 16 + 8 * (l >> 5) + j;
        w1b[i] = (__bf16)(k < 4 * NCELL ? w1[n * K1 + ref_col(k)] : 0.f);
    }
    if (i < HID) b1c[i] = b1[i] + (float)(__bf16)w1[i * K1 + CENTRE_COL];
    if (i < HID2 * HID) {
        const int j = i & 7, l = (i >> 3) & 63, blk = i >> 9;
        const int s = blk % 2, kc = (blk / 2) % (HID / 32), t = blk / (2 * (HID / 32));
        const int n = t * 32 + (l & 31), k = kc * 32 + s * 16 + 8 * (l >> 5) + j;
        w2b[i] = (__bf16)w2[n * HID + k];
        if (w2t) {  // w2t_tile order: columns = fc2 inputs (512), K = fc2 outputs (256)
            const int tt = blk / (2 * (HID2 / 32)), kc2 = (blk / 2) % (HID2 / 32);
            const int nn = tt * 32 + (l & 31), kk = kc2 * 32 + s * 16 + 8 * (l >> 5) + j;
            w2t[i] = (__bf16)w2[kk * HID + nn];
        }
    }
}

// X3 operand copies (evx_qmlp_pack3): W1 hi over K1X (compact K, then the danger column of
// cell c at 512 + c) and lo over the compact K, both in w1_tile order; b1c = b1 + W1[:, centre]
// in f32; W2 / W2^T hi and lo
__global__ __launch_bounds__(256) void pack3_kernel(const float* __restrict__ w1, const float* __restrict__ b1,
                                                    const float* __restrict__ w2, __bf16* __restrict__ w1b,
                                                    __bf16* __restrict__ w1l, float* __restrict__ b1c,
                                                    __bf16* __restrict__ w2b, __bf16* __restrict__ w2l,
                                                    __bf16* __restrict__ w2t, __bf16* __restrict__ w2tl) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < HID * K1X) {  // destination index -> (tile, chunk, step, lane, j), NKC1X chunks
        const int j = i & 7, l = (i >> 3) & 63, blk = i >> 9;
        const int s = blk & 1, kc = (blk >> 1) % NKC1X, t = blk / (2 * NKC1X);
        const int n = t * 32 + (l & 31), k = kc * KC1 + s * 16 + 8 * (l >> 5) + j;
        const int rc = ref_col3(k);
        const float v = rc >= 0 ? w1[n * K1 + rc] : 0.f;
        w1b[i] = (__bf16)v;
    }
    if (i < HID * K1P) {  // lo over the compact K (NKC1 chunks)
        const int j = i & 7, l = (i >> 3) & 63, blk = i >> 9;
        const int s = blk & 1, kc = (blk >> 1) % NKC1, t = blk / (2 * NKC1);
        const int n = t * 32 + (l & 31), k = kc * KC1 + s * 16 + 8 * (l >> 5) + j;
        const float v = k < 4 * NCELL ? w1[n * K1 + ref_col(k)] : 0.f;
        __bf16 hi, lo;
        split2(v, hi, lo);
        w1l[i] = lo;
    }
    if (i < HID) b1c[i] = b1[i] + w1[i * K1 + CENTRE_COL];
    if (i < HID2 * HID) {
        const int j = i & 7, l = (i >> 3) & 63, blk = i >> 9;
        const int s = blk % 2, kc = (blk / 2) % (HID / 32), t = blk / (2 * (HID / 32));
        const int n = t * 32 + (l & 31), k = kc * 32 + s * 16 + 8 * (l >> 5) + j;
        split2(w2[n * HID + k], w2b[i], w2l[i]);
        if (w2t) {  // w2t_tile order: columns = fc2 inputs (512), K = fc2 outputs (256)
            const int tt = blk / (2 * (HID2 / 32)), kc2 = (blk / 2) % (HID2 / 32);
            const int nn = tt * 32 + (l & 31), kk = kc2 * 32 + s * 16 + 8 * (l >> 5) + j;
            split2(w2[kk * HID + nn], w2t[i], w2tl[i]);
        }
    }
}

// X3 act fast path operands: fc1's occupancy columns (reference channel 1 of cells 0..127,
// >= 121 zero) as hi / lo bf16 pairs, w1o_tile order (K = 128 in 4 chunks of 32)
__global__ __launch_bounds__(256) void pack_occ3_kernel(const float* __restrict__ w1, __bf16* __restrict__ w1o,
                                                        __bf16* __restrict__ w1ol) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= HID * 128) return;
    const int j = i & 7, l = (i >> 3) & 63, blk = i >> 9;
    const int s = blk & 1, kc = (blk >> 1) & 3, t = blk >> 3;
    const int n = t * 32 + (l & 31), c = kc * 32 + s * 16 + 8 * (l >> 5) + j;
    __bf16 hi = (__bf16)0.f, lo = (__bf16)0.f;
    if (c < NCELL) split2(w1[n * K1 + c * 6 + 1], hi, lo);
    w1o[i] = hi;
    w1ol[i] = lo;
}

// ================================================================ backward
// DQNAgent.learn's loss.backward() for the MLP (agents/dqn_agent.py:150-158):
//   fc3: dW3 = dQ^T H2, db3 = sum dQ, dZ2 = (dQ W3) * [H2 > 0], db2 = sum dZ2
//   fc2: dW2 = dZ2^T H1, dZ1 = (dZ2 W2) * scale * [H1 > 0], db1 = sum dZ1
//        ([H1 > 0] is keep AND relu' since H1 = keep * scale * relu(z))
//   fc1: dW1 = dZ1^T X over the compact K, scattered to the reference's columns;
//        the constant centre column (channel 5, x = 1) gets sum dZ1 = db1, channel 0
//        (x = 0) gets nothing
// Every gradient sum is ordered (no f32 atomics, the same bits on every run): the weight
// gradients by split-K partials (gemm_tn_body), the fc3 / bias sums by per-block partials
// (p3: qbwd3, pz1: qdz1), all added in a fixed order by reduce2_kernel.
struct Bwd {
    int B;
    const float* dq;    // [B][5]
    const float* h2;    // [B][256]
    const __bf16* h1;   // [B][512]
    const __bf16* x;    // [B][512] compact K (qfc1's X)
    const float* w3;    // [5][256]
    const __bf16* w2t;  // fc2.weight^T in w2t_tile order
    float scale;
    __bf16* dz2;        // [B][256]
    __bf16* dz1;        // [B][512]
    float *gw1, *gb1, *gw2, *gb2, *gw3, *gb3;
    // X3: lo planes of h1 / dz2 / dz1, fc2.weight^T lo; x is [B][640]
    const __bf16* h1l;
    const __bf16* w2tl;
    __bf16* dz2l;
    __bf16* dz1l;
    float* p3;    // qbwd3 block partials [nb3][P3W]: dW3 [5][256], db2 [256], db3 [5], TD loss
    float* pz1;   // qdz1 column-sum partials [ndzx][512] (db1 = the centre column of dW1)
    int64_t gsP;  // grouped: floats between consecutive nets' partial regions
    // TD step inside qbwd3 (td != 0; else dq is given): DQNAgent.learn's target and MSE
    // (agents/dqn_agent.py:143-151) per row from Q, Qt, act, rew, done (and importance weights w)
    int td;
    const float *Q, *Qt, *rew, *w;
    const int32_t* act;
    const uint8_t* done;
    float gamma;
    float* td_abs;
};
// net g's view of a blocked grouped backward (see fwd_net; x3: two planes per activation)
__device__ __forceinline__ Bwd bwd_net(const Bwd& a0, int g) {
    Bwd a = a0;
    const size_t G = (size_t)g, B = (size_t)a.B;
    a.dq += G * B * NACT;
    a.h2 += G * B * HID2;
    a.h1 += G * 2 * B * HID;
    a.h1l = a.h1 + B * HID;
    a.x += G * B * K1X;
    a.w3 += G * NPAR;
    a.w2t += G * HID2 * HID;
    a.w2tl += G * HID2 * HID;
    a.dz2 += G * 2 * B * HID2;
    a.dz2l = a.dz2 + B * HID2;
    a.dz1 += G * 2 * B * HID;
    a.dz1l = a.dz1 + B * HID;
    a.gw1 += G * NPAR;
    a.gb1 += G * NPAR;
    a.gw2 += G * NPAR;
    a.gb2 += G * NPAR;
    a.gw3 += G * NPAR;
    a.gb3 += G * NPAR;
    a.p3 += G * a.gsP;
    a.pz1 += G * a.gsP;
    return a;
}

// fc3 backward: thread n of a 128-row block walks the rows (coalesced over n) in chunks of 32.
// The block's fc3 gradients leave as one partial row p3[block] (P3W floats: dW3, db2, db3),
// summed over blocks in block order by reduce2_kernel (f32 atomics here made the learn chain
// differ between same-seed runs at the ulp level).
// Small batches take rb = 64 or 32 rows per block (qbwd3_rows: B = 4096 had 32 blocks).
constexpr int R3 = 128, R3C = 32;
constexpr int P3W = NACT * HID2 + HID2 + 8;  // dW3 [5][256] | db2 [256] | db3 [5] | TD loss (+ pad)
constexpr int P3G = NACT * HID2 + HID2 + NACT;  // gradient columns of a p3 row; column P3G: the TD loss
// (B = 4096: 16-row blocks, learn 115.4 -> 114.3 us with dW1's 16 splits below)
inline int qbwd3_rows(int B) { return B >= 16384 ? 128 : B >= 8192 ? 64 : B > 2048 ? 16 : 32; }
template <bool X3 = false, bool GR = false>  // GR: blockIdx.y = net
__global__ __launch_bounds__(256) void qbwd3_kernel(Bwd a0, int rb) {
    Bwd ag;
    if constexpr (GR) ag = bwd_net(a0, (int)blockIdx.y);
    const Bwd& a = GR ? ag : a0;
    __shared__ float dqs[R3][NACT];
    __shared__ float lred[R3];
    const int n = threadIdx.x, b0 = blockIdx.x * rb;
    if (a.td) {  // thread n < rb: row b0 + n's TD error -> its dQ row and squared error (the mean over B)
        if (n < rb) {
            const int i = b0 + n;
            float part = 0.f;
            float dq[NACT];
#pragma unroll
            for (int t = 0; t < NACT; t++) dq[t] = 0.f;
            if (i < a.B) {
                float mx = a.Qt[(size_t)i * NACT];
#pragma unroll
                for (int j = 1; j < NACT; j++) mx = fmaxf(mx, a.Qt[(size_t)i * NACT + j]);
                const float y = a.rew[i] + a.gamma * mx * (a.done[i] ? 0.f : 1.f);
                const int ai = a.act[i];
                const float d = a.Q[(size_t)i * NACT + ai] - y;
                const float wi = a.w ? a.w[i] : 1.f;
                part = a.w ? wi * (d * d) : d * d;
                const float gd = a.w ? wi * (2.f * d) : 2.f * d;
#pragma unroll
                for (int t = 0; t < NACT; t++) dq[t] = t == ai ? gd / (float)a.B : 0.f;
                if (a.td_abs) a.td_abs[i] = fabsf(d);
            }
#pragma unroll
            for (int t = 0; t < NACT; t++) dqs[n][t] = dq[t];
            lred[n] = part;
        }
    } else {
        for (int i = n; i < rb * NACT; i += 256) {
            const int r = i / NACT;
            dqs[r][i - r * NACT] = b0 + r < a.B ? a.dq[(size_t)(b0 + r) * NACT + (i - r * NACT)] : 0.f;
        }
    }
    __syncthreads();
    if (a.td && n == 0) {  // the block's squared errors in row order
        float l = 0.f;
        for (int r = 0; r < rb; r++) l += lred[r];
        a.p3[(size_t)blockIdx.x * P3W + P3G] = l;
    }
    float w3[NACT], gw[NACT], gb2 = 0.f;
#pragma unroll
    for (int t = 0; t < NACT; t++) {
        w3[t] = a.w3[t * HID2 + n];
        gw[t] = 0.f;
    }
    // each full 32-row chunk loads its H2 values before any use (the stores into dz2 keep the
    // compiler from hoisting them)
    auto row = [&](int r, float hv) {
        float dz = 0.f;
#pragma unroll
        for (int t = 0; t < NACT; t++) {
            const float d = dqs[r][t];
            gw[t] += d * hv;
            dz += d * w3[t];
        }
        dz = hv > 0.f ? dz : 0.f;
        if constexpr (X3) {
            split2(dz, a.dz2[(size_t)(b0 + r) * HID2 + n], a.dz2l[(size_t)(b0 + r) * HID2 + n]);
        } else {
            a.dz2[(size_t)(b0 + r) * HID2 + n] = (__bf16)dz;
        }
        gb2 += dz;
    };
    if (rb == 16 && b0 + 16 <= a.B) {  // small batches: 16-row blocks, loads batched the same way
        float hvr[16];
#pragma unroll
        for (int r = 0; r < 16; r++) hvr[r] = a.h2[(size_t)(b0 + r) * HID2 + n];
#pragma unroll
        for (int r = 0; r < 16; r++) row(r, hvr[r]);
    } else
    for (int c0 = 0; c0 < rb; c0 += R3C) {
        if (c0 + R3C <= rb && b0 + c0 + R3C <= a.B) {
            float hvr[R3C];
#pragma unroll
            for (int r = 0; r < R3C; r++) hvr[r] = a.h2[(size_t)(b0 + c0 + r) * HID2 + n];
#pragma unroll
            for (int r = 0; r < R3C; r++) row(c0 + r, hvr[r]);
        } else {
            for (int r = c0; r < rb && b0 + r < a.B; r++) row(r, a.h2[(size_t)(b0 + r) * HID2 + n]);
            break;
        }
    }
    float* pr = a.p3 + (size_t)blockIdx.x * P3W;
#pragma unroll
    for (int t = 0; t < NACT; t++) pr[t * HID2 + n] = gw[t];
    pr[NACT * HID2 + n] = gb2;
    if (n < NACT) {
        float s = 0.f;
        for (int r = 0; r < rb; r++) s += dqs[r][n];
        pr[NACT * HID2 + HID2 + n] = s;
    }
}

// dZ1 = (dZ2 W2) * scale * [H1 > 0]: 64-row tiles x 128 columns per workgroup (4 waves x
// 32 columns), K = 256. A tile's whole dZ2 block (64 x 256, x3: both planes) is staged in LDS
// at once and the next tile's is fetched into registers while this one's MFMAs run; the W2^T
// fragments stream from L2 four k-steps ahead. (Chunks of 32 k with one barrier each left
// every chunk waiting out a memory latency with one wave per SIMD: 120 us at B = 32768.)
constexpr int QZ_P = HID2 + 8;  // LDS row pitch (bf16): 528 B, conflict-free ds_read_b128 rows
constexpr int QZ_CP = 128 + 8;  // the dZ1 tile's row pitch (bf16)
constexpr int QZ_RM = 32;        // rows per dZ1 tile
static_assert(QZ_CP <= QZ_P, "each dZ1 plane overlays a dZ2 plane");
template <bool X3>
constexpr int qdz1_lds_bytes() { return (X3 ? 2 : 1) * QZ_RM * QZ_P * 2 + 2 * QZ_RM * 16; }  // + 2 tiles of [H1 > 0] bits
// Row tiles per qdz1 workgroup: the tiles' column sums (db1 and the centre column of dW1) leave
// as one partial row pz1[bx] per workgroup row, which reduce2_kernel adds in bx order; fewer,
// longer workgroups keep that reduction short. Up to QZ_RT tiles per workgroup while the grid
// keeps >= 256 qdz1 workgroups (qdz1_tiles_per_wg; B = 32768: 8, 8192: 2, 4096: 1).
constexpr int QZ_RT = 8;
inline int qdz1_tiles_per_wg(int B) { return B / 4096 < 1 ? 1 : (B / 4096 > QZ_RT ? QZ_RT : B / 4096); }
template <bool X3 = false>
__device__ __forceinline__ void qdz1_body(const Bwd& a, char* smem, int bx, int by, int ndzx) {
    constexpr int NPL = X3 ? 2 : 1;
    auto As = reinterpret_cast<__bf16 (*)[QZ_RM][QZ_P]>(smem);  // [NPL][QZ_RM][QZ_P]
    // [H1 > 0] of the tile's rows x 128 columns as bits (byte b of a row: columns 8b .. 8b + 7),
    // double-buffered by tile parity: H1 arrives with dZ2 in 16-B row pieces instead of the
    // 2-B loads of the accumulator layout (which cost 75 us at B = 32768)
    auto Ms = reinterpret_cast<uint32_t (*)[QZ_RM][4]>(smem + NPL * QZ_RM * QZ_P * 2);  // [2][QZ_RM][4]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    const int n0 = by * 128 + w * 32, col = n0 + (lane & 31);
    const int nrt = (a.B + QZ_RM * ndzx - 1) / (QZ_RM * ndzx);  // row tiles per workgroup
    const int t0 = bx * nrt, nt = min(nrt, (a.B + QZ_RM - 1) / QZ_RM - t0);
    constexpr int DP = QZ_RM * 32 / 256;  // dZ2 16-B pieces per thread and plane (a row: 32 pieces)
    constexpr int HP = QZ_RM * 16 / 256;  // H1 (and dZ1) 16-B pieces per thread and plane (a row: 16)
    // W2^T of the wave's 32 columns, every k-step, hi and lo: held in registers for all the workgroup's
    // row tiles (weight-stationary: streamed from L2 per 64-row tile it moved 128 KB per tile)
    bf16x8 bw[HID2 / 16][NPL];
#pragma unroll
    for (int ks = 0; ks < HID2 / 16; ks++) {
        const size_t o = w2t_tile(n0 >> 5, ks >> 1, ks & 1) + lane * 8;
        bw[ks][0] = *reinterpret_cast<const bf16x8*>(a.w2t + o);
        if constexpr (X3) bw[ks][NPL - 1] = *reinterpret_cast<const bf16x8*>(a.w2tl + o);
    }
    // staging: 16-B piece j of thread t = (row c >> 5, k 8 (c & 31)) for c = t + 256 j
    uint4 pre[NPL][DP], hpre[HP];
    auto fetch = [&](int m0) {
#pragma unroll
        for (int j = 0; j < HP; j++) {  // H1 piece j: row (c >> 4), columns 128 by + 8 (c & 15), c = t + 256 j
            const int c = tid + 256 * j, row = m0 + (c >> 4);
            hpre[j] = make_uint4(0u, 0u, 0u, 0u);
            if (row < a.B) hpre[j] = *reinterpret_cast<const uint4*>(a.h1 + (size_t)row * HID + by * 128 + (c & 15) * 8);
        }
#pragma unroll
        for (int p = 0; p < NPL; p++)
#pragma unroll
            for (int j = 0; j < DP; j++) {
                const int c = tid + 256 * j, row = m0 + (c >> 5);
                pre[p][j] = make_uint4(0u, 0u, 0u, 0u);
                if (row < a.B) pre[p][j] = *reinterpret_cast<const uint4*>((p ? a.dz2l : a.dz2) + (size_t)row * HID2 + (c & 31) * 8);
            }
    };
    constexpr int NKS = HID2 / 16;
    float cs = 0.f;
    if (nt > 0) fetch(t0 * QZ_RM);
    for (int t = 0; t < nt; t++) {
        const int m0 = (t0 + t) * QZ_RM;
#pragma unroll
        for (int p = 0; p < NPL; p++)
#pragma unroll
            for (int j = 0; j < DP; j++) {
                const int c = tid + 256 * j;
                *reinterpret_cast<uint4*>(&As[p][c >> 5][(c & 31) * 8]) = pre[p][j];
            }
#pragma unroll
        for (int j = 0; j < HP; j++) {
            const int c = tid + 256 * j;
            const uint32_t wv[4] = {hpre[j].x, hpre[j].y, hpre[j].z, hpre[j].w};
            uint32_t bits = 0u;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                bits |= (__builtin_bit_cast(float, wv[e] << 16) > 0.f ? 1u : 0u) << (2 * e);
                bits |= (__builtin_bit_cast(float, wv[e] & 0xffff0000u) > 0.f ? 1u : 0u) << (2 * e + 1);
            }
            reinterpret_cast<uint8_t*>(&Ms[t & 1][c >> 4][0])[c & 15] = (uint8_t)bits;
        }
        __syncthreads();
        if (t + 1 < nt) fetch(m0 + QZ_RM);
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; r++) acc[r] = 0.f;
#pragma unroll
        for (int ks = 0; ks < NKS; ks++) {
            const bf16x8 av = *reinterpret_cast<const bf16x8*>(&As[0][lane & 31][ks * 16 + 8 * h]);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bw[ks][0], acc, 0, 0, 0);
            if constexpr (X3) {
                const bf16x8 al = *reinterpret_cast<const bf16x8*>(&As[NPL - 1][lane & 31][ks * 16 + 8 * h]);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bw[ks][NPL - 1], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bw[ks][0], acc, 0, 0, 0);
            }
        }
        __syncthreads();  // every wave is done with the tile's dZ2: its LDS takes the dZ1 tile
        // dZ1 (hi / lo planes) through LDS over the dZ2 image, so that it leaves in 16-B row
        // pieces rather than 2-B stores of the accumulator layout
        auto Cs = reinterpret_cast<__bf16 (*)[QZ_RM][QZ_CP]>(smem);  // [NPL][QZ_RM][QZ_CP]
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
            const bool pos = (Ms[t & 1][rl][w] >> (lane & 31)) & 1u;
            const float v = pos && m0 + rl < a.B ? acc[r] * a.scale : 0.f;
            if constexpr (X3) {
                split2(v, Cs[0][rl][w * 32 + (lane & 31)], Cs[NPL - 1][rl][w * 32 + (lane & 31)]);
            } else {
                Cs[0][rl][w * 32 + (lane & 31)] = (__bf16)v;
            }
            cs += v;
        }
        __syncthreads();
#pragma unroll
        for (int p = 0; p < NPL; p++)
#pragma unroll
            for (int j = 0; j < HP; j++) {  // piece j: row c >> 4, columns 8 (c & 15), c = t + 256 j
                const int c = tid + 256 * j, row = m0 + (c >> 4);
                if (row < a.B)
                    *reinterpret_cast<uint4*>((p ? a.dz1l : a.dz1) + (size_t)row * HID + by * 128 + (c & 15) * 8) =
                        *reinterpret_cast<const uint4*>(&Cs[p][c >> 4][(c & 15) * 8]);
            }
        __syncthreads();  // the dZ1 image has been read: the next tile's dZ2 may be stashed
    }
    cs += __shfl_xor(cs, 32, 64);  // the two row halves of the column
    if (h == 0) a.pz1[(size_t)bx * HID + col] = cs;  // db1 = d/dW1 of the constant centre input
}

// C[m][n] += sum_k A[k][m] B[k][n] (both operands K-major bf16), 128x128 tiles of
// 4 waves (2x2 of 64x64), K chunks of 64 staged in LDS in their memory order ([k][m]) and
// read back by ds_read_b64_tr_b16, which hands every lane the 4 consecutive k of its column:
// no transpose in registers (the 8x8 VALU shuffle this replaced cost about as many cycles
// as the chunk's MFMAs). gridDim.z splits K: split z stores its tile to part[z][m][0, gridDim.x
// * TT) and reduce2_kernel adds the splits in z order into C (deterministic, and no atomic
// traffic through L2), columns n >= Nc skipped, remap: column n goes to ref_col(n) (fc1's
// compact K -> the reference's 726).
// LDS image of a plane: [TKC][TPT] bf16, 320-B rows: a transposed read's 32-lane half takes
// 4 rows x 64 B at banks 16 q + [0, 16) -- conflict-free (cdna_hip_programming.md T10)
constexpr int TT = 128, TKC = 64, TPT = TT + 32;
// the 32x32x16 operand fragment of rows (columns of the image) c0 .. c0 + 31, k = k0 .. k0 + 15:
// lane l gets column c0 + (l & 31), k = k0 + 8 (l >> 5) + 0 .. 7 (two transposed reads; lane
// 4q + p of each 16-lane group addresses row q of a 4-row block, columns 4p .. 4p + 3)
__device__ __forceinline__ bf16x8 tr_frag(const __bf16* img, int lane_off, int k0, int c0) {
    const __bf16* p0 = img + k0 * TPT + c0 + lane_off;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0 + 4 * TPT));
    const s16x4 v[2] = {lo, hi};
    return __builtin_bit_cast(bf16x8, v);
}
// AP / BP: planes of A / B (2 = X3 hi + lo at Al / Bl: products hi*hi + hi*lo + lo*hi).
// one weight-gradient GEMM of the backward (gemm_tn_kernel's arguments; grid = (N tiles, M tiles, splits))
struct GemmTN {
    const __bf16* A;
    int lda;
    const __bf16* Bm;
    int ldb, K, M, Nc, kper;
    float* C;
    int ldc, remap;
    float* part;
    const __bf16 *Al, *Bl;
    int gx, gy, gz;  // grid
    int64_t gsA, gsB, gsC, gsP;  // grouped: elements between consecutive nets' A (Al), B (Bl), C, part
};
__device__ __forceinline__ GemmTN tn_net(const GemmTN& g0, int g) {
    GemmTN t = g0;
    t.A += g * t.gsA;
    t.Al = adv(t.Al, (size_t)(g * t.gsA));
    t.Bm += g * t.gsB;
    t.Bl = adv(t.Bl, (size_t)(g * t.gsB));
    t.C += g * t.gsC;
    t.part = adv(t.part, (size_t)(g * t.gsP));
    return t;
}
template <int AP, int BP>
constexpr int gemm_tn_lds_bytes() { return (AP + BP) * TKC * TPT * 2; }
template <int AP = 1, int BP = 1>
__device__ __forceinline__ void gemm_tn_body(const GemmTN& g, char* smem, int bx, int by, int bz) {
    constexpr int NP = AP + BP;  // planes staged per chunk: A's, then B's
    auto img = reinterpret_cast<__bf16 (*)[TKC][TPT]>(smem);  // [NP][TKC][TPT]
    const __bf16* __restrict__ A = g.A;
    const __bf16* __restrict__ Bm = g.Bm;
    const int lda = g.lda, ldb = g.ldb, K = g.K, M = g.M, kper = g.kper;
    float* __restrict__ part = g.part;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    const int wm = w >> 1, wn = w & 1;
    const int m0 = by * TT, n0 = bx * TT;
    const int kb0 = bz * kper, ke = min(K, kb0 + kper);
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;
    // staging: thread t moves 16 B (8 columns) of rows (t >> 4) + 16 j of every plane; a
    // 16-lane group reads one 256-B row segment (whole cache lines)
    const int sr = tid >> 4, sc = (tid & 15) * 8;
    const __bf16* src[NP];
    int ld[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) {
        src[p] = p < AP ? (p == 0 ? A : g.Al) + m0 + sc : (p == AP ? Bm : g.Bl) + n0 + sc;
        ld[p] = p < AP ? lda : ldb;
    }
    uint4 rv[NP][4];
    auto fetch = [&](int k0) {
#pragma unroll
        for (int p = 0; p < NP; p++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int k = k0 + sr + 16 * j;
                rv[p][j] = make_uint4(0u, 0u, 0u, 0u);
                if (k < ke) rv[p][j] = *reinterpret_cast<const uint4*>(src[p] + (size_t)k * ld[p]);
            }
    };
    auto stash = [&]() {
#pragma unroll
        for (int p = 0; p < NP; p++)
#pragma unroll
            for (int j = 0; j < 4; j++) *reinterpret_cast<uint4*>(&img[p][sr + 16 * j][sc]) = rv[p][j];
    };
    const int q = (lane >> 2) & 3, pq = lane & 3;
    const int lane_off = (8 * h + q) * TPT + 16 * ((lane >> 4) & 1) + 4 * pq;
    if (kb0 < ke) fetch(kb0);
    for (int k0 = kb0; k0 < ke; k0 += TKC) {
        stash();
        __syncthreads();
        if (k0 + TKC < ke) fetch(k0 + TKC);
#pragma unroll
        for (int s = 0; s < TKC / 16; s++) {
            bf16x8 av[AP][2], bv[BP][2];
#pragma unroll
            for (int i = 0; i < 2; i++) {
#pragma unroll
                for (int p = 0; p < AP; p++) av[p][i] = tr_frag(&img[p][0][0], lane_off, s * 16, wm * 64 + i * 32);
#pragma unroll
                for (int p = 0; p < BP; p++) bv[p][i] = tr_frag(&img[AP + p][0][0], lane_off, s * 16, wn * 64 + i * 32);
            }
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[0][j], acc[i][j], 0, 0, 0);
                    if constexpr (BP > 1)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[BP - 1][j], acc[i][j], 0, 0, 0);
                    if constexpr (AP > 1)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[AP - 1][i], bv[0][j], acc[i][j], 0, 0, 0);
                }
        }
        __syncthreads();
    }
    const int Np = g.gx * TT;
    float* pz = part + (size_t)bz * M * Np;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int n = n0 + wn * 64 + j * 32 + (lane & 31);
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < M) pz[(size_t)m * Np + n] = acc[i][j][r];
            }
    }
}
// XCD-aware placement of a split-K launch's block b (linear over tiles x splits): blocks are
// dealt round-robin over the 8 XCDs (b and b + 8 share one), so block x + 8 j takes split
// x + 8 (j / T) and tile j % T -- the T tiles of one K split run on one XCD and share its L2,
// where the A and B chunks they have in common are fetched once instead of once per tile from
// the Infinity Cache (dW1: 5 column tiles re-read each A chunk, 4 row tiles each B chunk).
// gz not a multiple of 8: plain order.
__device__ __forceinline__ void tn_place(int b, int gx, int gy, int gz, int& bx, int& by, int& bz) {
    const int T = gx * gy;
    int tile;
    if ((gz & 7) == 0) {
        const int x = b & 7, j = b >> 3;
        bz = x + 8 * (j / T);
        tile = j % T;
    } else {
        bz = b / T;
        tile = b - bz * T;
    }
    by = tile / gx;
    bx = tile - by * gx;
}
template <int AP = 1, int BP = 1, bool GR = false>  // GR: blockIdx.z = net * gz + split; else a 1-D grid (tn_place)
__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(GemmTN g) {
    __shared__ __attribute__((aligned(16))) char smem[gemm_tn_lds_bytes<AP, BP>()];
    if constexpr (GR) {
        const int nz = (int)blockIdx.z / g.gz;
        gemm_tn_body<AP, BP>(tn_net(g, nz), smem, blockIdx.x, blockIdx.y, (int)blockIdx.z - nz * g.gz);
    } else {
        int bx, by, bz;
        tn_place((int)blockIdx.x, g.gx, g.gy, g.gz, bx, by, bz);
        gemm_tn_body<AP, BP>(g, smem, bx, by, bz);
    }
}
// dZ1 (qdz1) and dW2 = dZ2^T H1 (gemm_tn) in one launch: both need only qbwd3's outputs. Blocks
// [0, ndz) run qdz1 tiles (grid ndzx x HID / 128), the rest the dW2 split-K tiles; the LDS is one
// dynamic buffer sized for the larger of the two.
template <bool X3, int AP, int BP, bool GR = false>  // GR: blockIdx.y = net
__global__ __launch_bounds__(256, 2) void bwd_mid_kernel(Bwd a, int ndzx, GemmTN g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int b = (int)blockIdx.x, ndz = ndzx * (HID / 128);
    if (b < ndz) {
        if constexpr (GR) qdz1_body<X3>(bwd_net(a, (int)blockIdx.y), smem, b % ndzx, b / ndzx, ndzx);
        else qdz1_body<X3>(a, smem, b % ndzx, b / ndzx, ndzx);
    } else {
        const int t = b - ndz, gxy = g.gx * g.gy;  // ndz a multiple of 8 (B >= 4096): t keeps b's XCD
        if constexpr (GR) {
            gemm_tn_body<AP, BP>(tn_net(g, (int)blockIdx.y), smem, t % g.gx, (t % gxy) / g.gx, t / gxy);
        } else {
            int bx, by, bz;
            tn_place(t, g.gx, g.gy, g.gz, bx, by, bz);
            gemm_tn_body<AP, BP>(g, smem, bx, by, bz);
        }
    }
}

// Both split-K reductions of the backward (dW2 then dW1) in one launch, each workgroup also
// leaving the sum of squares of the final gradient values it produced (clip_grad_norm_'s
// partials; fixed order). The last workgroup adds the squares of the small gradients the
// other kernels finished (b1, the centre column of W1, b2, W3, b3); W1's channel-0 and
// non-centre channel-5 columns stay zero.
struct Red2 {
    const float* part2;  // dW2 partials [S2][HID2][HID]
    int S2;
    const float* part1;  // dW1 partials [S1][HID][Np1]
    int S1, Np1, Nc1, remap1;
    float *gw1, *gb1, *gw2, *gb2, *gw3, *gb3;  // gradients
    float* ss;           // [gridDim.x] squared-norm partials, or NULL
    int nb2, nb1;        // workgroups of the two reductions
    int64_t gsP;         // grouped (blockIdx.y = net): floats between consecutive nets' partials
    const float* p3;     // qbwd3's block partials [nb3][P3W]
    int nb3;
    const float* pz1;    // qdz1's column-sum partials [nz1][HID]
    int nz1;
    int acc;             // 1: the sums are added to the gradients; 0: they overwrite them (and W1's
                         // columns of constant inputs -- channel 0, channel 5 off the centre -- are zeroed)
    float* loss;         // qbwd3's TD step: loss[0] = the block partials' sum / B, or NULL
    int B;
};
// the small sums (dW3, db2, db3 from p3; db1 and W1's centre column from pz1): 16 columns per
// workgroup, the partial rows in 16 contiguous groups (16 lanes each), groups added in order (with
// 64 columns x 4 groups each thread's 64-load chain of qbwd3's 256 block rows at B = 32768 was the
// launch's tail)
constexpr int P3L = NACT * HID2 + HID2 + NACT + 1;  // live columns of a p3 row (the gradients, the TD loss)
constexpr int RSC = 16;                             // columns per small-sum workgroup
constexpr int NRS3 = (P3L + RSC - 1) / RSC, NRSZ = HID / RSC, NRSMALL = NRS3 + NRSZ;
__device__ __forceinline__ float red_sum256(float x, float* red) {
    red[threadIdx.x] = x;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    return red[0];
}
__global__ __launch_bounds__(256) void reduce2_kernel(Red2 r0) {
    __shared__ float red[256];
    Red2 r = r0;
    if (blockIdx.y) {  // grouped: net blockIdx.y's partials, gradients and norm partials
        const size_t G = blockIdx.y;
        r.part2 += G * r.gsP;
        r.part1 += G * r.gsP;
        r.gw1 += G * NPAR; r.gb1 += G * NPAR; r.gw2 += G * NPAR;
        r.gb2 += G * NPAR; r.gw3 += G * NPAR; r.gb3 += G * NPAR;
        r.ss = adv(r.ss, G * gridDim.x);
        r.p3 += G * r.gsP;
        r.pz1 += G * r.gsP;
        r.loss = adv(r.loss, G);
    }
    const int b = (int)blockIdx.x;
    float sq = 0.f;
    if (b < r.nb2) {  // dW2: 4 columns per thread
        const int q = b * 256 + (int)threadIdx.x, nq = HID >> 2;
        if (q < HID2 * nq) {
            const int m = q / nq, n = (q - m * nq) * 4;
            const float* src = r.part2 + (size_t)m * HID + n;
            float4 acc = *reinterpret_cast<const float4*>(src);
#pragma unroll 16
            for (int z = 1; z < r.S2; z++) {  // unrolled: 16 loads in flight, the adds still in z order
                const float4 v = *reinterpret_cast<const float4*>(src + (size_t)z * HID2 * HID);
                acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
            }
            float* dst = r.gw2 + (size_t)m * HID + n;
            const float4 old = r.acc ? *reinterpret_cast<const float4*>(dst) : make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 o = make_float4(old.x + acc.x, old.y + acc.y, old.z + acc.z, old.w + acc.w);
            *reinterpret_cast<float4*>(dst) = o;
            sq = o.x * o.x + o.y * o.y + o.z * o.z + o.w * o.w;
        }
    } else if (b < r.nb2 + r.nb1) {  // dW1: 4 compact columns (one cell) per thread
        const int q = (b - r.nb2) * 256 + (int)threadIdx.x, nq = r.Nc1 >> 2;
        if (q < HID * nq) {
            const int m = q / nq, n = (q - m * nq) * 4;
            const size_t zs = (size_t)HID * r.Np1;
            const float* src = r.part1 + (size_t)m * r.Np1 + n;
            float4 acc = *reinterpret_cast<const float4*>(src);
            float a4[4];
            if (r.remap1 == 3) {  // X3: cell n / 4's danger residual column (512 + n / 4) into its danger
                                  // column, summed in the same loop (one chain of load rounds, not two)
                const float* s2 = r.part1 + (size_t)m * r.Np1 + K1P + (n >> 2);
                float d = s2[0];
#pragma unroll 16
                for (int z = 1; z < r.S1; z++) {
                    const float4 v = *reinterpret_cast<const float4*>(src + (size_t)z * zs);
                    const float dv = s2[(size_t)z * zs];
                    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
                    d += dv;
                }
                a4[0] = acc.x; a4[1] = acc.y + d; a4[2] = acc.z; a4[3] = acc.w;
            } else {
#pragma unroll 16
                for (int z = 1; z < r.S1; z++) {
                    const float4 v = *reinterpret_cast<const float4*>(src + (size_t)z * zs);
                    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
                }
                a4[0] = acc.x; a4[1] = acc.y; a4[2] = acc.z; a4[3] = acc.w;
            }
#pragma unroll
            for (int t = 0; t < 4; t++) {
                float* dst = r.gw1 + (size_t)m * K1 + ref_col(n + t);
                const float o = (r.acc ? *dst : 0.f) + a4[t];
                *dst = o;
                sq += o * o;
            }
            if (!r.acc) {  // the cell's constant-input columns: channel 0 (always 0), channel 5 off the centre
                float* row = r.gw1 + (size_t)m * K1 + (n >> 2) * 6;
                row[0] = 0.f;
                if ((n >> 2) * 6 + 5 != CENTRE_COL) row[5] = 0.f;
            }
        }
    } else {  // the small gradients from qbwd3's / qdz1's partial rows
        const int sb = b - r.nb2 - r.nb1, c = (int)threadIdx.x & (RSC - 1), qw = (int)threadIdx.x / RSC;
        constexpr int NG = 256 / RSC;  // row groups
        const bool z1 = sb >= NRS3;
        const int col = (z1 ? sb - NRS3 : sb) * RSC + c;
        const int nrow = z1 ? r.nz1 : r.nb3, pitch = z1 ? HID : P3W, ncol = z1 ? HID : P3L;
        const float* src = (z1 ? r.pz1 : r.p3) + col;
        float acc = 0.f;
        if (col < ncol) {
            const int r1 = (qw + 1) * nrow / NG;
#pragma unroll 8
            for (int i = qw * nrow / NG; i < r1; i++) acc += src[(size_t)i * pitch];
        }
        red[threadIdx.x] = acc;
        __syncthreads();
        if (qw == 0 && col < ncol) {
            float tot = 0.f;  // groups in order, pairwise within each aligned quad
#pragma unroll
            for (int g = 0; g < NG; g += 4)
                tot += (red[g * RSC + c] + red[(g + 1) * RSC + c]) + (red[(g + 2) * RSC + c] + red[(g + 3) * RSC + c]);
            if (z1) {
                const float o = (r.acc ? r.gb1[col] : 0.f) + tot;
                float* cc = r.gw1 + (size_t)col * K1 + CENTRE_COL;  // d/dW1 of the constant centre input
                const float oc = (r.acc ? *cc : 0.f) + tot;
                r.gb1[col] = o;
                *cc = oc;
                sq = o * o + oc * oc;
            } else if (col == P3G) {  // the TD loss (qbwd3's TD step)
                if (r.loss) r.loss[0] = tot / (float)r.B;
            } else {
                float* dst = col < NACT * HID2 ? r.gw3 + col : col < P3G - NACT ? r.gb2 + (col - NACT * HID2)
                                                                                 : r.gb3 + (col - (P3G - NACT));
                const float o = (r.acc ? *dst : 0.f) + tot;
                *dst = o;
                sq = o * o;
            }
        }
        __syncthreads();  // red is reused below
    }
    const float t = red_sum256(sq, red);
    if (threadIdx.x == 0 && r.ss) r.ss[b] = t;
}

// clip_grad_norm_ + torch.optim.Adam (agents/dqn_agent.py:158-160) with the x3 operand
// repack (evx_qmlp_pack3) in one launch, from reduce2_kernel's squared-norm partials: every
// workgroup sums the same partials in the same order (the same norm everywhere), then each
// thread updates one parameter and writes its bf16 hi / lo copies straight into the MFMA
// operand tiles (the inverse of pack3's destination -> source map). The thread of b1[n]
// also owns W1[n][centre] (b1c = b1 + W1[:, centre] needs both updated values).
struct AdamPack {
    float *p, *g, *m, *v;
    const float* ss;
    int nss;
    float max_norm, beta1, beta2, eps, step_size, bc2_sqrt, weight_decay;
    __bf16 *w1b, *w1l, *w2b, *w2l, *w2t, *w2tl;
    __bf16 *w1o, *w1ol;  // x3 act fast path occupancy columns, or NULL
    float* b1c;
    float* norm_out;
};
// element (column col, contraction index k) of an operand in w1_tile / w2_tile / w2t_tile order
__device__ __forceinline__ size_t opnd_off(size_t tile, int col, int k) {
    return tile + (size_t)(((col & 31) + 32 * ((k >> 3) & 1)) * 8 + (k & 7));
}
__device__ __forceinline__ float adam_one(const AdamPack& a, int i, float coef) {
    float gi = a.g[i] * coef;
    const float p = a.p[i];
    if (a.weight_decay != 0.f) gi += a.weight_decay * p;
    const float mi = a.m[i] + (gi - a.m[i]) * (1.f - a.beta1);
    const float vi = a.v[i] * a.beta2 + (1.f - a.beta2) * gi * gi;
    a.m[i] = mi;
    a.v[i] = vi;
    a.g[i] = gi;
    const float denom = sqrtf(vi) / a.bc2_sqrt + a.eps;
    const float pn = p - a.step_size * (mi / denom);
    a.p[i] = pn;
    return pn;
}
__global__ __launch_bounds__(256) void adam_pack3_kernel(AdamPack a0) {
    __shared__ float red[256];
    AdamPack a = a0;
    if (blockIdx.y) {  // grouped: net blockIdx.y (clip_grad_norm_ and Adam per net)
        const size_t G = blockIdx.y;
        a.p += G * NPAR; a.g += G * NPAR; a.m += G * NPAR; a.v += G * NPAR;
        a.ss += G * a.nss;
        a.w1b += G * HID * K1X; a.w1l += G * HID * K1P;
        a.w2b += G * HID2 * HID; a.w2l += G * HID2 * HID;
        a.w2t = adv(a.w2t, G * HID2 * HID); a.w2tl = adv(a.w2tl, G * HID2 * HID);
        a.w1o = adv(a.w1o, G * HID * 128); a.w1ol = adv(a.w1ol, G * HID * 128);
        a.b1c += G * HID;
        a.norm_out = adv(a.norm_out, G);
    }
    float t = 0.f;
    for (int k = (int)threadIdx.x; k < a.nss; k += 256) t += a.ss[k];
    const float norm = sqrtf(red_sum256(t, red));
    float coef = 1.f;
    if (a.max_norm > 0.f) {
        coef = a.max_norm / (norm + 1e-6f);
        coef = coef < 1.f ? coef : 1.f;
    }
    const int i = (int)blockIdx.x * 256 + (int)threadIdx.x;
    if (i == 0 && a.norm_out) a.norm_out[0] = norm;
    if (i >= NPAR) return;
    if (i < OB1) {  // fc1.weight [512][726]: live columns of channels 1-4 -> compact k = 4c + ch - 1
        const int n = i / K1, rc = i - n * K1;
        if (rc == CENTRE_COL) return;  // updated by the b1[n] thread
        const float pn = adam_one(a, i, coef);
        const int c = rc / 6, ch = rc - c * 6;
        if (ch >= 1 && ch <= 4) {
            const int kk = 4 * c + ch - 1;
            __bf16 hi, lo;
            split2(pn, hi, lo);
            a.w1b[opnd_off(w1_tile(n >> 5, kk >> 5, (kk >> 4) & 1, NKC1X), n, kk)] = hi;
            a.w1l[opnd_off(w1_tile(n >> 5, kk >> 5, (kk >> 4) & 1, NKC1), n, kk)] = lo;
            if (ch == 2) {  // the danger column's hi also meets the residual slot 512 + c
                const int kr = K1P + c;
                a.w1b[opnd_off(w1_tile(n >> 5, kr >> 5, (kr >> 4) & 1, NKC1X), n, kr)] = hi;
            }
            if (ch == 1 && a.w1o) {  // occupancy column of cell c: the act fast path's operands
                const size_t oo = opnd_off(w1o_tile(n >> 5, c >> 5, (c >> 4) & 1), n, c);
                a.w1o[oo] = hi;
                a.w1ol[oo] = lo;
            }
        }
    } else if (i < OW2) {  // fc1.bias and W1[:, centre]: b1c = b1 + W1[:, centre]
        const int n = i - OB1;
        const float bn = adam_one(a, i, coef);
        const float wc = adam_one(a, n * K1 + CENTRE_COL, coef);
        a.b1c[n] = bn + wc;
    } else if (i < OB2) {  // fc2.weight [256][512]: W2 (cols = outputs) and W2^T (cols = inputs)
        const float pn = adam_one(a, i, coef);
        const int j = i - OW2, n = j / HID, kk = j - n * HID;
        __bf16 hi, lo;
        split2(pn, hi, lo);
        const size_t o2 = opnd_off(w2_tile(n >> 5, kk >> 5, (kk >> 4) & 1), n, kk);
        a.w2b[o2] = hi;
        a.w2l[o2] = lo;
        if (a.w2t) {
            const size_t ot = opnd_off(w2t_tile(kk >> 5, n >> 5, (n >> 4) & 1), kk, n);
            a.w2t[ot] = hi;
            a.w2tl[ot] = lo;
        }
    } else {
        adam_one(a, i, coef);
    }
}

// squared-norm partials of the flat gradient buffer (one per workgroup) for adam_pack3_kernel
// when the gradients changed after the backward (the multi-GPU all-reduce)
__global__ __launch_bounds__(256) void sumsq_parts_kernel(const float* __restrict__ g, float* __restrict__ ss) {
    __shared__ float red[256];
    float sq = 0.f;
    for (int i = (int)blockIdx.x * 256 + (int)threadIdx.x; i < NPAR; i += (int)gridDim.x * 256) sq += g[i] * g[i];
    const float t = red_sum256(sq, red);
    if (threadIdx.x == 0) ss[blockIdx.x] = t;
}

}  // namespace evxm

// ===================================================================== C-ABI
namespace {
thread_local char m_err[256] = "";
int mfail(int code, const char* msg) {
    snprintf(m_err, sizeof(m_err), "%s", msg);
    return code;
}
int mlaunch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) return 0;
    snprintf(m_err, sizeof(m_err), "%s: %s", what, hipGetErrorString(e));
    return -5;
}
}  // namespace

extern "C" {

const char* evx_qmlp_last_error(void) { return m_err; }

int evx_qmlp_pack(const float* w1, const float* b1, const float* w2, uint16_t* w1b, float* b1c, uint16_t* w2b,
                  uint16_t* w2t, uint16_t* w1o, void* stream) {
    if (!w1 || !b1 || !w2 || !w1b || !b1c || !w2b) return mfail(-22, "qmlp_pack: NULL argument");
    const int n = evxm::HID * evxm::K1P;
    hipLaunchKernelGGL(evxm::pack_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, w1, b1, w2,
                       reinterpret_cast<__bf16*>(w1b), b1c, reinterpret_cast<__bf16*>(w2b),
                       reinterpret_cast<__bf16*>(w2t), reinterpret_cast<__bf16*>(w1o));
    return mlaunch("qmlp_pack");
}

int evx_qmlp_pack_occ3(const float* w1, uint16_t* w1o, uint16_t* w1ol, void* stream) {
    if (!w1 || !w1o || !w1ol) return mfail(-22, "qmlp_pack_occ3: NULL argument");
    hipLaunchKernelGGL(evxm::pack_occ3_kernel, dim3(evxm::HID * 128 / 256), dim3(256), 0, (hipStream_t)stream, w1,
                       reinterpret_cast<__bf16*>(w1o), reinterpret_cast<__bf16*>(w1ol));
    return mlaunch("qmlp_pack_occ3");
}

int evx_qmlp_pack3(const float* w1, const float* b1, const float* w2, uint16_t* w1b, uint16_t* w1l, float* b1c,
                   uint16_t* w2b, uint16_t* w2l, uint16_t* w2t, uint16_t* w2tl, void* stream) {
    if (!w1 || !b1 || !w2 || !w1b || !w1l || !b1c || !w2b || !w2l) return mfail(-22, "qmlp_pack3: NULL argument");
    if ((w2t == nullptr) != (w2tl == nullptr)) return mfail(-22, "qmlp_pack3: w2t and w2tl go together");
    const int n = evxm::HID * evxm::K1X;
    hipLaunchKernelGGL(evxm::pack3_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, w1, b1, w2,
                       reinterpret_cast<__bf16*>(w1b), reinterpret_cast<__bf16*>(w1l), b1c,
                       reinterpret_cast<__bf16*>(w2b), reinterpret_cast<__bf16*>(w2l), reinterpret_cast<__bf16*>(w2t),
                       reinterpret_cast<__bf16*>(w2tl));
    return mlaunch("qmlp_pack3");
}

// the x3 act kernel for the dropout mode of a (fc1_slab_m)
// SAVE: the learner's online forward (no row permutation; X from x_expand_kernel)
extern "C++" template <bool GR, bool SAVE = false>
static void launch_act3(const evxm::Fwd& a, int32_t n, int nets, hipStream_t st) {
    {
        static std::atomic<uint64_t> attr_done;
        const void* kh[3] = {(const void*)evxm::qact3h_kernel<GR, 0, SAVE>, (const void*)evxm::qact3h_kernel<GR, 1, SAVE>,
                             (const void*)evxm::qact3h_kernel<GR, 2, SAVE>};
        evxh::max_lds_once(attr_done, kh, 3, evxm::ACT3H_LDS);
    }
    const dim3 grid((unsigned)((n + 63) / 64), (unsigned)nets);
    if (a.drop_mask)
        hipLaunchKernelGGL((evxm::qact3h_kernel<GR, 2, SAVE>), grid, dim3(256), evxm::ACT3H_LDS, st, a);
    else if (a.drop_thresh)
        hipLaunchKernelGGL((evxm::qact3h_kernel<GR, 1, SAVE>), grid, dim3(256), evxm::ACT3H_LDS, st, a);
    else
        hipLaunchKernelGGL((evxm::qact3h_kernel<GR, 0, SAVE>), grid, dim3(256), evxm::ACT3H_LDS, st, a);
}

static int make_fwd(const evx_layout* lay, const evx_obs* obs, int32_t n, const evx_qmlp_params* p,
                    const evx_qmlp_dropout* drop, const evx_qmlp_fwd_out* out, evxm::Fwd& a) {
    if (!lay || !obs || !p || !out) return mfail(-22, "qmlp_forward: NULL argument");
    if (!p->w1 || !p->b1c || !p->w2 || !p->b2 || !p->w3 || !p->b3) return mfail(-22, "qmlp_forward: missing parameter");
    if (!out->h1) return mfail(-22, "qmlp_forward: h1 buffer required");
    if (!lay->danger_o32 || !lay->cellinfo || !lay->obs_feat)
        return mfail(-22, "qmlp_forward: layout tables missing (obs_feat)");
    a.N = n;
    a.obs = obs;
    a.cellinfo = lay->cellinfo;
    a.danger = lay->danger_o32;
    a.feat = lay->obs_feat;
    a.feats = lay->layout_set ? lay->obs_feats : nullptr;
    a.t_max = lay->t_max;
    a.L = lay->L;
    a.W = lay->W;
    a.ox0 = lay->ox0;
    a.oy0 = lay->oy0;
    a.OX = lay->OX;
    a.OY = lay->OY;
    a.exit_x = lay->exit_x;
    a.exit_y = lay->exit_y;
    a.w1 = reinterpret_cast<const __bf16*>(p->w1);
    a.b1 = p->b1c;
    a.w2 = reinterpret_cast<const __bf16*>(p->w2);
    a.b2 = p->b2;
    a.w3 = p->w3;
    a.b3 = p->b3;
    a.drop_seed = drop ? drop->seed : 0u;
    a.drop_stream = drop ? drop->stream : 0u;
    a.drop_row0 = drop ? drop->row0 : 0u;
    if (a.drop_row0 & 1u) return mfail(-22, "qmlp_forward: dropout row0 must be even (one hash per row pair)");
    const float dp = drop ? drop->p : 0.f;
    a.drop_thresh = dp > 0.f ? (uint32_t)((double)dp * 65536.0) : 0u;  // 16-bit uniforms
    if (dp > 0.f && a.drop_thresh == 0u) a.drop_thresh = 1u;
    a.drop_scale = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
    a.h1 = reinterpret_cast<__bf16*>(out->h1);
    a.x = reinterpret_cast<__bf16*>(out->x);
    a.h2 = out->h2;
    a.q = out->q;
    a.actions = out->actions;
    a.epsilon = out->epsilon;
    a.act_seed = out->act_seed;
    a.act_offset = out->act_offset;
    a.w1o = reinterpret_cast<const __bf16*>(p->w1o);
    a.stat = (p->w1o && !a.feats) ? p->stat : nullptr;  // the table is per layout: single layout only
    a.stat_fs = p->stat_fs;
    a.stat_x0 = p->stat_nx > 0 ? p->stat_x0 : 0;
    a.stat_nx = p->stat_nx > 0 ? p->stat_nx : lay->L + 2;
    if (a.stat && (a.stat_x0 < 0 || a.stat_x0 + a.stat_nx > lay->L + 2))
        return mfail(-22, "qmlp: the table's centre range must lie in [0, L + 2)");
    a.raw = nullptr;
    a.rest_ws = nullptr;
    a.xin = nullptr;
    a.xtab = (p->x3 && a.stat) ? reinterpret_cast<const __bf16*>(p->stat_xin) : nullptr;
    a.drop_mask = drop ? drop->mask : nullptr;
    if (a.drop_mask && !(dp > 0.f)) return mfail(-22, "qmlp_forward: an explicit dropout mask needs p > 0 (its scale)");
    a.feat_lo = nullptr;
    a.feats_lo = nullptr;
    a.w1l = a.w2l = nullptr;
    a.h1l = nullptr;
    a.w1ol = nullptr;
    if (p->x3) {
        if (!p->w1l || !p->w2l) return mfail(-22, "qmlp_forward: x3 needs w1l / w2l (evx_qmlp_pack3)");
        if (!lay->obs_feat_lo || (lay->layout_set && !lay->obs_feats_lo))
            return mfail(-22, "qmlp_forward: x3 needs the layout's obs_feat_lo");
        a.feat_lo = lay->obs_feat_lo;
        a.feats_lo = lay->layout_set ? lay->obs_feats_lo : nullptr;
        a.w1l = reinterpret_cast<const __bf16*>(p->w1l);
        a.w2l = reinterpret_cast<const __bf16*>(p->w2l);
        a.h1l = a.h1 ? a.h1 + (size_t)n * evxm::HID : nullptr;  // lo plane after the hi plane
        a.w1ol = reinterpret_cast<const __bf16*>(p->w1ol);
        if (!a.w1ol) a.stat = nullptr;  // the x3 table path needs the occupancy columns' lo part
    }
    a.perm = out->perm;
    a.rpe = out->rows_per_env > 0 ? out->rows_per_env : 1;
    a.gn = 0;
    a.g = 0;
    // rows_per_env even: dropout row pairs stay together in a tile
    if (a.perm && (a.rpe & 1)) return mfail(-22, "qmlp_forward: rows_per_env must be even (dropout row pairs)");
    return 0;
}

static int launch_fwd(const evxm::Fwd& a0, const evxm::Fwd& a1, int32_t n, int pairs, bool fc23, hipStream_t st,
                      bool x3 = false, int nets = 1) {
    const unsigned blocks = (unsigned)((n + evxm::RM - 1) / evxm::RM);
    const unsigned big = (unsigned)((n + 127) / 128);
    if (nets > 1) {  // grouped (x3 only): blockIdx.z = net * pairs + problem
        const unsigned z = (unsigned)(pairs * nets);
        if (big * z >= 384)
            hipLaunchKernelGGL((evxm::qfc1_kernel<4, 1, 8, true, true>), dim3(big, 2, z), dim3(512), 0, st, a0, a1, pairs);
        else
            hipLaunchKernelGGL((evxm::qfc1_kernel<2, 1, 4, true, true>), dim3(blocks, 4, z), dim3(256), 0, st, a0, a1, pairs);
        int rc = mlaunch("qfc1 grouped");
        if (rc || !fc23) return rc;
        hipLaunchKernelGGL((evxm::qfc23_kernel<true, true>), dim3(blocks, 1, z), dim3(256), 0, st, a0, a1, pairs);
        return mlaunch("qfc23 grouped");
    }
    if (x3) {  // f32-accurate: 128 x 256 tiles for large batches (register budget), else 64 x 128
        // one problem (the learner's online forward beside the target through the fused act):
        // 64 x 256 tiles at any batch (learn 391 -> 382 us at B = 32768 vs 128 x 256)
        if (pairs == 1 && fc23)
            hipLaunchKernelGGL((evxm::qfc1_kernel<2, 2, 4, true>), dim3(blocks, 2, pairs), dim3(256), 0, st, a0, a1, pairs);
        else if (big * pairs >= 384)
            hipLaunchKernelGGL((evxm::qfc1_kernel<4, 1, 8, true>), dim3(big, 2, pairs), dim3(512), 0, st, a0, a1, pairs);
        else
            hipLaunchKernelGGL((evxm::qfc1_kernel<2, 1, 4, true>), dim3(blocks, 4, pairs), dim3(256), 0, st, a0, a1, pairs);
        int rc = mlaunch("qfc1");
        if (rc || !fc23) return rc;
        // 32-row tiles while 64-row ones would leave CUs without a workgroup (cfg2's B = 4096: learn
        // 0.133 -> 0.128 ms; fc1 in 32 x 64 tiles of 2 waves for small problems measured slower)
        if ((int64_t)blocks * pairs < 256)
            hipLaunchKernelGGL((evxm::qfc23_kernel<true, false, 1>), dim3((n + 31) / 32, 1, pairs), dim3(256), 0, st, a0, a1,
                               pairs);
        else
            hipLaunchKernelGGL(evxm::qfc23_kernel<true>, dim3(blocks, 1, pairs), dim3(256), 0, st, a0, a1, pairs);
        return mlaunch("qfc23");
    }
    if (big * pairs >= 384)  // enough 128-row tiles (all 512 columns each) to fill the chip
        hipLaunchKernelGGL((evxm::qfc1_kernel<4, 2, 8>), dim3(big, 1, pairs), dim3(512), 0, st, a0, a1, pairs);
    else
        hipLaunchKernelGGL((evxm::qfc1_kernel<2, 1, 4>), dim3(blocks, 4, pairs), dim3(256), 0, st, a0, a1, pairs);
    int rc = mlaunch("qfc1");
    if (rc || !fc23) return rc;
    hipLaunchKernelGGL(evxm::qfc23_kernel<false>, dim3(blocks, 1, pairs), dim3(256), 0, st, a0, a1, pairs);
    return mlaunch("qfc23");
}

int evx_qmlp_forward(const evx_layout* lay, const evx_obs* obs, int32_t n, const evx_qmlp_params* p,
                     const evx_qmlp_dropout* drop, const evx_qmlp_fwd_out* out, void* stream) {
    if (n <= 0) return 0;
    evxm::Fwd a;
    int rc = make_fwd(lay, obs, n, p, drop, out, a);
    if (rc) return rc;
    return launch_fwd(a, a, n, 1, out->q || out->actions || out->h2, (hipStream_t)stream, p->x3 != 0);
}

// diagnostic builds only: copy the act stamps out (-1 when the build has none)
int evx_diag_act3p_stamps(long long* host, int32_t n) {
#ifdef EVX_ACT_STAMPS
    if (n > 256 * evxm::A3P_MAXIT * evxm::A3P_NST) n = 256 * evxm::A3P_MAXIT * evxm::A3P_NST;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(evxm::g_act3p_st), (size_t)n * 8) == hipSuccess ? n : -5;
#else
    (void)host;
    (void)n;
    return -1;
#endif
}

int evx_diag_act_stamps(long long* host, int32_t n) {
#ifdef EVX_ACT_STAMPS
    if (n > 8192 * evxm::ACT_NST) n = 8192 * evxm::ACT_NST;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(evxm::g_act_st), (size_t)n * 8) == hipSuccess ? n : -5;
#else
    (void)host;
    (void)n;
    return -1;
#endif
}

}  // extern "C"

// the x3 act: the persistent 128-row kernel when its table path applies (a table attached, the hash
// or no dropout) and the launch has >= 4 tiles per CU (its cross-tile pipeline; with one tile per CU,
// cfg2's 32 768 rows, the 64-row kernel's two workgroups per CU measured faster: 16.1 vs 15.3 M
// env-steps/s); else (or kernel64) the 64-row kernel
static void act_x3(const evxm::Fwd& a, int32_t n, hipStream_t st, bool kernel64) {
    const int ntiles = (n + 127) / 128, ncu = evxh::cu_count();
    if (!kernel64 && a.stat && !a.drop_mask && ntiles >= 4 * ncu) {
        {
            static std::atomic<uint64_t> attr_done;
            const void* kp[2] = {(const void*)evxm::qact3p_kernel<0>, (const void*)evxm::qact3p_kernel<1>};
            evxh::max_lds_once(attr_done, kp, 2, evxm::ACT3P_LDS);
            static std::atomic<uint64_t> attr_done2;
            const void* kr[2] = {(const void*)evxm::qact3h_rest_kernel<0>, (const void*)evxm::qact3h_rest_kernel<1>};
            evxh::max_lds_once(attr_done2, kr, 2, evxm::ACT3H_LDS);
        }
        // the table-path tiles on the persistent kernel, then the others (if any) on the 64-row body
        // (listed: one workgroup per CU over their halves; else every row re-checked)
        const dim3 grid((unsigned)std::min(ntiles, ncu));
        const dim3 rgrid(a.rest_ws ? (unsigned)std::min(2 * ntiles, ncu) : (unsigned)((n + 1023) / 1024));
        if (a.drop_thresh) {
            hipLaunchKernelGGL(evxm::qact3p_kernel<1>, grid, dim3(512), evxm::ACT3P_LDS, st, a, ntiles);
            hipLaunchKernelGGL(evxm::qact3h_rest_kernel<1>, rgrid, dim3(256), evxm::ACT3H_LDS, st, a);
        } else {
            hipLaunchKernelGGL(evxm::qact3p_kernel<0>, grid, dim3(512), evxm::ACT3P_LDS, st, a, ntiles);
            hipLaunchKernelGGL(evxm::qact3h_rest_kernel<0>, rgrid, dim3(256), evxm::ACT3H_LDS, st, a);
        }
        return;
    }
    launch_act3<false>(a, n, 1, st);
}

static int qmlp_act_impl(const evx_layout* lay, const evx_obs* obs, int32_t n, const evx_qmlp_params* p,
                         const evx_qmlp_dropout* drop, const evx_qmlp_fwd_out* out, void* stream, bool kernel64) {
    if (n <= 0) return 0;
    if (!out) return mfail(-22, "qmlp_act: NULL out");
    if (!out->q && !out->actions) return mfail(-22, "qmlp_act: needs q or actions");
    evx_qmlp_fwd_out o = *out;
    o.h1 = o.h1 ? o.h1 : reinterpret_cast<uint16_t*>(1);  // unused: H1 stays in LDS
    o.x = nullptr;
    o.h2 = nullptr;
    evxm::Fwd a;
    int rc = make_fwd(lay, obs, n, p, drop, &o, a);
    if (rc) return rc;
    a.h1 = nullptr;
    a.h1l = nullptr;
    a.rest_ws = out->act_ws;
    {
        static std::atomic<uint64_t> attr_done;
        const void* ks[1] = {(const void*)evxm::qact_kernel};
        evxh::max_lds_once(attr_done, ks, 1, evxm::ACT_LDS);
    }
    if (p->x3)
        act_x3(a, n, (hipStream_t)stream, kernel64);
    else
        hipLaunchKernelGGL(evxm::qact_kernel, dim3((unsigned)((n + 127) / 128)), dim3(512), evxm::ACT_LDS,
                           (hipStream_t)stream, a);
    return mlaunch("qact");
}

extern "C" {

int64_t evx_qmlp_act_ws_ints(int32_t n) { return n > 0 ? 2 + ((int64_t)n + 127) / 128 : 2; }

int evx_qmlp_act(const evx_layout* lay, const evx_obs* obs, int32_t n, const evx_qmlp_params* p,
                 const evx_qmlp_dropout* drop, const evx_qmlp_fwd_out* out, void* stream) {
    return qmlp_act_impl(lay, obs, n, p, drop, out, stream, false);
}

int evx_qmlp_act64(const evx_layout* lay, const evx_obs* obs, int32_t n, const evx_qmlp_params* p,
                   const evx_qmlp_dropout* drop, const evx_qmlp_fwd_out* out, void* stream) {
    return qmlp_act_impl(lay, obs, n, p, drop, out, stream, true);
}

int evx_qmlp_expand_x3(const evx_layout* lay, const evx_obs* obs, int32_t n, uint16_t* x, void* stream) {
    if (n <= 0) return 0;
    if (!lay || !obs || !x) return mfail(-22, "qmlp_expand_x3: NULL argument");
    if (!lay->obs_feat || !lay->obs_feat_lo || (lay->layout_set && (!lay->obs_feats || !lay->obs_feats_lo)))
        return mfail(-22, "qmlp_expand_x3: layout tables missing (obs_feat, obs_feat_lo)");
    evxm::Fwd a{};
    a.N = n;
    a.obs = obs;
    a.feat = lay->obs_feat;
    a.feats = lay->layout_set ? lay->obs_feats : nullptr;
    a.feat_lo = lay->obs_feat_lo;
    a.feats_lo = lay->layout_set ? lay->obs_feats_lo : nullptr;
    a.L = lay->L;
    a.W = lay->W;
    a.t_max = lay->t_max;
    a.x = reinterpret_cast<__bf16*>(x);
    const int64_t nx = (int64_t)n * 20;
    hipLaunchKernelGGL(evxm::x_expand_kernel, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
    return mlaunch("qmlp_expand_x3");
}

int evx_qmlp_stat_x(const evx_layout* lay, const evx_obs* obs, const uint16_t* x, int32_t n, const evx_qmlp_params* p,
                    float* out, void* stream) {
    if (!x) return evx_qmlp_stat(lay, obs, n, p, out, stream);
    if (n <= 0) return 0;
    if (!out || !p) return mfail(-22, "qmlp_stat_x: NULL argument");
    if (!p->x3) return mfail(-22, "qmlp_stat_x: the X input is the x3 layout (p->x3)");
    evx_qmlp_fwd_out o{};
    o.h1 = reinterpret_cast<uint16_t*>(out);  // not written in raw mode
    evxm::Fwd a;
    int rc = make_fwd(lay, obs, n, p, nullptr, &o, a);
    if (rc) return rc;
    a.h1 = nullptr;
    a.h1l = nullptr;
    a.stat = nullptr;
    a.perm = nullptr;
    a.raw = out;
    a.xin = reinterpret_cast<const __bf16*>(x);
    const unsigned blocks = (unsigned)((n + evxm::RM - 1) / evxm::RM);
    hipLaunchKernelGGL((evxm::qfc1_kernel<2, 1, 4, true, false, true>), dim3(blocks, 4, 1), dim3(256), 0,
                       (hipStream_t)stream, a, a, 1);
    return mlaunch("qmlp_stat_x");
}

int evx_qmlp_stat(const evx_layout* lay, const evx_obs* obs, int32_t n, const evx_qmlp_params* p, float* out,
                  void* stream) {
    if (n <= 0) return 0;
    if (!out) return mfail(-22, "qmlp_stat: NULL out");
    evx_qmlp_fwd_out o{};
    o.h1 = reinterpret_cast<uint16_t*>(out);  // not written in raw mode
    evxm::Fwd a;
    int rc = make_fwd(lay, obs, n, p, nullptr, &o, a);
    if (rc) return rc;
    a.h1 = nullptr;
    a.h1l = nullptr;
    a.stat = nullptr;
    a.perm = nullptr;
    a.raw = out;
    return launch_fwd(a, a, n, 1, false, (hipStream_t)stream, p->x3 != 0);
}

int evx_qmlp_forward2(const evx_layout* lay, int32_t n, const evx_obs* obs0, const evx_qmlp_params* p0,
                      const evx_qmlp_dropout* drop0, const evx_qmlp_fwd_out* out0, const evx_obs* obs1,
                      const evx_qmlp_params* p1, const evx_qmlp_dropout* drop1, const evx_qmlp_fwd_out* out1,
                      void* stream) {
    if (n <= 0) return 0;
    evxm::Fwd a0, a1;
    int rc = make_fwd(lay, obs0, n, p0, drop0, out0, a0);
    if (!rc) rc = make_fwd(lay, obs1, n, p1, drop1, out1, a1);
    if (rc) return rc;
    if (!(out0->q || out0->actions || out0->h2) || !(out1->q || out1->actions || out1->h2))
        return mfail(-22, "qmlp_forward2: both problems need an fc2/fc3 output");
    if ((p0->x3 != 0) != (p1->x3 != 0)) return mfail(-22, "qmlp_forward2: both problems in one precision");
    // (at n >= 32768 only: a fused act workgroup lives ~65 us on the full path, so below a full
    // round of workgroups the two-kernel forward wins -- B = 4096: learn 187 vs 127 us)
    const int dm0 = a0.drop_mask ? 2 : a0.drop_thresh ? 1 : 0, dm1 = a1.drop_mask ? 2 : a1.drop_thresh ? 1 : 0;
    if (p0->x3 && out1->q && !out1->h2 && !out1->actions && !out1->x && n >= 8192 && n < 32768 && a0.stat && a1.stat &&
        !a0.perm && !a0.actions && a0.x && a0.h1 && a0.h1l && a0.h2 && a0.q && dm0 == dm1) {
        // both forwards through the act tables in one launch (qfwd2_kernel), X by its own launch
        a1.perm = nullptr;
        a1.actions = nullptr;
        a1.h1 = a1.h1l = nullptr;
        {
            static std::atomic<uint64_t> attr_done;
            const void* kf[3] = {(const void*)evxm::qfwd2_kernel<0>, (const void*)evxm::qfwd2_kernel<1>,
                                 (const void*)evxm::qfwd2_kernel<2>};
            evxh::max_lds_once(attr_done, kf, 3, evxm::ACT3H_LDS);
        }
        const int64_t nx = (int64_t)n * 20;
        hipLaunchKernelGGL(evxm::x_expand_kernel, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a0);
        const dim3 grid((unsigned)((n + 63) / 64), 2);
        if (dm0 == 2)
            hipLaunchKernelGGL(evxm::qfwd2_kernel<2>, grid, dim3(256), evxm::ACT3H_LDS, (hipStream_t)stream, a0, a1);
        else if (dm0 == 1)
            hipLaunchKernelGGL(evxm::qfwd2_kernel<1>, grid, dim3(256), evxm::ACT3H_LDS, (hipStream_t)stream, a0, a1);
        else
            hipLaunchKernelGGL(evxm::qfwd2_kernel<0>, grid, dim3(256), evxm::ACT3H_LDS, (hipStream_t)stream, a0, a1);
        return mlaunch("qmlp_forward2 paired");
    }
    if (p0->x3 && out1->q && !out1->h2 && !out1->actions && !out1->x && n >= 32768) {
        // x3 learner: the second problem (the target net: Q only) through the fused act kernel
        // (H1 / H2 stay in LDS, 64-row tiles, two workgroups per CU) instead of qfc1 + qfc23
        // writing and re-reading both H1 planes; the first problem alone through qfc1 + qfc23
        // the target net's own act table (static features x W1, rebuilt at each target sync --
        // evacx.trainer attaches it to both nets): replay rows past the fire's last step (every
        // row once the fire has stopped spreading: fire_step persists across resets) start fc1
        // from it, the others run the full path per 64-row tile.
        a1.perm = nullptr;
        a1.actions = nullptr;
        a1.h1 = a1.h1l = nullptr;
        if (a0.stat && !a0.perm && !a0.actions && a0.x && a0.h1 && a0.h1l && a0.h2 && a0.q) {
            // the online net's act table too (rebuilt after every update, so it matches the weights
            // this forward reads): the online forward through the fused act kernel's table path,
            // H1 planes / H2 / Q saved for the backward, X expanded by its own launch -- instead of
            // qfc1's K = 640 products over staged A tiles and qfc23 re-reading both H1 planes
            const int64_t nx = (int64_t)n * 20;
            hipLaunchKernelGGL(evxm::x_expand_kernel, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0,
                               (hipStream_t)stream, a0);
            launch_act3<false, true>(a0, n, 1, (hipStream_t)stream);
        } else {
            // (the online forward through the fused kernel on the full path with X saved measured no
            // faster than qfc1 + qfc23 at B = 32768: learn 0.420 vs 0.427 ms)
            int rc2 = launch_fwd(a0, a0, n, 1, true, (hipStream_t)stream, true);
            if (rc2) return rc2;
        }
        launch_act3<false>(a1, n, 1, (hipStream_t)stream);
        return mlaunch("qmlp_forward2 target act");
    }
    return launch_fwd(a0, a1, n, 2, true, (hipStream_t)stream, p0->x3 != 0);
}

// K splits of a weight-gradient GEMM: the most splits, a multiple of 8 (tn_place), whose
// tiles x splits fit `slots` workgroups at once (two per CU: 512; dW2 shares its launch with
// the 256 dZ1 workgroups: 256). dW1 (x3: 20 tiles) at B = 32768 -> 24 splits, 480 workgroups,
// 60 per XCD.
static int ksplit_kper(int B, int tiles, int slots, int minrows) {
    // ... and no more than one split per `minrows` rows (dW1: 1024 -- below that its partials'
    // reduction outweighs the parallelism, B = 8192: learn 171 -> 154 us; dW2, whose launch the
    // dZ1 tiles share: 256)
    const int S = std::max(8, std::min(slots / tiles / 8 * 8, B / minrows / 8 * 8));
    int kper = (B + S - 1) / S;
    return (kper + evxm::TKC - 1) / evxm::TKC * evxm::TKC;
}
static int dw2_kper(int B) { return ksplit_kper(B, 8, 256, 256); }
// (B <= 4096: one split per 256 rows -- 16 at cfg2's B = 4096, 160 -> 320 workgroups)
static int dw1_kper(int B, bool x3) { return ksplit_kper(B, x3 ? 20 : 16, 512, B <= 4096 ? 256 : 1024); }
static int qbwd3_blocks(int B) { return (B + evxm::qbwd3_rows(B) - 1) / evxm::qbwd3_rows(B); }
static int qdz1_wgx(int B) {
    const int qrt = evxm::qdz1_tiles_per_wg(B);
    return (B + evxm::RM * qrt - 1) / (evxm::RM * qrt);
}

// the backward's partials, in this order (all live until reduce2_kernel): dW2's split-K tiles,
// dW1's, qbwd3's block rows [nb3][P3W], qdz1's column sums [ndzx][HID]
static int64_t part2_floats(int32_t B) {
    const int64_t s2 = (B + dw2_kper(B) - 1) / dw2_kper(B);
    return s2 * evxm::HID2 * evxm::HID;
}
static int64_t part_p3_off(int32_t B) {
    const int64_t s1 = std::max((B + dw1_kper(B, false) - 1) / dw1_kper(B, false),
                                (B + dw1_kper(B, true) - 1) / dw1_kper(B, true));  // bf16 / x3 dW1 splits
    return part2_floats(B) + s1 * evxm::HID * evxm::K1X;  // K1X: the x3 dW1 width
}
static int64_t part_pz1_off(int32_t B) { return part_p3_off(B) + (int64_t)qbwd3_blocks(B) * evxm::P3W; }
int64_t evx_qmlp_backward_part_floats(int32_t B) {
    if (B <= 0) return 0;
    return part_pz1_off(B) + (int64_t)qdz1_wgx(B) * evxm::HID;
}

// workgroups of reduce2_kernel = squared-norm partials the backward leaves for evx_qmlp_adam_pack3
static int norm_parts() {
    return (evxm::HID2 * evxm::HID / 4 + 255) / 256 + (evxm::HID * evxm::NCELL + 255) / 256 + evxm::NRSMALL;
}
int32_t evx_qmlp_norm_parts(void) { return norm_parts(); }
int64_t evx_qmlp_nparams(void) { return evxm::NPAR; }

extern "C++" {
// dZ1 + dW2 (bwd_mid), dW1 (gemm_tn), then every reduction + the squared-norm partials
// (reduce2): all sums in a fixed order
template <bool X3, int AP2, int BP2, int AP1, int BP1>
static void launch_tail(const evxm::Bwd& a, int32_t B, const evx_qmlp_grads* g, float* ss, hipStream_t st,
                        int nets, int acc, float* loss) {
    // dW2 = dZ2^T H1 (256 x 512); dW1 = dZ1^T X (512 x compact K -> 726); K = B split into S tiles
    evxm::GemmTN g2{a.dz2, evxm::HID2, a.h1, evxm::HID, B, evxm::HID2, evxm::HID, dw2_kper(B), g->w2, evxm::HID, 0,
                    g->part, X3 ? a.dz2l : nullptr, X3 ? a.h1l : nullptr, evxm::HID / evxm::TT, evxm::HID2 / evxm::TT, 0};
    g2.gz = (B + g2.kper - 1) / g2.kper;
    const int KX = X3 ? evxm::K1X : evxm::K1P;
    evxm::GemmTN g1{a.dz1, evxm::HID, a.x, KX, B, evxm::HID, X3 ? evxm::K1X : 4 * evxm::NCELL,
                    dw1_kper(B, X3), g->w1, evxm::K1, X3 ? 3 : 1, g->part + part2_floats(B),
                    X3 ? a.dz1l : nullptr, nullptr, KX / evxm::TT, evxm::HID / evxm::TT, 0};
    g1.gz = (B + g1.kper - 1) / g1.kper;
    const int ndzx = qdz1_wgx(B);
    const int64_t pf = evx_qmlp_backward_part_floats(B);
    evxm::Red2 r{g->part, g2.gz, g1.part, g1.gz, g1.gx * evxm::TT, 4 * evxm::NCELL, X3 ? 3 : 1,
                 g->w1, g->b1, g->w2, g->b2, g->w3, g->b3, ss,
                 (evxm::HID2 * evxm::HID / 4 + 255) / 256, (evxm::HID * evxm::NCELL + 255) / 256, 0,
                 a.p3, qbwd3_blocks(B), a.pz1, ndzx, acc, loss, B};
    constexpr int lds = std::max(evxm::qdz1_lds_bytes<X3>(), evxm::gemm_tn_lds_bytes<AP2, BP2>());
    const unsigned nmid = (unsigned)(ndzx * (evxm::HID / 128) + g2.gx * g2.gy * g2.gz);
    if (nets > 1) {  // grouped (x3): net g's operands, gradients and partials (fwd_net / bwd_net)
        g2.gsA = 2 * (int64_t)B * evxm::HID2;
        g2.gsB = 2 * (int64_t)B * evxm::HID;
        g2.gsC = evxm::NPAR;
        g2.gsP = pf;
        g1.gsA = 2 * (int64_t)B * evxm::HID;
        g1.gsB = (int64_t)B * evxm::K1X;
        g1.gsC = evxm::NPAR;
        g1.gsP = pf;
        r.gsP = pf;
        {  // the LDS limit at the device's maximum: lds depends on B, the attribute is set once
            static std::atomic<uint64_t> attr_done;
            const void* ks[1] = {(const void*)evxm::bwd_mid_kernel<X3, AP2, BP2, true>};
            evxh::max_lds_once(attr_done, ks, 1, 160 * 1024);
        }
        hipLaunchKernelGGL((evxm::bwd_mid_kernel<X3, AP2, BP2, true>), dim3(nmid, nets), dim3(256), lds, st, a, ndzx, g2);
        hipLaunchKernelGGL((evxm::gemm_tn_kernel<AP1, BP1, true>), dim3(g1.gx, g1.gy, g1.gz * nets), dim3(256), 0, st, g1);
        hipLaunchKernelGGL(evxm::reduce2_kernel, dim3((unsigned)norm_parts(), nets), dim3(256), 0, st, r);
        return;
    }
    // qdz1 and the dW2 tiles in one launch (both read only qbwd3's outputs), then the dW1
    // tiles, then every reduction + the squared-norm partials in one launch
    {
        static std::atomic<uint64_t> attr_done;
        const void* ks[1] = {(const void*)evxm::bwd_mid_kernel<X3, AP2, BP2>};
        evxh::max_lds_once(attr_done, ks, 1, 160 * 1024);
    }
    hipLaunchKernelGGL((evxm::bwd_mid_kernel<X3, AP2, BP2>), dim3(nmid), dim3(256), lds, st, a, ndzx, g2);
    hipLaunchKernelGGL((evxm::gemm_tn_kernel<AP1, BP1>), dim3(g1.gx * g1.gy * g1.gz), dim3(256), 0, st, g1);
    hipLaunchKernelGGL(evxm::reduce2_kernel, dim3((unsigned)norm_parts()), dim3(256), 0, st, r);
}
}  // extern "C++"

// td: the TD step runs inside qbwd3 (dq unused; the loss from reduce2), or NULL (dq given).
// zero_grads != 0: the reductions overwrite the gradients (every element: W1's constant-input
// columns are written as zeros), else they add to them.
struct TdIn {
    const float *Q, *Qt, *rew, *w;
    const int32_t* act;
    const uint8_t* done;
    float gamma;
    float *loss, *td_abs;
};
static int qmlp_backward(const evx_qmlp_params* p, int32_t B, const float* dq, const uint16_t* x, const uint16_t* h1,
                         const float* h2, float drop_p, uint16_t* dz2, uint16_t* dz1, const evx_qmlp_grads* g,
                         int32_t zero_grads, float* ss, void* stream, int nets = 1, const TdIn* td = nullptr) {
    if (!p || !g || !(dq || td) || !x || !h1 || !h2 || !dz2 || !dz1) return mfail(-22, "qmlp_backward: NULL argument");
    if (td && (!td->Q || !td->Qt || !td->act || !td->rew || !td->done || !td->loss))
        return mfail(-22, "qmlp_td_backward: NULL TD argument");
    if (td && nets > 1) return mfail(-22, "qmlp_td_backward: one net");
    if (!p->w2t || !p->w3) return mfail(-22, "qmlp_backward: w2t / w3 required");
    if (!g->w1 || !g->b1 || !g->w2 || !g->b2 || !g->w3 || !g->b3) return mfail(-22, "qmlp_backward: missing grad");
    if (ss && (g->b1 != g->w1 + evxm::OB1 || g->w2 != g->w1 + evxm::OW2 || g->b2 != g->w1 + evxm::OB2 ||
               g->w3 != g->w1 + evxm::OW3 || g->b3 != g->w1 + evxm::OB3))
        return mfail(-22, "qmlp_backward: norm partials need the gradients as one flat state_dict-order buffer");
    if (!g->part) return mfail(-22, "qmlp_backward: g->part required (evx_qmlp_backward_part_floats(B) floats)");
    if (B <= 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const int rb3 = evxm::qbwd3_rows(B);
    const int acc = zero_grads ? 0 : 1;
    evxm::Bwd a;
    a.B = B;
    a.dq = dq;
    a.h2 = h2;
    a.h1 = reinterpret_cast<const __bf16*>(h1);
    a.x = reinterpret_cast<const __bf16*>(x);
    a.w3 = p->w3;
    a.w2t = reinterpret_cast<const __bf16*>(p->w2t);
    a.scale = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
    a.dz2 = reinterpret_cast<__bf16*>(dz2);
    a.dz1 = reinterpret_cast<__bf16*>(dz1);
    a.gw1 = g->w1;
    a.gb1 = g->b1;
    a.gw2 = g->w2;
    a.gb2 = g->b2;
    a.gw3 = g->w3;
    a.gb3 = g->b3;
    a.h1l = nullptr;
    a.w2tl = nullptr;
    a.dz2l = a.dz1l = nullptr;
    a.p3 = g->part + part_p3_off(B);
    a.pz1 = g->part + part_pz1_off(B);
    a.gsP = evx_qmlp_backward_part_floats(B);
    a.td = td != nullptr;
    a.Q = td ? td->Q : nullptr;
    a.Qt = td ? td->Qt : nullptr;
    a.rew = td ? td->rew : nullptr;
    a.w = td ? td->w : nullptr;
    a.act = td ? td->act : nullptr;
    a.done = td ? td->done : nullptr;
    a.gamma = td ? td->gamma : 0.f;
    a.td_abs = td ? td->td_abs : nullptr;
    float* loss = td ? td->loss : nullptr;
    if (p->x3) {
        if (!p->w2tl) return mfail(-22, "qmlp_backward: x3 needs w2tl (evx_qmlp_pack3)");
        a.h1l = a.h1 + (size_t)B * evxm::HID;  // lo planes after the hi planes
        a.w2tl = reinterpret_cast<const __bf16*>(p->w2tl);
        a.dz2l = a.dz2 + (size_t)B * evxm::HID2;
        a.dz1l = a.dz1 + (size_t)B * evxm::HID;
        if (nets > 1) {
            hipLaunchKernelGGL((evxm::qbwd3_kernel<true, true>), dim3((unsigned)((B + rb3 - 1) / rb3), nets),
                               dim3(256), 0, st, a, rb3);
            launch_tail<true, 2, 2, 2, 1>(a, B, g, ss, st, nets, acc, nullptr);
            return mlaunch("qmlp_backward grouped");
        }
        hipLaunchKernelGGL(evxm::qbwd3_kernel<true>, dim3((unsigned)((B + rb3 - 1) / rb3)), dim3(256), 0, st, a, rb3);
        // dW2: both operands split; dW1 over the 640 x3 columns (X exact in bf16): the danger
        // residual column of a cell adds into its danger column
        launch_tail<true, 2, 2, 2, 1>(a, B, g, ss, st, 1, acc, loss);
        return mlaunch("qmlp_backward");
    }
    hipLaunchKernelGGL(evxm::qbwd3_kernel<false>, dim3((unsigned)((B + rb3 - 1) / rb3)), dim3(256), 0, st, a, rb3);
    launch_tail<false, 1, 1, 1, 1>(a, B, g, ss, st, 1, acc, loss);
    return mlaunch("qmlp_backward");
}

int evx_qmlp_td_backward_ss(const evx_qmlp_params* p, int32_t B, const float* Q, const float* Qt, const int32_t* act,
                            const float* rew, const uint8_t* done, float gamma, const float* w, float* loss,
                            float* td_abs, const uint16_t* x, const uint16_t* h1, const float* h2, float drop_p,
                            uint16_t* dz2, uint16_t* dz1, const evx_qmlp_grads* g, float* ss, void* stream) {
    const TdIn td{Q, Qt, rew, w, act, done, gamma, loss, td_abs};
    return qmlp_backward(p, B, nullptr, x, h1, h2, drop_p, dz2, dz1, g, 1, ss, stream, 1, &td);
}

int evx_qmlp_backward(const evx_qmlp_params* p, int32_t B, const float* dq, const uint16_t* x, const uint16_t* h1,
                      const float* h2, float drop_p, uint16_t* dz2, uint16_t* dz1, const evx_qmlp_grads* g,
                      int32_t zero_grads, void* stream) {
    return qmlp_backward(p, B, dq, x, h1, h2, drop_p, dz2, dz1, g, zero_grads, nullptr, stream);
}

int evx_qmlp_backward_ss(const evx_qmlp_params* p, int32_t B, const float* dq, const uint16_t* x, const uint16_t* h1,
                         const float* h2, float drop_p, uint16_t* dz2, uint16_t* dz1, const evx_qmlp_grads* g,
                         int32_t zero_grads, float* ss, void* stream) {
    if (!ss) return mfail(-22, "qmlp_backward_ss: NULL ss");
    return qmlp_backward(p, B, dq, x, h1, h2, drop_p, dz2, dz1, g, zero_grads, ss, stream);
}

int evx_qmlp_sumsq_parts(const float* g, float* ss, void* stream) {
    if (!g || !ss) return mfail(-22, "qmlp_sumsq_parts: NULL argument");
    hipLaunchKernelGGL(evxm::sumsq_parts_kernel, dim3((unsigned)norm_parts()), dim3(256), 0, (hipStream_t)stream, g, ss);
    return mlaunch("qmlp_sumsq_parts");
}

static int adam_pack3(float* p, float* g, float* m, float* v, float max_norm, const evx_adam* h, uint16_t* w1b,
                      uint16_t* w1l, float* b1c, uint16_t* w2b, uint16_t* w2l, uint16_t* w2t, uint16_t* w2tl,
                      uint16_t* w1o, uint16_t* w1ol, const float* ss, int32_t nss, float* norm_out, void* stream,
                      int nets);
int evx_qmlp_adam_pack3(float* p, float* g, float* m, float* v, float max_norm, const evx_adam* h, uint16_t* w1b,
                        uint16_t* w1l, float* b1c, uint16_t* w2b, uint16_t* w2l, uint16_t* w2t, uint16_t* w2tl,
                        uint16_t* w1o, uint16_t* w1ol, const float* ss, int32_t nss, float* norm_out, void* stream) {
    return adam_pack3(p, g, m, v, max_norm, h, w1b, w1l, b1c, w2b, w2l, w2t, w2tl, w1o, w1ol, ss, nss, norm_out,
                      stream, 1);
}
int evx_qmlp_adam_pack3_g(float* p, float* g, float* m, float* v, float max_norm, const evx_adam* h, uint16_t* w1b,
                          uint16_t* w1l, float* b1c, uint16_t* w2b, uint16_t* w2l, uint16_t* w2t, uint16_t* w2tl,
                          uint16_t* w1o, uint16_t* w1ol, const float* ss, int32_t nss, float* norm_out, int32_t nets,
                          void* stream) {
    if (nets < 1 || nets > 1024) return mfail(-22, "qmlp_adam_pack3_g: nets must be 1..1024");
    return adam_pack3(p, g, m, v, max_norm, h, w1b, w1l, b1c, w2b, w2l, w2t, w2tl, w1o, w1ol, ss, nss, norm_out,
                      stream, nets);
}
static int adam_pack3(float* p, float* g, float* m, float* v, float max_norm, const evx_adam* h, uint16_t* w1b,
                      uint16_t* w1l, float* b1c, uint16_t* w2b, uint16_t* w2l, uint16_t* w2t, uint16_t* w2tl,
                      uint16_t* w1o, uint16_t* w1ol, const float* ss, int32_t nss, float* norm_out, void* stream,
                      int nets) {
    if ((w1o == nullptr) != (w1ol == nullptr)) return mfail(-22, "qmlp_adam_pack3: w1o and w1ol go together");
    if (!p || !g || !m || !v || !h || !w1b || !w1l || !b1c || !w2b || !w2l || !ss)
        return mfail(-22, "qmlp_adam_pack3: NULL argument");
    if ((w2t == nullptr) != (w2tl == nullptr)) return mfail(-22, "qmlp_adam_pack3: w2t and w2tl go together");
    if (nss <= 0) return mfail(-22, "qmlp_adam_pack3: no norm partials");
    evxm::AdamPack a;
    a.p = p; a.g = g; a.m = m; a.v = v;
    a.ss = ss; a.nss = nss;
    const double bc1 = 1.0 - pow((double)h->beta1, (double)h->step);
    const double bc2 = 1.0 - pow((double)h->beta2, (double)h->step);
    a.max_norm = max_norm; a.beta1 = h->beta1; a.beta2 = h->beta2; a.eps = h->eps;
    a.step_size = (float)(h->lr / bc1);
    a.bc2_sqrt = (float)sqrt(bc2);
    a.weight_decay = h->weight_decay;
    a.w1b = reinterpret_cast<__bf16*>(w1b); a.w1l = reinterpret_cast<__bf16*>(w1l);
    a.w2b = reinterpret_cast<__bf16*>(w2b); a.w2l = reinterpret_cast<__bf16*>(w2l);
    a.w2t = reinterpret_cast<__bf16*>(w2t); a.w2tl = reinterpret_cast<__bf16*>(w2tl);
    a.b1c = b1c; a.norm_out = norm_out;
    a.w1o = reinterpret_cast<__bf16*>(w1o); a.w1ol = reinterpret_cast<__bf16*>(w1ol);
    hipLaunchKernelGGL(evxm::adam_pack3_kernel, dim3((unsigned)((evxm::NPAR + 255) / 256), nets), dim3(256), 0,
                       (hipStream_t)stream, a);
    return mlaunch("qmlp_adam_pack3");
}

// ------------------------------------------------ grouped nets
// Every per-net buffer is an array [nets][one net's buffer]: the pointers passed are net 0's.
static int group_check(int32_t nets, const evx_qmlp_params* p, const char* what) {
    if (nets < 1 || nets > 1024) return mfail(-22, "grouped qmlp: nets must be 1..1024");
    if (!p || !p->x3) return mfail(-22, "grouped qmlp: x3 parameters required (the [nets] operand layout is x3's)");
    (void)what;
    return 0;
}

int evx_qmlp_act_g(const evx_layout* lay, const evx_obs* obs, int32_t n, int32_t nets, const evx_qmlp_params* p,
                   const evx_qmlp_dropout* drop, const evx_qmlp_fwd_out* out, void* stream) {
    int rc = group_check(nets, p, "act");
    if (rc) return rc;
    if (n <= 0) return 0;
    if (!out || (!out->q && !out->actions)) return mfail(-22, "qmlp_act_g: needs q or actions");
    if (out->perm) return mfail(-22, "qmlp_act_g: no act permutation with grouped nets");
    if (p->stat) return mfail(-22, "qmlp_act_g: the act table path is single-net");
    if (n & 1) return mfail(-22, "qmlp_act_g: rows per net must be even (dropout row pairs)");
    evx_qmlp_fwd_out o = *out;
    o.h1 = reinterpret_cast<uint16_t*>(1);
    o.x = nullptr;
    o.h2 = nullptr;
    evxm::Fwd a;
    rc = make_fwd(lay, obs, n, p, drop, &o, a);
    if (rc) return rc;
    a.h1 = nullptr;
    a.h1l = nullptr;
    a.gn = nets;
    launch_act3<true>(a, n, nets, (hipStream_t)stream);
    return mlaunch("qact_g");
}

int evx_qmlp_forward2_g(const evx_layout* lay, int32_t n, int32_t nets, const evx_obs* obs0, const evx_qmlp_params* p0,
                        const evx_qmlp_dropout* drop0, const evx_qmlp_fwd_out* out0, const evx_obs* obs1,
                        const evx_qmlp_params* p1, const evx_qmlp_dropout* drop1, const evx_qmlp_fwd_out* out1,
                        void* stream) {
    int rc = group_check(nets, p0, "forward2");
    if (!rc) rc = group_check(nets, p1, "forward2");
    if (rc) return rc;
    if (n <= 0) return 0;
    if (n & 1) return mfail(-22, "qmlp_forward2_g: rows per net must be even (dropout row pairs)");
    evxm::Fwd a0, a1;
    rc = make_fwd(lay, obs0, n, p0, drop0, out0, a0);
    if (!rc) rc = make_fwd(lay, obs1, n, p1, drop1, out1, a1);
    if (rc) return rc;
    if (a0.stat || a1.stat || a0.perm || a1.perm) return mfail(-22, "qmlp_forward2_g: no table path / permutation");
    if (!(out0->q || out0->h2) || !(out1->q || out1->h2)) return mfail(-22, "qmlp_forward2_g: needs fc2/fc3 outputs");
    if ((int64_t)n * nets * 2 > (int64_t)1 << 31) return mfail(-22, "qmlp_forward2_g: too many rows");
    return launch_fwd(a0, a1, n, 2, true, (hipStream_t)stream, true, nets);
}

int evx_qmlp_backward_ss_g(const evx_qmlp_params* p, int32_t B, int32_t nets, const float* dq, const uint16_t* x,
                           const uint16_t* h1, const float* h2, float drop_p, uint16_t* dz2, uint16_t* dz1,
                           const evx_qmlp_grads* g, float* ss, void* stream) {
    int rc = group_check(nets, p, "backward");
    if (rc) return rc;
    if (!g || !g->part) return mfail(-22, "qmlp_backward_ss_g: split-K partials required ([nets][part floats(B)])");
    if (!ss) return mfail(-22, "qmlp_backward_ss_g: NULL ss");
    return qmlp_backward(p, B, dq, x, h1, h2, drop_p, dz2, dz1, g, 0, ss, stream, nets);
}

}  // extern "C"
