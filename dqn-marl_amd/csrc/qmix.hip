// QMIX / VDN value mixing on the device: the reference's MixingNetwork
// (runners/train_qmix.py:39-54) and its learn step's loss (:78-104) over a batch of B joint
// transitions of n agents whose per-agent Q values come from the grouped net kernels
// (evx_qmlp_forward2_g: Q and target Q as [n][B][A]).
//
//   q_tot = relu(q @ |W1| + b1) @ |W2| + b2        (q: the chosen-action Q of every agent)
//   y     = r + gamma * q_tot'(max_a Q'_i) * (1 - done)   (target mixer on the target nets)
//   loss  = mean((q_tot - y)^2)
//
// qmix_rows_kernel: one thread per transition runs both mixers, the loss term and the
// backward through the online mixer (torch.abs' gradient is sign(W), relu's [out > 0]); it
// writes d loss / d Q of every agent at its taken action (dQ [n][B][A], 0 elsewhere -- the
// grouped backward's input), stages the row's factors in LDS, and thread k of the workgroup
// then sums parameter k's gradient over the workgroup's rows in row order. qmix_reduce_kernel
// adds the workgroups' partials in workgroup order (deterministic) into the mixer gradient
// (state_dict order: fc1_weight [n][32], fc1_bias [32], fc2_weight [32][1], fc2_bias [1]) and
// the loss. Extra workgroups of the rows launch clear the agents' gradient buffer, as
// td_loss_zero does for one net.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>

#include "evacx.h"
#include "evx_host.h"

namespace evxx {

constexpr int EMB = 32;   // MixingNetwork embed_dim (train_qmix.py:40)
constexpr int NMAX = 16;  // agents per launch
constexpr int ROWS = 256;
__host__ __device__ constexpr int mix_params(int n) { return n * EMB + EMB + EMB + 1; }

// per-row factors staged for the parameter sums: q_i (n), dh_j (32), hid_j (32), dqt
__global__ __launch_bounds__(ROWS) void qmix_rows_kernel(const float* __restrict__ Q, const float* __restrict__ Qt, int A,
                                                         const int32_t* __restrict__ act, const float* __restrict__ rew,
                                                         const uint8_t* __restrict__ done, float gamma, int B, int n,
                                                         const float* __restrict__ mix, const float* __restrict__ mix_t,
                                                         float* __restrict__ dQ, float* __restrict__ part, int nrow_blocks,
                                                         float* __restrict__ zero, int64_t nzero) {
    if ((int)blockIdx.x >= nrow_blocks) {  // clear the agents' gradients for the grouped backward
        const int64_t z0 = ((int64_t)blockIdx.x - nrow_blocks) * ROWS + threadIdx.x;
        const int64_t zs = ((int64_t)gridDim.x - nrow_blocks) * ROWS;
        for (int64_t k = z0; k < nzero; k += zs) zero[k] = 0.f;
        return;
    }
    extern __shared__ float sm[];  // [ROWS][n + 2 EMB + 2]
    const int W = n + 2 * EMB + 2;
    const int t = (int)threadIdx.x, b = (int)blockIdx.x * ROWS + t;
    float* rowf = sm + (size_t)t * W;
    const int NP = mix_params(n);
    const float* w1 = mix;
    const float* b1 = mix + n * EMB;
    const float* w2 = b1 + EMB;
    const float b2 = w2[EMB];
    const float* tw1 = mix_t;
    const float* tb1 = mix_t + n * EMB;
    const float* tw2 = tb1 + EMB;
    const float tb2 = tw2[EMB];
    float lossv = 0.f;
    if (b < B) {
        float q[NMAX], qt[NMAX];
        int a[NMAX];
        for (int i = 0; i < n; i++) {
            const size_t r = (size_t)i * B + b;
            a[i] = act[r];
            q[i] = Q[r * A + a[i]];  // q_network(s).gather(1, a)
            float mx = Qt[r * A];
            for (int j = 1; j < A; j++) mx = fmaxf(mx, Qt[r * A + j]);  // target_network(s').max(1)[0]
            qt[i] = mx;
        }
        // target mixer -> y (no gradient)
        float tot_t = 0.f;
        for (int j = 0; j < EMB; j++) {
            float pre = 0.f;
            for (int i = 0; i < n; i++) pre += qt[i] * fabsf(tw1[i * EMB + j]);
            pre += tb1[j];
            tot_t += (pre > 0.f ? pre : 0.f) * fabsf(tw2[j]);
        }
        tot_t += tb2;
        const float y = rew[b] + gamma * tot_t * (done[b] ? 0.f : 1.f);
        // online mixer
        float hid[EMB];
        float tot = 0.f;
        for (int j = 0; j < EMB; j++) {
            float pre = 0.f;
            for (int i = 0; i < n; i++) pre += q[i] * fabsf(w1[i * EMB + j]);
            pre += b1[j];
            hid[j] = pre > 0.f ? pre : 0.f;
            tot += hid[j] * fabsf(w2[j]);
        }
        tot += b2;
        const float d = tot - y;
        lossv = d * d;
        const float dqt = 2.f * d / (float)B;  // mse_loss(mean) backward
        float dq[NMAX];
        for (int i = 0; i < n; i++) dq[i] = 0.f;
        for (int j = 0; j < EMB; j++) {
            const float dh = hid[j] > 0.f ? dqt * fabsf(w2[j]) : 0.f;
            rowf[n + j] = dh;
            rowf[n + EMB + j] = hid[j];
            for (int i = 0; i < n; i++) dq[i] += dh * fabsf(w1[i * EMB + j]);
        }
        for (int i = 0; i < n; i++) {
            rowf[i] = q[i];
            const size_t r = (size_t)i * B + b;
            for (int j = 0; j < A; j++) dQ[r * A + j] = j == a[i] ? dq[i] : 0.f;
        }
        rowf[n + 2 * EMB] = dqt;
    } else {
        for (int k = 0; k < W; k++) rowf[k] = 0.f;
    }
    rowf[n + 2 * EMB + 1] = lossv;
    __syncthreads();
    // parameter k's gradient (w.r.t. |W| for the weights; sign applied in the reduce) over this
    // workgroup's rows, in row order; k = NP: the loss sum
    const int nr = min(ROWS, B - (int)blockIdx.x * ROWS);
    for (int k = t; k <= NP; k += ROWS) {
        float s = 0.f;
        if (k < n * EMB) {  // fc1_weight[i][j]: q_i * dh_j
            const int i = k / EMB, j = k - i * EMB;
            for (int r = 0; r < nr; r++) s += sm[(size_t)r * W + i] * sm[(size_t)r * W + n + j];
        } else if (k < n * EMB + EMB) {  // fc1_bias[j]: dh_j
            const int j = k - n * EMB;
            for (int r = 0; r < nr; r++) s += sm[(size_t)r * W + n + j];
        } else if (k < n * EMB + 2 * EMB) {  // fc2_weight[j]: dqt * hid_j
            const int j = k - n * EMB - EMB;
            for (int r = 0; r < nr; r++) s += sm[(size_t)r * W + n + 2 * EMB] * sm[(size_t)r * W + n + EMB + j];
        } else if (k == NP - 1) {  // fc2_bias: dqt
            for (int r = 0; r < nr; r++) s += sm[(size_t)r * W + n + 2 * EMB];
        } else {  // the loss
            for (int r = 0; r < nr; r++) s += sm[(size_t)r * W + n + 2 * EMB + 1];
        }
        part[(size_t)blockIdx.x * (NP + 1) + k] = s;
    }
}

__global__ __launch_bounds__(256) void qmix_reduce_kernel(const float* __restrict__ part, int nblk, int n, int B,
                                                          const float* __restrict__ mix, float* __restrict__ grad,
                                                          float* __restrict__ loss) {
    const int NP = mix_params(n);
    for (int k = (int)threadIdx.x; k <= NP; k += 256) {
        float s = 0.f;
        for (int z = 0; z < nblk; z++) s += part[(size_t)z * (NP + 1) + k];
        if (k == NP) {
            loss[0] = s / (float)B;
        } else {
            const bool absw = k < n * EMB || (k >= n * EMB + EMB && k < n * EMB + 2 * EMB);
            if (absw) {  // torch.abs backward: grad * sign(w)
                const float w = mix[k];
                s = w > 0.f ? s : (w < 0.f ? -s : 0.f);
            }
            grad[k] = s;
        }
    }
}

}  // namespace evxx

namespace {
thread_local char x_err[256] = "";
int xfail(int code, const char* msg) {
    snprintf(x_err, sizeof(x_err), "%s", msg);
    return code;
}
}  // namespace

extern "C" {

const char* evx_qmix_last_error(void) { return x_err; }

int32_t evx_qmix_nparams(int32_t n) { return evxx::mix_params(n); }

int64_t evx_qmix_part_floats(int32_t B, int32_t n) {
    if (B <= 0 || n <= 0) return 0;
    return (int64_t)((B + evxx::ROWS - 1) / evxx::ROWS) * (evxx::mix_params(n) + 1);
}

int evx_qmix_loss(const float* Q, const float* Qt, int32_t A, const int32_t* act, const float* rew, const uint8_t* done,
                  float gamma, int32_t B, int32_t n, const float* mix, const float* mix_t, float* dQ, float* mix_grad,
                  float* loss, float* part, float* zero, int64_t nzero, void* stream) {
    if (B <= 0) return 0;
    if (n < 1 || n > evxx::NMAX) return xfail(-22, "qmix_loss: 1..16 agents");
    if (A < 1 || A > 64) return xfail(-22, "qmix_loss: 1..64 actions");
    if (!Q || !Qt || !act || !rew || !done || !mix || !mix_t || !dQ || !mix_grad || !loss || !part)
        return xfail(-22, "qmix_loss: NULL argument");
    const int nrb = (B + evxx::ROWS - 1) / evxx::ROWS;
    const int nz = zero && nzero > 0 ? (int)std::min<int64_t>((nzero + 256 * 16 - 1) / (256 * 16), 512) : 0;
    const size_t lds = (size_t)evxx::ROWS * (n + 2 * evxx::EMB + 2) * 4;
    {
        static std::atomic<uint64_t> attr_done;
        const void* ks[1] = {(const void*)evxx::qmix_rows_kernel};
        evxh::max_lds_once(attr_done, ks, 1, 160 * 1024);
    }
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(evxx::qmix_rows_kernel, dim3(nrb + nz), dim3(evxx::ROWS), lds, st, Q, Qt, A, act, rew, done, gamma,
                       B, n, mix, mix_t, dQ, part, nrb, nz ? zero : nullptr, nzero);
    hipLaunchKernelGGL(evxx::qmix_reduce_kernel, dim3(1), dim3(256), 0, st, part, nrb, n, B, mix, mix_grad, loss);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(x_err, sizeof(x_err), "qmix_loss: %s", hipGetErrorString(e));
        return -5;
    }
    return 0;
}

}  // extern "C"
