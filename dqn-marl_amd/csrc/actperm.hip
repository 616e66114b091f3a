// Row order of the x3 act (DQNAgent.act, agents/dqn_agent.py:101-124, for every robot of every env):
// rows sorted by (table path or not, window centre). The act's table path starts fc1 from a
// per-centre row of the static features' contribution (2 KB per row, evx_qmlp_stat); rows that
// share a centre are then adjacent, so a 64-row tile reads a few table rows (L1 / L2 hits) instead
// of 64 scattered ones from the MALL. The act keeps every row's results and dropout mask at its own
// row (qact3h_kernel DM 3: each tile row hashes its own pair), so the order changes no result.
// A stable radix sort (rocPRIM) of (key << row) pairs: deterministic.
#include <cstdio>
#include <cstring>

#include <hip/hip_runtime.h>

#include <rocprim/rocprim.hpp>

#include "evacx.h"

namespace {
thread_local char p_err[256] = "";
int pfail(int code, const char* msg) {
    snprintf(p_err, sizeof(p_err), "%s", msg);
    return code;
}
constexpr unsigned KEY_BITS = 21;  // bit 20: not on the table path; bits 0-19: centre cell x (W + 2) + y

__global__ __launch_bounds__(256) void act_row_keys(const evx_obs* __restrict__ obs, int n, int L, int W, int t_max,
                                                    int stat_fs, int x0, int nx, uint32_t* __restrict__ keys,
                                                    int32_t* __restrict__ rows) {
    const int r = (int)(blockIdx.x * 256 + threadIdx.x);
    if (r >= n) return;
    const int4 c = *reinterpret_cast<const int4*>(&obs[r].cx);  // cx, cy, fire_step, layout
    const int fs = min(max(c.z, 0), t_max);
    const bool tab = stat_fs >= 0 && fs == stat_fs && c.x >= x0 && c.x < x0 + nx && c.y >= 0 && c.y <= W + 1;
    const int cx = min(max(c.x, 0), L + 1), cy = min(max(c.y, 0), W + 1);
    keys[r] = (tab ? 0u : 1u << 20) | (uint32_t)(cx * (W + 2) + cy);
    rows[r] = r;
}
}  // namespace

extern "C" {

const char* evx_act_row_perm_last_error(void) { return p_err; }

int64_t evx_act_row_perm_bytes(int32_t n) {
    if (n <= 0) return 0;
    size_t bytes = 0;
    if (rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const int32_t*)nullptr,
                                  (int32_t*)nullptr, (size_t)n, 0u, KEY_BITS) != hipSuccess)
        return -1;
    return (int64_t)bytes;
}

int evx_act_row_perm(const evx_layout* lay, const evx_obs* obs, int32_t n, int32_t stat_fs, int32_t stat_x0,
                     int32_t stat_nx, uint32_t* keys, int32_t* rows, int32_t* perm, void* temp, int64_t temp_bytes,
                     void* stream) {
    if (n <= 0) return 0;
    if (!lay || !obs || !keys || !rows || !perm || !temp) return pfail(-22, "act_row_perm: NULL argument");
    if ((int64_t)(lay->L + 2) * (lay->W + 2) > (1 << 20)) return pfail(-22, "act_row_perm: grid too large for the key");
    const int64_t need = evx_act_row_perm_bytes(n);
    if (need < 0 || temp_bytes < need) return pfail(-22, "act_row_perm: temp storage too small (evx_act_row_perm_bytes)");
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(act_row_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, obs, n, lay->L, lay->W,
                       lay->t_max, stat_fs, stat_x0, stat_nx, keys, rows);
    if (hipGetLastError() != hipSuccess) return pfail(-5, "act_row_perm: key launch failed");
    size_t bytes = (size_t)temp_bytes;
    if (rocprim::radix_sort_pairs(temp, bytes, (const uint32_t*)keys, keys + n, (const int32_t*)rows, perm, (size_t)n,
                                  0u, KEY_BITS, st) != hipSuccess)
        return pfail(-5, "act_row_perm: radix sort failed");
    return 0;
}

}  // extern "C"
