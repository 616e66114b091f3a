// Static floor field on the device for many layouts at once:
// Map.Init_Potential (Louvre_Evacuation/envs/map.py:127-148) -- an 8-neighbour
// shortest-path field from the exits (initial distance 1, step cost 1.0 orthogonal /
// 1.4 diagonal, relaxing only cells that pass Check_Valid on the pre-potential grid),
// then + 200 * danger(t = 0)^2 on every reachable cell.
//
// The reference runs heapq Dijkstra with strict '<'. Adding a positive cost in float64
// is monotone, so Dijkstra's result is the least fixed point of
//     d[v] = min(d[v], min over neighbours u of fl(d[u] + cost(u, v)))
// over valid v with the sources at 1 -- the minimum over all paths of the left-fold
// rounded path sums. Any order of relaxations that runs to a fixed point reaches that
// same point, so a parallel in-place relaxation gives bit-identical float64 values.
//
// One 1024-thread workgroup per layout (layouts are independent: one per workgroup, no
// cross-workgroup traffic). The field lives in LDS when it fits (<= 18,432 cells =
// 144 KB of f64: up to a 133 x 133 padded grid) and in global memory (L2) otherwise.
// Each pass walks the thread's cells alternately forwards and backwards (in-place
// updates carry a value along the sweep within one pass); a pass with no change ends
// the loop. The +200 danger^2 term is an input (`pen`, computed on the host exactly as
// the reference: CPython float ** 2 is libm pow, which is not x * x for every x).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <string>

#include "evacx.h"
#include "evx_host.h"

namespace evxf {
constexpr int NT = 1024;
constexpr int LDS_CELLS = 18432;

static std::string g_err;
static int fail(int code, const std::string& m) {
    g_err = m;
    return code;
}

// MoveTO (envs/map.py:11-19): index < 4 orthogonal (cost 1.0), else diagonal (1.4)
__constant__ int MDX[8] = {1, 0, -1, 0, 1, -1, -1, 1};
__constant__ int MDY[8] = {0, -1, 0, 1, -1, -1, 1, 1};

template <bool INLDS>
__global__ __launch_bounds__(NT) void floor_kernel(int GX, int GY, const uint8_t* __restrict__ valid,
                                                   const uint8_t* __restrict__ source, const double* __restrict__ pen,
                                                   double* __restrict__ floor, int32_t* __restrict__ passes,
                                                   int max_passes) {
    extern __shared__ double sd[];
    __shared__ int changed;
    const int tid = threadIdx.x, n = GX * GY;
    const size_t base = (size_t)blockIdx.x * n;
    const uint8_t* V = valid + base;
    const uint8_t* S = source + base;
    double* D = INLDS ? sd : floor + base;
    const double inf = __builtin_inf();
    for (int c = tid; c < n; c += NT) D[c] = S[c] ? 1.0 : inf;
    const int per = (n + NT - 1) / NT;
    // cells this thread relaxes (valid, not an exit) as a register mask: bit k <-> cell
    // tid + k * NT for k < 64; beyond (grids over 65,536 cells) the flags are re-read
    uint64_t rm = 0;
    for (int k = 0; k < per && k < 64; k++) {
        const int c = tid + k * NT;
        if (c < n && V[c] && !S[c]) rm |= 1ull << k;
    }
    __syncthreads();
    int pass = 0;
    for (;;) {
        if (tid == 0) changed = 0;
        __syncthreads();
        bool any = false;
#pragma unroll 4
        for (int k0 = 0; k0 < per; k0++) {
            const int k = (pass & 1) ? per - 1 - k0 : k0;
            const int c = tid + k * NT;
            const bool relax = k < 64 ? ((rm >> k) & 1ull) != 0 : (c < n && V[c] && !S[c]);
            if (!relax) continue;  // sources stay at 1 (every path sum is >= 2)
            const int x = c / GY, y = c - x * GY;
            const double cur = D[c];
            double best = cur;
#pragma unroll
            for (int i = 0; i < 8; i++) {  // v = u + MoveTO[i]  <=>  u = v - MoveTO[i]
                const int ux = x - MDX[i], uy = y - MDY[i];
                if (ux < 0 || ux >= GX || uy < 0 || uy >= GY) continue;
                const double cand = D[ux * GY + uy] + (i < 4 ? 1.0 : 1.4);
                best = cand < best ? cand : best;
            }
            if (best < cur) {
                D[c] = best;
                any = true;
            }
        }
        if (any) changed = 1;
        __syncthreads();
        const int ch = changed;
        __syncthreads();
        pass++;
        if (!ch || pass >= max_passes) break;  // every wave reads the same flag: uniform exit
    }
    for (int c = tid; c < n; c += NT) {
        double d = D[c];
        if (d != inf && pen) d = d + pen[base + c];
        floor[base + c] = d;
    }
    if (tid == 0 && passes) passes[blockIdx.x] = pass;
}
}  // namespace evxf

extern "C" {

const char* evx_floor_last_error(void) { return evxf::g_err.c_str(); }

int evx_floor_field(int32_t n_layouts, int32_t GX, int32_t GY, const uint8_t* valid, const uint8_t* source,
                    const double* pen, double* floor, int32_t* passes, void* stream) {
    using namespace evxf;
    if (n_layouts <= 0) return 0;
    if (GX < 3 || GY < 3) return fail(-22, "floor_field: grid must be at least 3 x 3");
    if ((int64_t)GX * GY > (1 << 26)) return fail(-22, "floor_field: grid too large");
    if (!valid || !source || !floor) return fail(-22, "floor_field: NULL argument");
    const int n = GX * GY;
    const int max_passes = n + 2;  // a shortest path visits each cell once: n passes always suffice
    hipStream_t s = (hipStream_t)stream;
    if (n <= LDS_CELLS) {
        const size_t lds = (size_t)n * sizeof(double);
        static std::atomic<uint64_t> attr_done;
        bool ok = true;
        evxh::once_per_device(attr_done, [&] {
            ok = hipFuncSetAttribute((const void*)floor_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     LDS_CELLS * (int)sizeof(double)) == hipSuccess;
        });
        if (!ok) return fail(-5, "floor_field: cannot raise the LDS limit");
        hipLaunchKernelGGL(floor_kernel<true>, dim3(n_layouts), dim3(NT), lds, s, GX, GY, valid, source, pen, floor,
                           passes, max_passes);
    } else {
        hipLaunchKernelGGL(floor_kernel<false>, dim3(n_layouts), dim3(NT), 0, s, GX, GY, valid, source, pen, floor,
                           passes, max_passes);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(-5, std::string("floor_field launch: ") + hipGetErrorString(e));
    return 0;
}

}  // extern "C"
