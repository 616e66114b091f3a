// MI355X (gfx950) evacuation cellular automaton: env reset / step / observation.
//
// One 256-thread workgroup owns one env instance for a whole step. Person state
// (packed cell+flags, health f64, acc f64) lives in registers, K persons per
// thread (person p = tid + k*256, so every global access is coalesced). The
// occupancy grid is an LDS bitmap, the move-conflict table an LDS array of
// 16-bit entries, and the two MT19937 streams LDS rings (evx_device.h).
//
// The step is the reference's EvacuationEnv.step (envs/evacuation_env.py:122-172)
// and EvacuationEnvMulti.step (envs/evacuation_env_multi.py:55-89), evaluated
// bit-exactly in parallel:
//   * RNG draws are assigned to persons by prefix sums in person order, so the
//     parallel planners read exactly the words the sequential reference loop
//     consumes (numpy stream: People.update_health envs/people.py:61-88;
//     Python stream: People.find_best_direction envs/people.py:255-297);
//   * move_plan's dict insertion order == the order of each target's FIRST
//     planner, found by an LDS atomic-min per target cell;
//   * random.shuffle runs only for contested targets, in that order, on lane 0;
//   * execute_move's last-writer-wins on People.rmap (envs/people.py:299-314)
//     becomes an atomic-max of (first-planner, sub-step) per touched cell.
// f64 arithmetic is compiled with -ffp-contract=off (no FMA) to match CPython.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "evacx.h"
#include "evx_device.h"

namespace evx {

constexpr int RING_PY = 4096;  // >= 256 persons x 8 candidates x 2 words
constexpr int RING_NP = 1024;  // >= 256 persons x 2 words, >= 851
constexpr int GRP_CAP = 256;
constexpr uint32_t NIL = 0xffffffffu;
constexpr int SHUF_CHUNK = 2048;

// MoveTO (envs/map.py:11-19)
__constant__ int c_dx[8] = {1, 0, -1, 0, 1, -1, -1, 1};
__constant__ int c_dy[8] = {0, -1, 0, 1, -1, -1, 1, 1};

struct Geo {
    int L, W, GY, G, RW, P, R;
};

__device__ __forceinline__ int pk_x(uint32_t v) { return v & 0xfff; }
__device__ __forceinline__ int pk_y(uint32_t v) { return (v >> 12) & 0xfff; }
__device__ __forceinline__ bool pk_safe(uint32_t v) { return (v >> 24) & 1; }
__device__ __forceinline__ bool pk_dead(uint32_t v) { return (v >> 25) & 1; }
__device__ __forceinline__ int rp_x(uint32_t v) { return (int)(int16_t)(v & 0xffff); }
__device__ __forceinline__ int rp_y(uint32_t v) { return (int)(int16_t)(v >> 16); }
__device__ __forceinline__ uint32_t rp_pack(int x, int y) {
    return (uint32_t)(uint16_t)(int16_t)x | ((uint32_t)(uint16_t)(int16_t)y << 16);
}
__device__ __forceinline__ bool bit_get(const uint32_t* b, int i) { return (b[i >> 5] >> (i & 31)) & 1u; }

// Map.Check_Valid on integer coordinates (envs/map.py:85-92)
__device__ __forceinline__ bool check_valid(const Geo& g, const uint32_t* validb, int x, int y) {
    if (x >= g.L + 1 || x <= 0 || y >= g.W + 1 || y <= 0) return false;
    return bit_get(validb, x * g.GY + y);
}

// Person.update_health (envs/people.py:61-88); returns true if the person died.
__device__ __forceinline__ bool update_health(double& h, double danger, double u) {
    double loss;
    if (danger >= 0.8) loss = danger * 50.0 + (1.0 + (3.0 - 1.0) * u);
    else if (danger >= 0.5) loss = danger * 40.0 + (0.8 + (2.0 - 0.8) * u);
    else if (danger >= 0.2) loss = danger * 30.0 + (0.5 + (1.5 - 0.5) * u);
    else loss = danger * 20.0 + (0.2 + (1.0 - 0.2) * u);
    if (h < 50) loss *= 1.2;
    h -= loss;
    bool dead = false;
    if (h <= 0) {
        h = 0;
        dead = true;
    } else if (h <= 8.0) {
        dead = true;
    }
    return dead;
}

// Person.update_state speed (envs/people.py:37-44)
__device__ __forceinline__ double person_speed(double h) {
    if (h < 20) return 0.4;
    return 1.0 * (0.3 + 0.7 * (h / 100.0));
}

// Build the compact observation of one robot with one wave (bits by ballot).
__device__ __forceinline__ void write_obs(const Geo& g, const uint32_t* validb, const uint32_t* rmapb, int cx,
                                          int cy, int fs, evx_obs* dst) {
    const int lane = threadIdx.x & 63;
    bool b0 = false, b1 = false;
    {
        const int c = lane, i = c / 11, j = c % 11;
        const int mx = cx + i - 5, my = cy + j - 5;
        if (check_valid(g, validb, mx, my)) b0 = bit_get(rmapb, mx * g.GY + my);
    }
    {
        const int c = lane + 64, i = c / 11, j = c % 11;
        const int mx = cx + i - 5, my = cy + j - 5;
        if (c < 121 && check_valid(g, validb, mx, my)) b1 = bit_get(rmapb, mx * g.GY + my);
    }
    const unsigned long long m0 = __ballot(b0), m1 = __ballot(b1);
    if (lane == 0) {
        uint4 a = make_uint4((uint32_t)m0, (uint32_t)(m0 >> 32), (uint32_t)m1, (uint32_t)(m1 >> 32));
        uint4 b = make_uint4((uint32_t)cx, (uint32_t)cy, (uint32_t)fs, 0u);
        reinterpret_cast<uint4*>(dst)[0] = a;
        reinterpret_cast<uint4*>(dst)[1] = b;
    }
}

// Store the MT state after consuming up to raw index `head` (CPython index semantics).
__device__ __forceinline__ void mt_store(uint32_t* ring, int mask, int& front, int head, uint32_t* gst) {
    if (head <= MT_N) {
        // no twist happened: words unchanged, only the index moves
        if (threadIdx.x == 0) gst[MT_N] = (uint32_t)head;
        return;
    }
    const int b = MT_N * ((head - 1) / MT_N);
    mt_ensure(ring, mask, front, b + MT_N);
    for (int i = threadIdx.x; i < MT_N; i += NT) gst[i] = ring[(b + i) & mask];
    if (threadIdx.x == 0) gst[MT_N] = (uint32_t)(head - b);
}

__device__ __forceinline__ void mt_load(uint32_t* ring, const uint32_t* gst, int& head) {
    for (int i = threadIdx.x; i < MT_N; i += NT) ring[i] = gst[i];
    head = (int)gst[MT_N];
}

struct StepLds {
    // word offsets into dynamic LDS
    int regionA, claim, pyring, npring, rmapb, validb, lhead, lnext, confl, grp, robots, wsum, dsum, ctrl, total;
    int regionA_words;
};

__host__ __device__ inline StepLds step_lds(int G, int P, int R) {
    StepLds s;
    const int RW = (G + 31) / 32;
    const int CW = (G + 1) / 2;
    int a = CW + RING_PY + RING_NP;
    if (a < 4 * P) a = 4 * P;
    a = (a + 3) & ~3;
    int o = 0;
    s.regionA = o;
    s.claim = o;
    s.pyring = o + CW;
    s.npring = o + CW + RING_PY;
    s.regionA_words = a;
    o += a;
    s.rmapb = o; o += RW;
    s.validb = o; o += RW;
    s.lhead = o; o += P;
    s.lnext = o; o += (P + 1) / 2;
    s.confl = o; o += (P + 31) / 32;
    s.grp = o; o += GRP_CAP;
    s.robots = o; o += R;
    o = (o + 1) & ~1;
    s.wsum = o; o += NWAVE;
    o = (o + 1) & ~1;
    s.dsum = o; o += 2 * NWAVE + 8;
    s.ctrl = o; o += 16;
    s.total = (o + 3) & ~3;
    return s;
}

template <int K>
__global__ __launch_bounds__(NT) void env_step_kernel(evx_layout lay, evx_state st, const int32_t* __restrict__ actions,
                                                      evx_step_out out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int e = blockIdx.x;
    const int tid = threadIdx.x;
    Geo g;
    g.L = lay.L; g.W = lay.W; g.GY = lay.W + 2; g.G = (lay.L + 2) * (lay.W + 2);
    g.RW = (g.G + 31) / 32; g.P = lay.P; g.R = lay.R;
    const int P = g.P, R = g.R;
    const StepLds S = step_lds(g.G, P, R);
    uint32_t* claim = smem + S.claim;
    uint32_t* pyring = smem + S.pyring;
    uint32_t* npring = smem + S.npring;
    uint32_t* rmapb = smem + S.rmapb;
    uint32_t* validb = smem + S.validb;
    uint32_t* lhead = smem + S.lhead;
    uint16_t* lnext = reinterpret_cast<uint16_t*>(smem + S.lnext);
    uint32_t* confl = smem + S.confl;
    int* grp = reinterpret_cast<int*>(smem + S.grp);
    uint32_t* robots = smem + S.robots;
    int* wsum = reinterpret_cast<int*>(smem + S.wsum);
    double* dsum = reinterpret_cast<double*>(smem + S.dsum);
    int* ctrl = reinterpret_cast<int*>(smem + S.ctrl);
    double* distbuf = reinterpret_cast<double*>(smem + S.regionA);
    double* hbuf = distbuf + P;

    // ---------------------------------------------------------------- load
    const int CW = (g.G + 1) / 2;
    for (int i = tid; i < g.RW; i += NT) {
        rmapb[i] = st.rmap[(size_t)e * g.RW + i];
        validb[i] = lay.valid_bits[i];
    }
    for (int i = tid; i < CW; i += NT) claim[i] = 0xffffffffu;
    for (int i = tid; i < P; i += NT) lhead[i] = NIL;
    for (int i = tid; i < (P + 31) / 32; i += NT) confl[i] = 0;
    int py_head, np_head;
    mt_load(pyring, st.py_mt + (size_t)e * EVX_MT_WORDS, py_head);
    mt_load(npring, st.np_mt + (size_t)e * EVX_MT_WORDS, np_head);
    int py_front = MT_N, np_front = MT_N;
    const int* scal_g = st.scal + (size_t)e * 4;
    const int fs = scal_g[0], cur_step = scal_g[1], prev_evac = scal_g[2], prev_dead = scal_g[3];
    uint32_t view = st.view[e];
    // Map.move_robot for every robot (envs/map.py:160-201); robots never interact.
    if (tid < R) {
        uint32_t rp = st.robots[(size_t)e * R + tid];
        const int a = actions[(size_t)e * R + tid];
        if (a >= 0 && a <= 4) {
            const int x = rp_x(rp), y = rp_y(rp);
            int nx = x, ny = y;
            if (a == 0) nx = x + 1;
            else if (a == 1) ny = y - 1;
            else if (a == 2) nx = x - 1;
            else if (a == 3) ny = y + 1;
            if (lay.rx_lo <= nx && nx <= lay.rx_hi && 0 <= ny && ny <= g.W && nx >= 1 && nx <= g.L && ny >= 1 &&
                ny <= g.W && ((lay.valid_bits[(nx * g.GY + ny) >> 5] >> ((nx * g.GY + ny) & 31)) & 1u))
                rp = rp_pack(nx, ny);
        }
        robots[tid] = rp;
        st.robots[(size_t)e * R + tid] = rp;
        if (tid == 0) ctrl[0] = (a >= 0 && a <= 4) ? 1 : 0;
    }
    __syncthreads();
    if (ctrl[0]) view = robots[0];  // robot_position refreshed only after a valid action
    __syncthreads();

    // ------------------------------------------------ per-person registers
    uint32_t pk[K];
    double hh[K], ac[K];
    int tg[K], pfv[K];
    bool act0[K];
    const uint32_t* pk_g = st.pk + (size_t)e * P;
    const double* h_g = st.health + (size_t)e * P;
    const double* a_g = st.acc + (size_t)e * P;
#pragma unroll
    for (int k = 0; k < K; k++) {
        const int p = tid + k * NT;
        pk[k] = (p < P) ? pk_g[p] : (3u << 24);
        act0[k] = (p < P) && !((pk[k] >> 24) & 3u);
        // health of every non-dead person feeds the reward's sum (safe ones included)
        hh[k] = ((p < P) && !((pk[k] >> 25) & 1u)) ? h_g[p] : 0.0;
        ac[k] = act0[k] ? a_g[p] : 0.0;
        tg[k] = -1;
        pfv[k] = -1;
    }
    const double* dpt = lay.danger_p + (size_t)fs * g.G;

    // ------------------------------- People.run phases 1+2, row by row
#pragma unroll
    for (int k = 0; k < K; k++) {
        const int p = tid + k * NT;
        // phase 1: Person.update_state -> update_health (numpy stream)
        double dg = 0.0;
        if (act0[k]) dg = dpt[pk_x(pk[k]) * g.GY + pk_y(pk[k])];
        const bool need = act0[k] && dg > 0;
        int tot;
        int off = block_exscan(need ? 2 : 0, wsum, tot);
        mt_ensure(npring, RING_NP - 1, np_front, np_head + tot);
        bool alive = act0[k];
        if (need) {
            const double u = mt_double(npring, RING_NP - 1, np_head + off);
            if (update_health(hh[k], dg, u)) {
                pk[k] |= (2u << 24);
                alive = false;
            }
        }
        np_head += tot;
        // phase 2: accumulate, plan with find_best_direction (Python stream)
        bool planner = false;
        if (alive) {
            ac[k] += person_speed(hh[k]) * 0.5;
            if (ac[k] >= 1.0) {
                ac[k] -= 1.0;
                planner = true;
            }
        }
        int cand = 0, ncand = 0;
        const int x = pk_x(pk[k]), y = pk_y(pk[k]);
        if (planner) {
#pragma unroll
            for (int d = 0; d < 8; d++) {
                const int nx = x + c_dx[d], ny = y + c_dy[d];
                if (check_valid(g, validb, nx, ny) && !bit_get(rmapb, nx * g.GY + ny)) {
                    cand |= 1 << d;
                    ncand++;
                }
            }
        }
        off = block_exscan(2 * ncand, wsum, tot);
        mt_ensure(pyring, RING_PY - 1, py_front, py_head + tot);
        if (planner && ncand) {
            const double fxy = lay.floor[x * g.GY + y];
            int best = -1;
            double maxs = -INFINITY;
            int idx = py_head + off;
            for (int d = 0; d < 8; d++) {
                if (!((cand >> d) & 1)) continue;
                const int nx = x + c_dx[d], ny = y + c_dy[d];
                const double delta_p = fxy - lay.floor[nx * g.GY + ny];
                int md2 = 0x7fffffff;
                for (int r = 0; r < R; r++) {
                    const uint32_t rp = robots[r];
                    const int dx = nx - rp_x(rp), dy = ny - rp_y(rp);
                    const int d2 = dx * dx + dy * dy;
                    md2 = d2 < md2 ? d2 : md2;
                }
                double effect = 0.0;
                if (md2 < lay.repel_d2) effect = lay.repel_k / (sqrt((double)md2) + 0.1);
                const double u = -0.1 + (0.1 - -0.1) * mt_double(pyring, RING_PY - 1, idx);
                idx += 2;
                const double score = delta_p * 5.0 + effect + u;
                if (score > maxs) {
                    maxs = score;
                    best = d;
                }
            }
            if (best >= 0) tg[k] = (x + c_dx[best]) * g.GY + (y + c_dy[best]);
        }
        py_head += tot;
        (void)p;
    }

    // ------------------------------------ targets: first planner per cell
#pragma unroll
    for (int k = 0; k < K; k++)
        if (tg[k] >= 0) lds_min16(claim, tg[k], (uint32_t)(tid + k * NT));
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; k++) {
        if (tg[k] >= 0) {
            const int p = tid + k * NT;
            const int pf = (int)lds_read16(claim, tg[k]);
            pfv[k] = pf;
            if (pf != p) {
                atomicOr(&confl[pf >> 5], 1u << (pf & 31));
                const uint32_t old = atomicExch(&lhead[pf], (uint32_t)p);
                lnext[p] = (uint16_t)(old & 0xffffu);
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; k++)
        if (tg[k] >= 0 && pfv[k] == tid + k * NT) lds_set16_ffff(claim, tg[k]);

    // ------------------------- random.shuffle of contested targets (lane 0)
    if (tid == 0) {
        ctrl[0] = 0;                 // word index into confl
        ctrl[1] = (int)confl[0];     // remaining bits of that word
        ctrl[2] = py_head;
        ctrl[3] = 0;                 // done
        ctrl[4] = 0;                 // error
    }
    __syncthreads();
    {
        const int NCW = (P + 31) / 32;
        int last_head = -1;
        while (true) {
            const int h0 = ctrl[2];
            mt_ensure(pyring, RING_PY - 1, py_front, h0 + SHUF_CHUNK);
            __syncthreads();
            if (tid == 0) {
                int wi = ctrl[0];
                uint32_t m = (uint32_t)ctrl[1];
                int head = ctrl[2];
                int done = 0;
                const int avail = py_front;
                while (true) {
                    while (m == 0) {
                        wi++;
                        if (wi >= NCW) break;
                        m = confl[wi];
                    }
                    if (wi >= NCW) {
                        done = 1;
                        break;
                    }
                    const int pf = wi * 32 + (__ffs(m) - 1);
                    int n = 0;
                    grp[n++] = pf;
                    for (uint32_t q = lhead[pf]; q != NIL && (q & 0xffffu) != 0xffffu; q = lnext[q]) {
                        if (n >= GRP_CAP) {
                            ctrl[4] = 1;
                            break;
                        }
                        grp[n++] = (int)q;
                    }
                    for (int a = 2; a < n; a++) {  // movers in person order
                        const int v = grp[a];
                        int b = a - 1;
                        while (b >= 1 && grp[b] > v) {
                            grp[b + 1] = grp[b];
                            b--;
                        }
                        grp[b + 1] = v;
                    }
                    const int hsave = head;
                    bool ok = true;
                    for (int i = n - 1; i >= 1 && ok; i--) {  // Lib/random.py shuffle
                        const uint32_t bound = (uint32_t)(i + 1);
                        const int kb = bit_length(bound);
                        uint32_t r;
                        while (true) {
                            if (head >= avail) {
                                ok = false;
                                break;
                            }
                            r = mt_word(pyring, RING_PY - 1, head++) >> (32 - kb);
                            if (r < bound) break;
                        }
                        if (ok) {
                            const int t = grp[i];
                            grp[i] = grp[r];
                            grp[r] = t;
                        }
                    }
                    if (!ok) {
                        head = hsave;
                        break;
                    }
                    lhead[pf] = (uint32_t)grp[0];  // winner
                    m &= m - 1;
                }
                ctrl[0] = wi;
                ctrl[1] = (int)m;
                ctrl[2] = head;
                ctrl[3] = done;
            }
            __syncthreads();
            if (ctrl[3]) break;
            if (ctrl[2] == last_head) {  // no progress: cannot happen with sane streams
                if (tid == 0) ctrl[4] = 2;
                break;
            }
            last_head = ctrl[2];
        }
        py_head = ctrl[2];
        if (ctrl[4] && out.err && tid == 0) atomicOr(out.err, ctrl[4]);
    }
    __syncthreads();

    // --------------------------------------------- execute_move, in order
    // event code: min over 0xffff - (first_planner<<2 | sub<<1 | value)
    uint32_t code_old[K], code_new[K];
    int oldc[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        code_old[k] = code_new[k] = 0;
        oldc[k] = -1;
        if (tg[k] >= 0) {
            const int p = tid + k * NT;
            const int pf = pfv[k];
            const bool contested = (confl[pf >> 5] >> (pf & 31)) & 1u;
            const int w = contested ? (int)lhead[pf] : pf;
            const int cell_old = pk_x(pk[k]) * g.GY + pk_y(pk[k]);
            if (w == p) {
                const bool ex = (lay.cellinfo[tg[k]] >> 1) & 1u;
                code_old[k] = 0xffffu - (((uint32_t)pf << 2) | 0u);
                code_new[k] = 0xffffu - (((uint32_t)pf << 2) | 2u | (ex ? 0u : 1u));
                oldc[k] = cell_old;
                lds_min16(claim, cell_old, code_old[k]);
                lds_min16(claim, tg[k], code_new[k]);
                const int nx = tg[k] / g.GY, ny = tg[k] % g.GY;
                pk[k] = (uint32_t)nx | ((uint32_t)ny << 12) | (ex ? (1u << 24) : 0u);
                if (st.thmap) atomicAdd(&st.thmap[(size_t)e * g.G + tg[k]], 1);
            } else {
                if (st.thmap) atomicAdd(&st.thmap[(size_t)e * g.G + cell_old], 1);
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; k++) {
        if (oldc[k] >= 0) {
            if (lds_read16(claim, oldc[k]) == code_old[k])
                atomicAnd(&rmapb[oldc[k] >> 5], ~(1u << (oldc[k] & 31)));
            if (lds_read16(claim, tg[k]) == code_new[k]) {
                if (code_new[k] & 1u)  // value 0 (safe): code = ffff - (..|2|0) -> low bit 1
                    atomicAnd(&rmapb[tg[k] >> 5], ~(1u << (tg[k] & 31)));
                else
                    atomicOr(&rmapb[tg[k] >> 5], 1u << (tg[k] & 31));
            }
        }
    }
    // MT states go out now: the reward scratch below reuses the ring memory
    mt_store(pyring, RING_PY - 1, py_front, py_head, st.py_mt + (size_t)e * EVX_MT_WORDS);
    mt_store(npring, RING_NP - 1, np_front, np_head, st.np_mt + (size_t)e * EVX_MT_WORDS);
    __syncthreads();
    for (int i = tid; i < g.RW; i += NT) st.rmap[(size_t)e * g.RW + i] = rmapb[i];

    // ---------------------------------- fire update (both fire models)
    const int fs1 = fs < lay.t_max ? fs + 1 : fs;

    // ------------------------------------ _calculate_reward + counters
    const int vx = rp_x(view), vy = rp_y(view);
    int evac_t = 0, dead_t = 0;
    double gq_t = 0.0;
    int nrem = 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
        const int p = tid + k * NT;
        const bool inr = p < P;
        const bool sf = inr && pk_safe(pk[k]), dd = inr && pk_dead(pk[k]);
        evac_t += sf;
        dead_t += dd;
        const bool rem = inr && !sf && !dd;
        const int x2 = 2 * pk_x(pk[k]) + 1, y2 = 2 * pk_y(pk[k]) + 1;
        const long long dxr = x2 - 2LL * vx, dyr = y2 - 2LL * vy;
        const long long n4 = dxr * dxr + dyr * dyr;  // (2*distance)^2, exact
        if (rem && n4 <= 100) {
            const long long ex2 = x2 - 2LL * lay.exit_x, ey2 = y2 - 2LL * lay.exit_y;
            const long long ne = ex2 * ex2 + ey2 * ey2;
            if (ne > 1600) gq_t += 2.0;
            else if (ne > 400) gq_t += 1.5;
            else gq_t += 1.0;
            if (hh[k] < 80) gq_t += 1.0;
        }
        int tot;
        const int off = block_exscan(rem ? 1 : 0, wsum, tot);
        if (rem) distbuf[nrem + off] = 0.5 * sqrt((double)n4);
        nrem += tot;
        if (inr) hbuf[p] = dd ? -1.0 : hh[k];
    }
    const int evac = block_sum(evac_t, wsum);
    const int dead = block_sum(dead_t, wsum);
    const double gq = block_sum_d(gq_t, dsum);
    // order-sensitive f64 sums: Python sum (sequential) and numpy pairwise mean
    if (tid == 0) {
        double total = 0.0;
        for (int p = 0; p < P; p++) {
            const double v = hbuf[p];
            if (v >= 0.0) total += v;
        }
        dsum[2 * NWAVE] = total;
    } else if (tid == 64) {
        dsum[2 * NWAVE + 1] = nrem > 0 ? np_pairwise_sum(distbuf, nrem) / (double)nrem : 0.0;
    }
    __syncthreads();
    if (tid == 0) {
        const int remaining = P - evac - dead;
        double reward = 0.0;
        reward += (evac - prev_evac) * lay.evac_reward;
        reward += gq;
        if (remaining > 0) {
            const double avg = dsum[2 * NWAVE + 1];
            const double dr = 2.0 - fabs(avg - 8.0) * 0.2;
            reward += dr > 0 ? dr : 0.0;
        }
        if (remaining > 0) {
            const double urgency = (double)remaining / (double)P;
            reward += -0.05 - (urgency * 0.1);
        } else {
            reward -= 0.02;
        }
        const double total = dsum[2 * NWAVE];
        if (P - dead > 0) {
            const double avg_h = total / (double)(P - dead);
            reward += (avg_h - 90) * 0.05;
        }
        if (evac == P) {
            const int tb = 300 - cur_step;
            const double time_bonus = (tb > 0 ? tb : 0) * 0.2;
            const double fah = total / (double)P;  // no one is dead when all evacuated
            reward += 100 + time_bonus + (fah - 80) * 1.0;
        }
        reward -= (dead - prev_dead) * lay.death_penalty;
        reward -= dead * lay.death_acc_penalty;
        reward += (P - dead) * lay.alive_bonus;
        if (cur_step > 0) {
            const double eff = (double)evac / (double)cur_step;
            if (eff > 0.1) reward += eff * 5;
        }
        const int step1 = cur_step + 1;
        out.reward[e] = reward;
        out.done[e] = (evac + dead == P) || (0.5 * (double)step1 >= 600.0);
        if (out.counts) {
            out.counts[2 * e] = evac;
            out.counts[2 * e + 1] = dead;
        }
        int* sg = st.scal + (size_t)e * 4;
        sg[0] = fs1;
        sg[1] = step1;
        sg[2] = evac;
        sg[3] = dead;
        st.view[e] = view;
    }

    // ------------------------------------------------- observations
    {
        const int w = tid >> 6;
        for (int r = w; r < R; r += NWAVE) {
            const uint32_t c = (r == 0) ? view : robots[r];
            write_obs(g, validb, rmapb, rp_x(c), rp_y(c), fs1, out.obs + (size_t)e * R + r);
        }
    }

    // ---------------------------------------------------- store state
    uint32_t* pk_o = st.pk + (size_t)e * P;
    double* h_o = st.health + (size_t)e * P;
    double* a_o = st.acc + (size_t)e * P;
#pragma unroll
    for (int k = 0; k < K; k++) {
        const int p = tid + k * NT;
        if (act0[k]) {
            pk_o[p] = pk[k];
            h_o[p] = hh[k];
            a_o[p] = ac[k];
        }
    }
}

// ------------------------------------------------------------------ reset
struct ResetLds {
    int pyring, validb, rmapb, pos, ctrl, total;
};
__host__ __device__ inline ResetLds reset_lds(int G, int P) {
    ResetLds s;
    const int RW = (G + 31) / 32;
    int o = 0;
    s.pyring = o; o += RING_PY;
    s.validb = o; o += RW;
    s.rmapb = o; o += RW;
    s.pos = o; o += P;
    s.ctrl = o; o += 8;
    s.total = (o + 3) & ~3;
    return s;
}

__global__ __launch_bounds__(NT) void env_reset_kernel(evx_layout lay, evx_state st, const uint8_t* __restrict__ mask,
                                                       evx_obs* obs, int32_t* err) {
    const int e = blockIdx.x;
    if (mask && !mask[e]) return;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int tid = threadIdx.x;
    Geo g;
    g.L = lay.L; g.W = lay.W; g.GY = lay.W + 2; g.G = (lay.L + 2) * (lay.W + 2);
    g.RW = (g.G + 31) / 32; g.P = lay.P; g.R = lay.R;
    const int P = g.P, R = g.R;
    const ResetLds S = reset_lds(g.G, P);
    uint32_t* pyring = smem + S.pyring;
    uint32_t* validb = smem + S.validb;
    uint32_t* rmapb = smem + S.rmapb;
    uint32_t* pos = smem + S.pos;
    int* ctrl = reinterpret_cast<int*>(smem + S.ctrl);
    for (int i = tid; i < g.RW; i += NT) {
        validb[i] = lay.valid_bits[i];
        rmapb[i] = 0;
    }
    int py_head;
    mt_load(pyring, st.py_mt + (size_t)e * EVX_MT_WORDS, py_head);
    int py_front = MT_N;
    if (tid == 0) {
        ctrl[0] = 0;        // next person
        ctrl[1] = py_head;  // stream head
        ctrl[2] = 0;        // done
    }
    __syncthreads();
    // People.__init__ placement (envs/people.py:183-194): sequential rejection
    // sampling with random.randint(1, L-2) / randint(1, W-2).
    const uint32_t nx = (uint32_t)(g.L - 2), ny = (uint32_t)(g.W - 2);
    const int kx = bit_length(nx), ky = bit_length(ny);
    int last = -1;
    while (true) {
        const int h0 = ctrl[1];
        mt_ensure(pyring, RING_PY - 1, py_front, h0 + SHUF_CHUNK);
        __syncthreads();
        if (tid == 0) {
            int i = ctrl[0], head = ctrl[1];
            const int avail = py_front;
            while (i < P) {
                const int hs = head;
                bool ok = true;
                int x = 0, y = 0;
                while (true) {
                    uint32_t r;
                    do {
                        if (head >= avail) { ok = false; break; }
                        r = mt_word(pyring, RING_PY - 1, head++) >> (32 - kx);
                    } while (r >= nx);
                    if (!ok) break;
                    x = 1 + (int)r;
                    do {
                        if (head >= avail) { ok = false; break; }
                        r = mt_word(pyring, RING_PY - 1, head++) >> (32 - ky);
                    } while (r >= ny);
                    if (!ok) break;
                    y = 1 + (int)r;
                    if (check_valid(g, validb, x, y)) break;
                }
                if (!ok) {
                    head = hs;
                    break;
                }
                pos[i] = (uint32_t)x | ((uint32_t)y << 12);
                i++;
            }
            ctrl[0] = i;
            ctrl[1] = head;
            ctrl[2] = (i >= P);
        }
        __syncthreads();
        if (ctrl[2]) break;
        if (ctrl[1] == last) {
            if (tid == 0 && err) atomicOr(err, 4);
            break;
        }
        last = ctrl[1];
    }
    py_head = ctrl[1];
    uint32_t* pk_o = st.pk + (size_t)e * P;
    double* h_o = st.health + (size_t)e * P;
    double* a_o = st.acc + (size_t)e * P;
    for (int p = tid; p < P; p += NT) {
        const uint32_t v = pos[p];
        pk_o[p] = v;
        h_o[p] = 100.0;
        a_o[p] = 0.0;
        const int c = (int)(v & 0xfff) * g.GY + (int)((v >> 12) & 0xfff);
        atomicOr(&rmapb[c >> 5], 1u << (c & 31));
    }
    if (st.thmap) {
        int32_t* th = st.thmap + (size_t)e * g.G;
        for (int i = tid; i < g.G; i += NT) th[i] = 0;
        __syncthreads();
        for (int p = tid; p < P; p += NT) {
            const uint32_t v = pos[p];
            th[(int)(v & 0xfff) * g.GY + (int)((v >> 12) & 0xfff)] = 1;
        }
    }
    __syncthreads();
    for (int i = tid; i < g.RW; i += NT) st.rmap[(size_t)e * g.RW + i] = rmapb[i];
    uint32_t view;
    if (lay.reset_robots) {
        if (tid < R) st.robots[(size_t)e * R + tid] = rp_pack(lay.robot_init[2 * tid], lay.robot_init[2 * tid + 1]);
        view = rp_pack(lay.robot_init[0], lay.robot_init[1]);
    } else {
        view = rp_pack(lay.reset_view_x, lay.reset_view_y);
    }
    __syncthreads();
    if (tid == 0) {
        st.view[e] = view;
        int* sg = st.scal + (size_t)e * 4;
        sg[1] = 0;
        sg[2] = 0;
        sg[3] = 0;
    }
    const int fs = st.scal[(size_t)e * 4];
    if (obs) {
        const int w = tid >> 6;
        for (int r = w; r < R; r += NWAVE) {
            const uint32_t c = (r == 0) ? view : st.robots[(size_t)e * R + r];
            write_obs(g, validb, rmapb, rp_x(c), rp_y(c), fs, obs + (size_t)e * R + r);
        }
    }
    mt_store(pyring, RING_PY - 1, py_front, py_head, st.py_mt + (size_t)e * EVX_MT_WORDS);
}

// ---------------------------------------------------- observation expand
// EvacuationEnv._get_state (envs/evacuation_env.py:84-120) from the compact form.
template <typename T>
__global__ __launch_bounds__(256) void obs_expand_kernel(evx_layout lay, const evx_obs* __restrict__ obs, int64_t n,
                                                         T* __restrict__ out) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = n * 726;
    if (gid >= total) return;
    const int64_t o = gid / 726;
    const int rem = (int)(gid - o * 726);
    const int c = rem / 6, ch = rem - c * 6;
    const int i = c / 11, j = c - i * 11;
    const evx_obs ob = obs[o];
    const int mx = ob.cx + i - 5, my = ob.cy + j - 5;
    const int GY = lay.W + 2;
    const bool inb = mx >= 0 && mx <= lay.L + 1 && my >= 0 && my <= lay.W + 1;
    const bool valid = mx >= 1 && mx <= lay.L && my >= 1 && my <= lay.W && (lay.cellinfo[mx * GY + my] & 1u);
    T v = 0;
    if (ch == 1) {
        v = ((ob.occ[c >> 5] >> (c & 31)) & 1u) ? (T)1 : (T)0;
    } else if (ch == 2) {
        const int ti = mx - lay.ox0, tj = my - lay.oy0;
        if (ti >= 0 && ti < lay.OX && tj >= 0 && tj < lay.OY) {
            const size_t idx = ((size_t)ob.fire_step * lay.OX + ti) * lay.OY + tj;
            if constexpr (sizeof(T) == 8) v = (T)lay.danger_o[idx];
            else v = (T)lay.danger_o32[idx];
        }
    } else if (ch == 3) {
        v = (!valid || (inb && ((lay.cellinfo[mx * GY + my] >> 2) & 1u))) ? (T)1 : (T)0;
    } else if (ch == 4) {
        v = (mx == lay.exit_x && my == lay.exit_y) ? (T)1 : (T)0;
    } else if (ch == 5) {
        v = (i == 5 && j == 5) ? (T)1 : (T)0;
    }
    out[gid] = v;
}

}  // namespace evx

// ===================================================================== C-ABI
namespace {
thread_local char g_err[512] = "";
int fail(int code, const char* msg) {
    snprintf(g_err, sizeof(g_err), "%s", msg);
    return code;
}
int hip_fail(hipError_t e, const char* what) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return -5;
}
int check_layout(const evx_layout* l) {
    if (!l) return fail(-22, "layout is NULL");
    if (l->L < 3 || l->W < 3 || l->L > 4000 || l->W > 4000) return fail(-22, "grid size out of range");
    if (l->P < 1 || l->P > 16383) return fail(-22, "P must be in [1, 16383]");
    if (l->R < 1 || l->R > 1024) return fail(-22, "R must be in [1, 1024]");
    if (!l->floor || !l->cellinfo || !l->valid_bits || !l->danger_p || !l->danger_o) return fail(-22, "missing table");
    return 0;
}
template <int K>
int launch_step(const evx_layout* l, const evx_state* s, const int32_t* a, const evx_step_out* o, hipStream_t st,
                size_t lds) {
    auto kern = evx::env_step_kernel<K>;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(kern, dim3(s->E), dim3(evx::NT), lds, st, *l, *s, a, *o);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "env_step launch");
}
}  // namespace

extern "C" {

const char* evx_last_error(void) { return g_err; }

int64_t evx_step_lds_bytes(const evx_layout* l) {
    if (check_layout(l)) return -1;
    const int G = (l->L + 2) * (l->W + 2);
    return (int64_t)evx::step_lds(G, l->P, l->R).total * 4;
}

int evx_env_step(const evx_layout* l, const evx_state* s, const int32_t* actions, const evx_step_out* o, void* stream) {
    int rc = check_layout(l);
    if (rc) return rc;
    if (!s || !o || !actions || !o->reward || !o->done || !o->obs) return fail(-22, "NULL argument");
    if (s->E <= 0) return 0;
    const int G = (l->L + 2) * (l->W + 2);
    const size_t lds = (size_t)evx::step_lds(G, l->P, l->R).total * 4;
    if (lds > 160 * 1024) return fail(-7, "layout needs more than 160 KiB of LDS");
    const int K = (l->P + evx::NT - 1) / evx::NT;
    hipStream_t st = (hipStream_t)stream;
    if (K <= 1) return launch_step<1>(l, s, actions, o, st, lds);
    if (K <= 2) return launch_step<2>(l, s, actions, o, st, lds);
    if (K <= 4) return launch_step<4>(l, s, actions, o, st, lds);
    if (K <= 9) return launch_step<9>(l, s, actions, o, st, lds);
    if (K <= 16) return launch_step<16>(l, s, actions, o, st, lds);
    if (K <= 36) return launch_step<36>(l, s, actions, o, st, lds);
    return fail(-22, "P too large");
}

int evx_env_reset(const evx_layout* l, const evx_state* s, const uint8_t* mask, evx_obs* obs, int32_t* err,
                  void* stream) {
    int rc = check_layout(l);
    if (rc) return rc;
    if (!s) return fail(-22, "NULL state");
    if (l->L < 4 || l->W < 4) return fail(-22, "reset needs L, W >= 4 (randint(1, L-2))");
    if (s->E <= 0) return 0;
    const int G = (l->L + 2) * (l->W + 2);
    const size_t lds = (size_t)evx::reset_lds(G, l->P).total * 4;
    if (lds > 160 * 1024) return fail(-7, "layout needs more than 160 KiB of LDS");
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)evx::env_reset_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(evx::env_reset_kernel, dim3(s->E), dim3(evx::NT), lds, (hipStream_t)stream, *l, *s, mask, obs,
                       err);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "env_reset launch");
}

int evx_obs_expand_f32(const evx_layout* l, const evx_obs* obs, int64_t n, float* out, void* stream) {
    int rc = check_layout(l);
    if (rc) return rc;
    if (!l->danger_o32) return fail(-22, "danger_o32 missing");
    if (n <= 0) return 0;
    const int64_t total = n * 726;
    hipLaunchKernelGGL(evx::obs_expand_kernel<float>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, *l, obs, n, out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "obs_expand launch");
}

int evx_obs_expand_f64(const evx_layout* l, const evx_obs* obs, int64_t n, double* out, void* stream) {
    int rc = check_layout(l);
    if (rc) return rc;
    if (n <= 0) return 0;
    const int64_t total = n * 726;
    hipLaunchKernelGGL(evx::obs_expand_kernel<double>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, *l, obs, n, out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "obs_expand launch");
}

// random.seed(int) -> init_by_array([seed]); numpy RandomState(int) -> init_genrand
static void init_genrand(uint32_t* mt, uint32_t s) {
    mt[0] = s;
    for (int i = 1; i < 624; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    mt[624] = 624;
}

int evx_seed_host(const uint32_t* seeds, int32_t n, uint32_t* py, uint32_t* np_) {
    if (!seeds || (!py && !np_) || n < 0) return fail(-22, "bad seed arguments");
    for (int s = 0; s < n; s++) {
        if (py) {
            uint32_t* mt = py + (size_t)s * 625;
            init_genrand(mt, 19650218u);
            int i = 1, j = 0;
            for (int k = 624; k; k--) {
                mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + seeds[s] + (uint32_t)j;
                i++;
                j = 0;
                if (i >= 624) {
                    mt[0] = mt[623];
                    i = 1;
                }
            }
            for (int k = 623; k; k--) {
                mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
                i++;
                if (i >= 624) {
                    mt[0] = mt[623];
                    i = 1;
                }
            }
            mt[0] = 0x80000000u;
            mt[624] = 624;
        }
        if (np_) init_genrand(np_ + (size_t)s * 625, seeds[s]);
    }
    return 0;
}

}  // extern "C"
