// MI355X (gfx950) evacuation cellular automaton: env reset / step / observation.
//
// One 512-thread workgroup (8 waves) owns one env instance for a whole step.
// Persons are processed in rows of 512 (person p = row*512 + tid, so global
// accesses are coalesced) by runtime loops (a small instruction footprint: the
// kernel is latency-bound and must not thrash the instruction cache).
// Per-person packed cell+flags, planned direction and first-planner index live
// in LDS; health/acc stream from HBM once per step. The occupancy grid is an
// LDS bitmap, the move-conflict table an LDS array of 16-bit entries, and the
// two MT19937 streams LDS rings (evx_device.h).
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

constexpr int RING = 2048;          // MT ring (words), >= 1078
constexpr int RMASK = RING - 1;
constexpr int WIN = RING - MT_GEN - 16;  // words per consumption window
constexpr int GRP_CAP = 256;
constexpr int PW_CAP = 256;         // pairwise-sum leaves
constexpr uint32_t NIL16 = 0xffffu;
constexpr int SHUF_CHUNK = 1024;
constexpr uint32_t NODIR = 0xffu;

struct Geo {
    int L, W, GY, G, RW, P, R;
};

__device__ __forceinline__ int move_dx(int d) { return (int)((0x8246u >> (2 * d)) & 3u) - 1; }  // MoveTO x
__device__ __forceinline__ int move_dy(int d) { return (int)((0xA091u >> (2 * d)) & 3u) - 1; }  // MoveTO y
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

// Compact observation of one robot built by one wave (bits by ballot).
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
__device__ __forceinline__ void mt_store(uint32_t* ring, int& front, int head, uint32_t* gst) {
    if (head <= MT_N) {
        if (threadIdx.x == 0) gst[MT_N] = (uint32_t)head;  // no twist: words unchanged
        return;
    }
    const int b = MT_N * ((head - 1) / MT_N);
    mt_ensure(ring, RMASK, front, b + MT_N);
    for (int i = threadIdx.x; i < MT_N; i += NT) gst[i] = ring[(b + i) & RMASK];
    if (threadIdx.x == 0) gst[MT_N] = (uint32_t)(head - b);
}

__device__ __forceinline__ void mt_load(uint32_t* ring, const uint32_t* gst, int& head) {
    for (int i = threadIdx.x; i < MT_N; i += NT) ring[i] = gst[i];
    head = (int)gst[MT_N];
}

struct StepLds {  // word offsets into dynamic LDS
    int region, pyring, npring, claim, distbuf, hbuf, pwsum;
    int pk, dir, pf, lhead, lnext, confl, rmapb, validb, grp, robots, wsum, dsum, ctrl, total;
};

__host__ __device__ inline StepLds step_lds(int G, int P, int R) {
    StepLds s;
    const int RW = (G + 31) / 32;
    const int CW = (G + 1) / 2;
    // region: rows -> [py ring][np ring]; claims..execute -> [py ring][claim];
    //         reward -> [distbuf P doubles][hbuf P doubles][leaf sums]
    int a = RING + (CW > RING ? CW : RING);
    const int P4 = (2 * P + 3) & ~3;  // 16-B aligned double arrays
    const int b = 2 * P4 + 2 * PW_CAP;
    if (a < b) a = b;
    a = (a + 3) & ~3;
    int o = 0;
    s.region = o;
    s.pyring = o;
    s.npring = o + RING;
    s.claim = o + RING;
    s.distbuf = o;
    s.hbuf = o + P4;
    s.pwsum = o + 2 * P4;
    o += a;
    s.pk = o; o += P;
    s.dir = o; o += (P + 3) / 4;
    s.pf = o; o += (P + 1) / 2;
    s.lhead = o; o += (P + 1) / 2;
    s.lnext = o; o += (P + 1) / 2;
    s.confl = o; o += (P + 31) / 32;
    s.rmapb = o; o += RW;
    s.validb = o; o += RW;
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

// Diagnostic phase stamps (evx_step_out.stamps; off when NULL).
#define EVX_STAMP(i)                                                                                   \
    do {                                                                                               \
        if (out.stamps && threadIdx.x == 0)                                                            \
            out.stamps[(size_t)blockIdx.x * 16 + (i)] = (int64_t)__builtin_amdgcn_s_memtime();         \
    } while (0)
#define EVX_COUNT(i, v)                                                                                \
    do {                                                                                               \
        if (out.stamps && threadIdx.x == 0) out.stamps[(size_t)blockIdx.x * 16 + (i)] = (v);           \
    } while (0)

__global__ __launch_bounds__(NT, 4) void env_step_kernel(evx_layout lay, evx_state st,
                                                         const int32_t* __restrict__ actions, evx_step_out out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int e = blockIdx.x;
    const int tid = threadIdx.x;
    EVX_STAMP(0);
    Geo g;
    g.L = lay.L; g.W = lay.W; g.GY = lay.W + 2; g.G = (lay.L + 2) * (lay.W + 2);
    g.RW = (g.G + 31) / 32; g.P = lay.P; g.R = lay.R;
    const int P = g.P, R = g.R;
    const int NROW = (P + NT - 1) / NT;
    const StepLds S = step_lds(g.G, P, R);
    uint32_t* pyring = smem + S.pyring;
    uint32_t* npring = smem + S.npring;
    uint32_t* claim = smem + S.claim;
    uint32_t* pkL = smem + S.pk;
    uint8_t* dirL = reinterpret_cast<uint8_t*>(smem + S.dir);
    uint16_t* pfL = reinterpret_cast<uint16_t*>(smem + S.pf);
    uint32_t* lhead = smem + S.lhead;  // 16-bit entries
    uint16_t* lnext = reinterpret_cast<uint16_t*>(smem + S.lnext);
    uint32_t* confl = smem + S.confl;
    uint32_t* rmapb = smem + S.rmapb;
    uint32_t* validb = smem + S.validb;
    int* grp = reinterpret_cast<int*>(smem + S.grp);
    uint32_t* robots = smem + S.robots;
    int* wsum = reinterpret_cast<int*>(smem + S.wsum);
    double* dsum = reinterpret_cast<double*>(smem + S.dsum);
    int* ctrl = reinterpret_cast<int*>(smem + S.ctrl);
    double* distbuf = reinterpret_cast<double*>(smem + S.distbuf);
    double* hbuf = reinterpret_cast<double*>(smem + S.hbuf);
    double* pwsum = reinterpret_cast<double*>(smem + S.pwsum);

    uint32_t* pk_g = st.pk + (size_t)e * P;
    double* h_g = st.health + (size_t)e * P;
    double* a_g = st.acc + (size_t)e * P;

    // ---------------------------------------------------------------- load
    for (int i = tid; i < g.RW; i += NT) {
        rmapb[i] = st.rmap[(size_t)e * g.RW + i];
        validb[i] = lay.valid_bits[i];
    }
    for (int p = tid; p < P; p += NT) pkL[p] = pk_g[p];
    for (int i = tid; i < (P + 1) / 2; i += NT) lhead[i] = 0xffffffffu;
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
            const int c = nx * g.GY + ny;
            if (lay.rx_lo <= nx && nx <= lay.rx_hi && 0 <= ny && ny <= g.W && nx >= 1 && nx <= g.L && ny >= 1 &&
                ny <= g.W && ((lay.valid_bits[c >> 5] >> (c & 31)) & 1u))
                rp = rp_pack(nx, ny);
        }
        robots[tid] = rp;
        st.robots[(size_t)e * R + tid] = rp;
        if (tid == 0) ctrl[0] = (a >= 0 && a <= 4) ? 1 : 0;
    }
    __syncthreads();
    if (ctrl[0]) view = robots[0];  // robot_position refreshed only after a valid action
    EVX_STAMP(1);

    // --------------------- People.run phases 1+2 (health, accumulate, plan)
    const double* dpt = lay.danger_p + (size_t)fs * g.G;
    for (int row = 0; row < NROW; row++) {
        const int p = row * NT + tid;
        const bool inr = p < P;
        uint32_t v = inr ? pkL[p] : (3u << 24);
        const bool act = !((v >> 24) & 3u);
        double hh = 0.0, ac = 0.0, dg = 0.0;
        const int x = pk_x(v), y = pk_y(v);
        if (act) {
            hh = h_g[p];
            ac = a_g[p];
            dg = dpt[x * g.GY + y];
        }
        // phase 1: Person.update_state -> update_health (numpy stream)
        const bool need = act && dg > 0;
        int tot;
        const int off = block_exscan(need ? 2 : 0, wsum, tot);
        bool alive = act;
        for (int lo = 0; lo < tot; lo += WIN) {  // windowed: rows may need more words than the ring
            mt_ensure(npring, RMASK, np_front, np_head + min(tot, lo + WIN));
            if (need && off >= lo && off < lo + WIN) {
                const double u = mt_double(npring, RMASK, np_head + off);
                if (update_health(hh, dg, u)) {
                    v |= (2u << 24);
                    alive = false;
                }
            }
        }
        np_head += tot;
        // phase 2: accumulate; plan with find_best_direction (Python stream)
        bool planner = false;
        if (alive) {
            ac += person_speed(hh) * 0.5;
            if (ac >= 1.0) {
                ac -= 1.0;
                planner = true;
            }
        }
        int cand = 0, ncand = 0;
        if (planner) {
            for (int d = 0; d < 8; d++) {
                const int nx = x + move_dx(d), ny = y + move_dy(d);
                if (check_valid(g, validb, nx, ny) && !bit_get(rmapb, nx * g.GY + ny)) {
                    cand |= 1 << d;
                    ncand++;
                }
            }
        }
        int tot2;
        const int off2 = block_exscan(2 * ncand, wsum, tot2);
        uint32_t best = NODIR;
        for (int lo = 0; lo < tot2; lo += WIN) {
            mt_ensure(pyring, RMASK, py_front, py_head + min(tot2, lo + WIN) + 16);
            if (ncand && off2 >= lo && off2 < lo + WIN) {
                const double fxy = lay.floor[x * g.GY + y];
                double maxs = -INFINITY;
                int idx = py_head + off2;
                for (int d = 0; d < 8; d++) {
                    if (!((cand >> d) & 1)) continue;
                    const int nx = x + move_dx(d), ny = y + move_dy(d);
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
                    const double u = -0.1 + (0.1 - -0.1) * mt_double(pyring, RMASK, idx);
                    idx += 2;
                    const double score = delta_p * 5.0 + effect + u;
                    if (score > maxs) {
                        maxs = score;
                        best = (uint32_t)d;
                    }
                }
            }
        }
        py_head += tot2;
        if (inr) {
            dirL[p] = (uint8_t)best;
            if (act) {
                pkL[p] = v;
                h_g[p] = hh;
                a_g[p] = ac;
            }
        }
    }
    // the numpy stream is finished for this step: its ring becomes the claim table
    mt_store(npring, np_front, np_head, st.np_mt + (size_t)e * EVX_MT_WORDS);
    EVX_COUNT(13, np_head);
    __syncthreads();
    EVX_STAMP(2);

    // ------------------------------------ targets: first planner per cell
    const int CW = (g.G + 1) / 2;
    for (int i = tid; i < CW; i += NT) claim[i] = 0xffffffffu;
    __syncthreads();
    for (int p = tid; p < P; p += NT) {
        const uint32_t d = dirL[p];
        if (d != NODIR) {
            const uint32_t v = pkL[p];
            lds_min16(claim, (pk_x(v) + move_dx(d)) * g.GY + pk_y(v) + move_dy(d), (uint32_t)p);
        }
    }
    __syncthreads();
    for (int p = tid; p < P; p += NT) {
        const uint32_t d = dirL[p];
        if (d != NODIR) {
            const uint32_t v = pkL[p];
            const int t = (pk_x(v) + move_dx(d)) * g.GY + pk_y(v) + move_dy(d);
            const uint32_t pf = lds_read16(claim, t);
            pfL[p] = (uint16_t)pf;
            if (pf != (uint32_t)p) {
                atomicOr(&confl[pf >> 5], 1u << (pf & 31));
                lnext[p] = (uint16_t)lds_exch16(lhead, (int)pf, (uint32_t)p);
            }
        }
    }
    __syncthreads();
    for (int p = tid; p < P; p += NT) {
        const uint32_t d = dirL[p];
        if (d != NODIR && pfL[p] == (uint32_t)p) {
            const uint32_t v = pkL[p];
            lds_set16_ffff(claim, (pk_x(v) + move_dx(d)) * g.GY + pk_y(v) + move_dy(d));
        }
    }
    EVX_STAMP(3);

    // ------------------------- random.shuffle of contested targets (lane 0)
    if (tid == 0) {
        ctrl[0] = 0;              // word index into confl
        ctrl[1] = (int)confl[0];  // remaining bits of that word
        ctrl[2] = py_head;
        ctrl[3] = 0;              // done
        ctrl[4] = 0;              // error
        ctrl[5] = 0;              // groups
    }
    __syncthreads();
    {
        const int NCW = (P + 31) / 32;
        int last_head = -1;
        while (true) {
            const int h0 = ctrl[2];
            mt_ensure(pyring, RMASK, py_front, h0 + SHUF_CHUNK);
            __syncthreads();
            if (tid == 0) {
                int wi = ctrl[0];
                uint32_t m = (uint32_t)ctrl[1];
                int head = ctrl[2];
                int done = 0, ngrp = ctrl[5];
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
                    for (uint32_t q = lds_read16(lhead, pf); q != NIL16; q = lnext[q]) {
                        if (n >= GRP_CAP) {
                            ctrl[4] = 1;
                            break;
                        }
                        grp[n++] = (int)q;
                    }
                    for (int a = 2; a < n; a++) {  // movers in person order
                        const int vv = grp[a];
                        int b = a - 1;
                        while (b >= 1 && grp[b] > vv) {
                            grp[b + 1] = grp[b];
                            b--;
                        }
                        grp[b + 1] = vv;
                    }
                    const int hsave = head;
                    bool ok = true;
                    for (int i = n - 1; i >= 1 && ok; i--) {  // Lib/random.py shuffle
                        const uint32_t bound = (uint32_t)(i + 1);
                        const int kb = bit_length(bound);
                        uint32_t r = 0;
                        while (true) {
                            if (head >= avail) {
                                ok = false;
                                break;
                            }
                            r = mt_word(pyring, RMASK, head++) >> (32 - kb);
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
                    // winner replaces the list head (read only for contested targets below)
                    lhead[pf >> 1] = (lhead[pf >> 1] & ~(0xffffu << ((pf & 1) * 16))) |
                                     ((uint32_t)grp[0] << ((pf & 1) * 16));
                    ngrp++;
                    m &= m - 1;
                }
                ctrl[0] = wi;
                ctrl[1] = (int)m;
                ctrl[2] = head;
                ctrl[3] = done;
                ctrl[5] = ngrp;
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
        EVX_COUNT(14, ctrl[5]);
    }
    mt_store(pyring, py_front, py_head, st.py_mt + (size_t)e * EVX_MT_WORDS);
    EVX_COUNT(12, py_head);
    __syncthreads();
    EVX_STAMP(4);

    // --------------------------------------------- execute_move, in order
    // event code: min over 0xffff - (first_planner<<2 | sub<<1 | value)
    for (int p = tid; p < P; p += NT) {
        const uint32_t d = dirL[p];
        if (d == NODIR) continue;
        const uint32_t v = pkL[p];
        const int pf = pfL[p];
        const bool contested = (confl[pf >> 5] >> (pf & 31)) & 1u;
        const int w = contested ? (int)lds_read16(lhead, pf) : pf;
        const int cold = pk_x(v) * g.GY + pk_y(v);
        if (w == p) {
            const int t = cold + move_dx(d) * g.GY + move_dy(d);
            const bool ex = (lay.cellinfo[t] >> 1) & 1u;
            lds_min16(claim, cold, 0xffffu - ((uint32_t)pf << 2));
            lds_min16(claim, t, 0xffffu - (((uint32_t)pf << 2) | 2u | (ex ? 0u : 1u)));
            if (st.thmap) atomicAdd(&st.thmap[(size_t)e * g.G + t], 1);
        } else {
            dirL[p] = (uint8_t)(0x80u | d);  // lost the conflict: stays
            if (st.thmap) atomicAdd(&st.thmap[(size_t)e * g.G + cold], 1);
        }
    }
    __syncthreads();
    for (int p = tid; p < P; p += NT) {
        const uint32_t d = dirL[p];
        if (d & 0x80u) continue;  // no plan, or lost
        const uint32_t v = pkL[p];
        const int pf = pfL[p];
        const int cold = pk_x(v) * g.GY + pk_y(v);
        const int t = cold + move_dx(d) * g.GY + move_dy(d);
        const bool ex = (lay.cellinfo[t] >> 1) & 1u;
        const uint32_t code_new = 0xffffu - (((uint32_t)pf << 2) | 2u | (ex ? 0u : 1u));
        if (lds_read16(claim, cold) == 0xffffu - ((uint32_t)pf << 2))
            atomicAnd(&rmapb[cold >> 5], ~(1u << (cold & 31)));
        if (lds_read16(claim, t) == code_new) {
            if (ex) atomicAnd(&rmapb[t >> 5], ~(1u << (t & 31)));
            else atomicOr(&rmapb[t >> 5], 1u << (t & 31));
        }
        pkL[p] = (uint32_t)(pk_x(v) + move_dx(d)) | ((uint32_t)(pk_y(v) + move_dy(d)) << 12) |
                 (ex ? (1u << 24) : 0u);
    }
    __syncthreads();
    for (int i = tid; i < g.RW; i += NT) st.rmap[(size_t)e * g.RW + i] = rmapb[i];
    EVX_STAMP(5);

    // ---------------------------------- fire update (both fire models)
    const int fs1 = fs < lay.t_max ? fs + 1 : fs;

    // ------------------------------------ _calculate_reward + counters
    const int vx = rp_x(view), vy = rp_y(view);
    int evac_t = 0, dead_t = 0;
    double gq_t = 0.0;
    int nrem = 0;
    for (int row = 0; row < NROW; row++) {
        const int p = row * NT + tid;
        const bool inr = p < P;
        const uint32_t v = inr ? pkL[p] : (3u << 24);
        const bool sf = inr && pk_safe(v), dd = inr && pk_dead(v);
        evac_t += sf;
        dead_t += dd;
        const double hv = (inr && !dd) ? h_g[p] : 0.0;
        const bool rem = inr && !sf && !dd;
        const long long x2 = 2 * pk_x(v) + 1, y2 = 2 * pk_y(v) + 1;
        const long long dxr = x2 - 2LL * vx, dyr = y2 - 2LL * vy;
        const long long n4 = dxr * dxr + dyr * dyr;  // (2*distance)^2, exact
        if (rem && n4 <= 100) {
            const long long ex2 = x2 - 2LL * lay.exit_x, ey2 = y2 - 2LL * lay.exit_y;
            const long long ne = ex2 * ex2 + ey2 * ey2;
            if (ne > 1600) gq_t += 2.0;
            else if (ne > 400) gq_t += 1.5;
            else gq_t += 1.0;
            if (hv < 80) gq_t += 1.0;
        }
        int tot;
        const int off = block_exscan(rem ? 1 : 0, wsum, tot);
        if (rem) distbuf[nrem + off] = 0.5 * sqrt((double)n4);
        nrem += tot;
        if (inr) hbuf[p] = hv;  // dead -> +0.0, which leaves the sequential sum unchanged
    }
    const int evac = block_sum(evac_t, wsum);
    const int dead = block_sum(dead_t, wsum);
    const double gq = block_sum_d(gq_t, dsum);  // multiples of 0.5: exact in any order
    EVX_STAMP(6);
    // Order-sensitive f64 sums. Python sum over not-dead healths (sequential,
    // wave 0 lane 0) runs beside numpy's pairwise mean (leaves on wave 1).
    if (tid == 0) {
        double total = 0.0;
        const double2* h2 = reinterpret_cast<const double2*>(hbuf);
        int p = 0;
        for (; p + 8 <= P; p += 8) {
            const double2 a = h2[p / 2], b = h2[p / 2 + 1], c = h2[p / 2 + 2], d = h2[p / 2 + 3];
            total += a.x; total += a.y; total += b.x; total += b.y;
            total += c.x; total += c.y; total += d.x; total += d.y;
        }
        for (; p < P; p++) total += hbuf[p];
        dsum[2 * NWAVE] = total;
    } else if (tid >= 64 && tid < 128 && nrem > 0) {
        int lo[4], ll[4];
        const int lane = tid - 64;
        int nleaf = 0;
        {
            int so[32], sl[32];
            int sp = 1;
            so[0] = 0; sl[0] = nrem;
            while (sp > 0) {
                sp--;
                const int o = so[sp], l = sl[sp];
                if (l <= 128) {
                    if ((nleaf & 63) == lane && (nleaf >> 6) < 4) {
                        lo[nleaf >> 6] = o;
                        ll[nleaf >> 6] = l;
                    }
                    nleaf++;
                } else {
                    int n2 = l / 2;
                    n2 -= n2 % 8;
                    so[sp] = o + n2; sl[sp] = l - n2; sp++;
                    so[sp] = o; sl[sp] = n2; sp++;
                }
            }
        }
        for (int j = 0; j < 4; j++) {
            const int li = j * 64 + lane;
            if (li < nleaf && li < PW_CAP) pwsum[li] = np_pairwise_leaf(distbuf + lo[j], ll[j]);
        }
        if (lane == 0) ctrl[6] = nleaf;
    }
    __syncthreads();
    if (tid == 64) {
        if (nrem > 0 && ctrl[6] <= PW_CAP) dsum[2 * NWAVE + 1] = np_pairwise_combine(nrem, pwsum) / (double)nrem;
        else if (nrem > 0) dsum[2 * NWAVE + 1] = 0.0, (out.err ? atomicOr(out.err, 8) : 0);
    }
    __syncthreads();
    EVX_STAMP(7);
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
    for (int p = tid; p < P; p += NT) pk_g[p] = pkL[p];
    EVX_STAMP(8);
}

// ------------------------------------------------------------------ reset
struct ResetLds {
    int pyring, validb, rmapb, pos, ctrl, total;
};
__host__ __device__ inline ResetLds reset_lds(int G, int P) {
    ResetLds s;
    const int RW = (G + 31) / 32;
    int o = 0;
    s.pyring = o; o += RING;
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
        mt_ensure(pyring, RMASK, py_front, h0 + SHUF_CHUNK);
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
                        r = mt_word(pyring, RMASK, head++) >> (32 - kx);
                    } while (r >= nx);
                    if (!ok) break;
                    x = 1 + (int)r;
                    do {
                        if (head >= avail) { ok = false; break; }
                        r = mt_word(pyring, RMASK, head++) >> (32 - ky);
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
    mt_store(pyring, py_front, py_head, st.py_mt + (size_t)e * EVX_MT_WORDS);
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
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)evx::env_step_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(evx::env_step_kernel, dim3(s->E), dim3(evx::NT), lds, (hipStream_t)stream, *l, *s, actions, *o);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "env_step launch");
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
        (void)hipFuncSetAttribute((const void*)evx::env_reset_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
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
            int i = 1;
            for (int k = 624; k; k--) {
                mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + seeds[s];  // j == 0
                i++;
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
