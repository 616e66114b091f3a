// MI355X (gfx950) evacuation cellular automaton: env reset / step / observation.
//
// Step: ONE WAVE (64 lanes, one workgroup) owns one env instance for a whole
// step, so there is no workgroup barrier on the path: scans are ballots and
// mbcnt, broadcasts are readlane/shuffles. Persons stream in rows of 64
// (person p = row*64 + lane, coalesced); the next row's person words, health,
// accumulator, danger, neighbour-validity mask and the 9 floor-field values
// around each person are prefetched one row ahead, so a row's work is ALU + LDS
// only. LDS per env (~22 KB at 130x130): occupancy bitmap, targeted /
// contested / vacated bitmaps, the two MT19937 rings; everything
// person-indexed stays in HBM.
//
// The step is the reference's EvacuationEnv.step (envs/evacuation_env.py:122-172)
// and EvacuationEnvMulti.step (envs/evacuation_env_multi.py:55-89), evaluated
// bit-exactly in parallel:
//   * RNG draws are assigned to persons by prefix sums in person order, so the
//     parallel planners read exactly the words the sequential reference loop
//     consumes (numpy stream: People.update_health envs/people.py:61-88;
//     Python stream: People.find_best_direction envs/people.py:255-297);
//   * a target cell is CONTESTED when a second planner sets its bit in the
//     targeted bitmap. Only contested planners enter the conflict machinery:
//     sorted by (target, person) they form move_plan's groups; each group's
//     first planner is its dict insertion position (envs/people.py:284-297), so
//     the groups sorted by first planner are shuffled (random.shuffle) on lane 0
//     in exactly the reference's order;
//   * execute_move's last-writer-wins on People.rmap (envs/people.py:299-314)
//     only matters on cells that are both vacated and entered by winners; those
//     few events are resolved by max (first planner, sub-step) in an LDS list.
// The reward's order-sensitive sums are evaluated in the reference's order:
// numpy's pairwise mean over streamed leaves, CPython's sequential health sum
// on lane 0. f64 arithmetic is compiled with -ffp-contract=off (no FMA).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <stdlib.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "evacx.h"
#include "evx_device.h"
#include "evx_draws.h"
#include "evx_host.h"

namespace evx {

constexpr uint32_t NODIR = 0xffu;

// step kernel (one wave per env)
constexpr int WR = 1024;             // the reset's MT ring words (>= 624 + 227)
constexpr int WRM = WR - 1;
constexpr int WWIN = MT_N - 16;      // scoring words readable per ensure of the step's 624-slot Python ring
constexpr int SHUF_WORDS = 384;      // words per shuffle chunk (a chunk's words stay in the 624-slot ring)
constexpr int CL_CAP = 510;          // contested movers sorted in LDS (more: global scratch): the list
                                     // (512 with sort padding) in the numpy ring, heads 256 | starts 256
                                     // in the planner queue (both dead after the rows)
constexpr int EV_CAP = 256;          // order-sensitive occupancy events
constexpr int LEAF_CAP = 256;        // numpy pairwise leaves (n <= 16383 needs <= 128)
constexpr int GRP_MAX = 128;         // movers of one contested target (8 neighbour cells; more only
                                     // where placement stacked persons on one cell; beyond: err 1)
constexpr int GBITS = 13;            // group index bits in a sorted group head
constexpr uint32_t DONEPK = 3u << 24;
#ifndef EVX_GQ
#define EVX_GQ 1
#endif
// 64-person groups per pipelined iteration of the rows loop (and the reward's): 1 -- the next
// group's data in flight while one is processed, no per-group selects -- keeps the kernel at 144
// VGPRs with no spill. Round 5 A/B (tools/gpu_r5_envab2.sh, env-only): GQ 2 (166 VGPRs) 0.704 ->
// 0.655 ms at 32768 envs, cfg4 6.03 -> 5.88 ms; GQ 3 / 4 at 2 waves per SIMD 0.86 ms, cfg4 6.21.
// (Round 2: 4 -> 2, 218 -> 168 VGPRs, 1.30 -> 1.21 ms.)
constexpr int GQ = EVX_GQ;

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

// Check_Valid, or (validb == nullptr) only its interior range test.
__device__ __forceinline__ bool in_map(const Geo& g, const uint32_t* validb, int x, int y) {
    if (validb) return check_valid(g, validb, x, y);
    return x >= 1 && x <= g.L && y >= 1 && y <= g.W;
}

// Compact observations of robots r0 .. r0 + 3 (< R) built by one wave in one pass: the 8 LDS
// bit reads per lane issue together, lane k stores robot r0 + k's record.
__device__ __forceinline__ void write_obs4(const Geo& g, const uint32_t* rmapb, const uint32_t* cen, int r0, int R,
                                           int fs, uint32_t lid, evx_obs* dst) {
    const int lane = threadIdx.x & 63;
    const int i0 = lane / 11, j0 = lane - 11 * (lane / 11);
    const int c1 = lane + 64, i1 = c1 / 11, j1 = c1 - 11 * (c1 / 11);
    unsigned long long m[4][2];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int r = r0 + k < R ? r0 + k : r0;
        const int cx = rp_x(cen[r]), cy = rp_y(cen[r]);
        bool b0 = false, b1 = false;
        {
            const int mx = cx + i0 - 5, my = cy + j0 - 5;
            if (in_map(g, nullptr, mx, my)) b0 = bit_get(rmapb, mx * g.GY + my);
        }
        {
            const int mx = cx + i1 - 5, my = cy + j1 - 5;
            if (c1 < 121 && in_map(g, nullptr, mx, my)) b1 = bit_get(rmapb, mx * g.GY + my);
        }
        m[k][0] = __ballot(b0);
        m[k][1] = __ballot(b1);
    }
    if (lane < 4 && r0 + lane < R) {
        const int k = lane;
        const unsigned long long a0 = k == 0 ? m[0][0] : k == 1 ? m[1][0] : k == 2 ? m[2][0] : m[3][0];
        const unsigned long long a1 = k == 0 ? m[0][1] : k == 1 ? m[1][1] : k == 2 ? m[2][1] : m[3][1];
        const uint32_t c = cen[r0 + k];
        uint4 a = make_uint4((uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a1, (uint32_t)(a1 >> 32));
        uint4 b = make_uint4((uint32_t)rp_x(c), (uint32_t)rp_y(c), (uint32_t)fs, lid);
        reinterpret_cast<uint4*>(dst + r0 + k)[0] = a;
        reinterpret_cast<uint4*>(dst + r0 + k)[1] = b;
    }
}

// Compact observations of robots r0 .. r0 + 15 (< R) in one pass: 4 lanes per robot, lane part q
// of robot r builds the window rows i = q, q + 4, q + 8 (< 11) -- two LDS words of the occupancy
// bitmap per row, funnel-shifted to the row's 11 cells (y = cy - 5 .. cy + 5), cells off the map
// interior masked (People.rmap is only set on valid cells, so Check_Valid reduces to the range
// test) -- into bits 11 i .. 11 i + 10 of the 121-bit occupancy word (cell c = 11 i + j, as
// _get_state's [i][j] flattening); the 4 lanes' words meet by xor-shuffles. Robot 0's window is
// centred on `view0` (Map.robot_position), the others on their own positions.
__device__ __forceinline__ void write_obs16(const Geo& g, const uint32_t* rmapb, const uint32_t* cen, uint32_t view0,
                                            int r0, int R, int fs, uint32_t lid, evx_obs* dst) {
    const int lane = threadIdx.x & 63;
    const int r = r0 + (lane >> 2), q = lane & 3;
    const uint32_t c = r < R ? (r == 0 ? view0 : cen[r]) : 0u;
    const int cx = rp_x(c), cy = rp_y(c), ylo = cy - 5;
    // columns j with 1 <= ylo + j <= W
    const int jlo = max(0, 1 - ylo), jhi = min(10, g.W - ylo);
    const uint32_t cmask = jhi >= jlo ? ((2u << jhi) - 1u) & ~((1u << jlo) - 1u) : 0u;
    uint32_t rw[3], w0[3], w1[3];
#pragma unroll
    for (int t = 0; t < 3; t++) {  // the row words, all reads issued together
        const int i = q + 4 * t, mx = cx + i - 5;
        const bool ok = r < R && i < 11 && mx >= 1 && mx <= g.L;
        const int base = ok ? mx * g.GY + ylo : 0;
        rw[t] = (uint32_t)base;
        w0[t] = ok ? rmapb[base >> 5] : 0u;
        w1[t] = ok ? rmapb[(base >> 5) + 1] : 0u;
    }
    uint32_t o0 = 0, o1 = 0, o2 = 0, o3 = 0;
#pragma unroll
    for (int t = 0; t < 3; t++) {
        const int i = q + 4 * t;
        const uint64_t two = ((uint64_t)w1[t] << 32) | w0[t];
        const uint64_t row = (uint64_t)((uint32_t)(two >> (rw[t] & 31u)) & cmask) << (11 * i & 31);
        const int wd = (11 * i) >> 5;  // the row's first word (bits may run into the next)
        const uint32_t lo = (uint32_t)row, hi = (uint32_t)(row >> 32);
        o0 |= wd == 0 ? lo : 0u;
        o1 |= wd == 1 ? lo : (wd == 0 ? hi : 0u);
        o2 |= wd == 2 ? lo : (wd == 1 ? hi : 0u);
        o3 |= wd == 3 ? lo : (wd == 2 ? hi : 0u);
    }
#pragma unroll
    for (int m = 1; m <= 2; m <<= 1) {
        o0 |= (uint32_t)__shfl_xor((int)o0, m, 64);
        o1 |= (uint32_t)__shfl_xor((int)o1, m, 64);
        o2 |= (uint32_t)__shfl_xor((int)o2, m, 64);
        o3 |= (uint32_t)__shfl_xor((int)o3, m, 64);
    }
    if (q == 0 && r < R) {
        reinterpret_cast<uint4*>(dst + r)[0] = make_uint4(o0, o1, o2, o3);
        reinterpret_cast<uint4*>(dst + r)[1] = make_uint4((uint32_t)cx, (uint32_t)cy, (uint32_t)fs, lid);
    }
}

// Compact observation of one robot built by one wave (bits by ballot).
__device__ __forceinline__ void write_obs(const Geo& g, const uint32_t* validb, const uint32_t* rmapb, int cx,
                                          int cy, int fs, uint32_t lid, evx_obs* dst) {
    const int lane = threadIdx.x & 63;
    bool b0 = false, b1 = false;
    {
        const int c = lane, i = c / 11, j = c % 11;
        const int mx = cx + i - 5, my = cy + j - 5;
        if (in_map(g, validb, mx, my)) b0 = bit_get(rmapb, mx * g.GY + my);
    }
    {
        const int c = lane + 64, i = c / 11, j = c % 11;
        const int mx = cx + i - 5, my = cy + j - 5;
        if (c < 121 && in_map(g, validb, mx, my)) b1 = bit_get(rmapb, mx * g.GY + my);
    }
    const unsigned long long m0 = __ballot(b0), m1 = __ballot(b1);
    if (lane == 0) {
        uint4 a = make_uint4((uint32_t)m0, (uint32_t)(m0 >> 32), (uint32_t)m1, (uint32_t)(m1 >> 32));
        uint4 b = make_uint4((uint32_t)cx, (uint32_t)cy, (uint32_t)fs, lid);
        reinterpret_cast<uint4*>(dst)[0] = a;
        reinterpret_cast<uint4*>(dst)[1] = b;
    }
}

// ===================================================== step: one wave per env
// Ordering inside one wave: LDS instructions of a wave execute in issue order,
// so lane-to-lane LDS hand-offs only need the compiler not to reorder them.
__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }
// A wave's own memory traffic complete (every lane sees every lane's LDS and global
// writes); no s_barrier: the waves of a workgroup may run different envs.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ int lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Extend the raw MT sequence in a WR-word ring until front >= upto. A batch of
// up to 227 words depends only on older words (x[n-227], x[n-624], x[n-623]).
__device__ __forceinline__ void mt_ensure_w(uint32_t* ring, int& front, int upto) {
    const int lane = (int)(threadIdx.x & 63);
    while (front < upto) {
        const int cnt = min(MT_LAG, upto - front);
        uint32_t lag[4], a[4], b[4];  // every operand of the round is read before any word is written
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int n = front + lane + 64 * j;
            lag[j] = ring[(n - MT_LAG) & WRM];
            a[j] = ring[(n - 624) & WRM];
            b[j] = ring[(n - 623) & WRM];
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int n = front + lane + 64 * j;
            if (lane + 64 * j < cnt) ring[n & WRM] = mt_twist1(lag[j], a[j], b[j]);
        }
        front += cnt;
        wave_fence();
    }
}

// Store the state after consuming up to raw index `head` (CPython index
// semantics). Needs front <= head + 400 so [b, b+624) is still in the ring.
__device__ __forceinline__ void mt_store_w(uint32_t* ring, int& front, int head, uint32_t* gst) {
    const int lane = (int)(threadIdx.x & 63);
    if (head <= MT_N) {
        if (lane == 0) gst[MT_N] = (uint32_t)head;  // no twist: words unchanged
        return;
    }
    const int b = MT_N * ((head - 1) / MT_N);
    mt_ensure_w(ring, front, b + MT_N);
    for (int i = lane; i < MT_N; i += 64) gst[i] = ring[(b + i) & WRM];
    if (lane == 0) gst[MT_N] = (uint32_t)(head - b);
}

// The numpy stream's ring: exactly the 624-word MT state, word n in slot n % 624 (the stream is
// read in order, at most 128 words ahead of the last word read, so the in-place twist -- every
// operand of a round loaded before any word of it is written -- never overwrites an unread
// word). 400 words less LDS per env than a 1024-word ring.
__device__ __forceinline__ int np_slot(int n) { return n - MT_N * (int)((uint32_t)n / (uint32_t)MT_N); }
// slot s + d of a 624-slot ring for 0 <= s < 624, 0 <= d < 624 (no division)
__device__ __forceinline__ int ring_add(int s, int d) { return s + d >= MT_N ? s + d - MT_N : s + d; }
// One in-place round of the 624-slot ring: words [front, front + cnt) (cnt <= 227), the slot of
// `front` given: word n's operands x[n - 624] (its own slot), x[n - 623] (the next), x[n - 227]
// (397 on) all sit at fixed offsets from n's slot, read before any word of the round is written.
__device__ __forceinline__ void ring_round(uint32_t* ring, int r0, int cnt) {
    const int lane = (int)(threadIdx.x & 63);
    uint32_t lag[4], a[4], b[4];
    int sl[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        sl[j] = ring_add(r0, min(lane + 64 * j, MT_N - 1));
        const int s1 = sl[j] + 1 == MT_N ? 0 : sl[j] + 1;
        lag[j] = ring[ring_add(sl[j], MT_N - MT_LAG)];
        a[j] = ring[sl[j]];
        b[j] = ring[s1];
    }
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (lane + 64 * j < cnt) ring[sl[j]] = mt_twist1(lag[j], a[j], b[j]);
    wave_fence();
}
__device__ __forceinline__ void np_ensure(uint32_t* ring, int& front, int upto) {
    const int lane = (int)(threadIdx.x & 63);
    while (front < upto) {
        const int cnt = min(MT_LAG, upto - front);
        ring_round(ring, np_slot(front), cnt);
        front += cnt;
    }
}
__device__ __forceinline__ double np_double(const uint32_t* ring, int idx) {
    const int s0 = np_slot(idx), s1 = s0 + 1 == MT_N ? 0 : s0 + 1;
    const uint32_t a = mt_temper(ring[s0]) >> 5, b = mt_temper(ring[s1]) >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
}
// mt_store_w for the numpy ring: the stream is consumed exactly up to front, so the block
// [b, b + 624) holding head - 1 completes in place
__device__ __forceinline__ void np_store(uint32_t* ring, int& front, int head, uint32_t* gst) {
    const int lane = (int)(threadIdx.x & 63);
    if (head <= MT_N) {
        if (lane == 0) gst[MT_N] = (uint32_t)head;
        return;
    }
    const int b = MT_N * ((head - 1) / MT_N);
    np_ensure(ring, front, b + MT_N);
    for (int i = lane; i < MT_N; i += 64) gst[i] = ring[i];
    if (lane == 0) gst[MT_N] = (uint32_t)(head - b);
}

// The step's Python stream in the same 624-slot in-place ring (word n in slot n % 624): unlike the
// numpy stream it is read ahead of the words consumed (scoring windows, shuffle windows: at most
// 128 words past the stream's final head), so a block boundary may be crossed before the block
// that holds the final head is stored. Rounds stop at block boundaries, and when the generation
// crosses boundary c (words from c on overwrite block [c - 624, c)) while the stream's final head
// may still lie in that block (head_lb, a lower bound of it, <= c), the block is stored first.
// The final head is never 624 words below the front, so no later crossing overwrites it.
__device__ __forceinline__ void py_ensure(uint32_t* ring, int& front, int upto, uint32_t* gst, int head_lb) {
    const int lane = (int)(threadIdx.x & 63);
    int r = np_slot(front);
    while (front < upto) {
        if (r == 0 && front >= 2 * MT_N && head_lb <= front) {
            for (int i = lane; i < MT_N; i += 64) gst[i] = ring[i];  // block [front - 624, front)
        }
        int cnt = min(MT_LAG, upto - front);
        // stop at the block boundary only where its block may have to be stored there
        if (head_lb <= front - r + MT_N) cnt = min(cnt, MT_N - r);
        ring_round(ring, r, cnt);
        front += cnt;
        r = ring_add(r, cnt);
    }
}
// The state after consuming up to raw index `head`: block b = [b, b + 624) holding head - 1, from
// the ring (front <= b + 624) or as py_ensure stored it when it crossed b + 624.
__device__ __forceinline__ void py_store(uint32_t* ring, int& front, int head, uint32_t* gst) {
    const int lane = (int)(threadIdx.x & 63);
    if (head <= MT_N) {
        if (lane == 0) gst[MT_N] = (uint32_t)head;  // no twist: words unchanged
        return;
    }
    const int b = MT_N * ((head - 1) / MT_N);
    if (front <= b + MT_N) {
        py_ensure(ring, front, b + MT_N, gst, head);
        for (int i = lane; i < MT_N; i += 64) gst[i] = ring[i];
    }
    if (lane == 0) gst[MT_N] = (uint32_t)(head - b);
}


// Ascending bitonic sort of a[0..64*R) by one wave in registers: element i = lane*R + r
// lives in register r of lane `lane`; stages with j < R are compare-exchanges between
// a lane's own registers, the others exchange register r with lane ^ (j / R) by
// shuffle. One load and one store of the array instead of an LDS round trip and a
// wave fence per stage (the LDS network's 45 stages at 512 keys).
template <int R, typename T>
__device__ __forceinline__ void wave_sort_reg(T* a) {
    const int lane = (int)(threadIdx.x & 63);
    constexpr int N = 64 * R;
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; r++) v[r] = a[lane * R + r];
#pragma unroll
    for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j < R) {
#pragma unroll
                for (int r = 0; r < R; r++) {
                    if (r & j) continue;
                    const bool asc = ((lane * R + r) & k) == 0;
                    const uint32_t x = v[r], y = v[r | j];
                    const uint32_t lo = x < y ? x : y, hi = x < y ? y : x;
                    v[r] = asc ? lo : hi;
                    v[r | j] = asc ? hi : lo;
                }
            } else {
                const int m = j / R;
                const bool upper = (lane & m) != 0;
                const bool asc = ((lane * R) & k) == 0;
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const uint32_t o = (uint32_t)__shfl_xor((int)v[r], m, 64);
                    const uint32_t lo = v[r] < o ? v[r] : o, hi = v[r] < o ? o : v[r];
                    v[r] = (upper != asc) ? lo : hi;  // the lower element keeps min when ascending
                }
            }
        }
    }
    wave_sync();
#pragma unroll
    for (int r = 0; r < R; r++) a[lane * R + r] = v[r];
    wave_sync();
}

// The bitonic merge of a 64 R block in registers in one direction: the stages j = 32 R .. 1 of
// a k > 64 R pass (the block is bitonic after that pass's larger-j stages).
template <int R, typename T>
__device__ __forceinline__ void wave_merge_reg(T* a, bool asc) {
    const int lane = (int)(threadIdx.x & 63);
    constexpr int N = 64 * R;
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; r++) v[r] = a[lane * R + r];
#pragma unroll
    for (int j = N >> 1; j > 0; j >>= 1) {
        if (j < R) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                if (r & j) continue;
                const uint32_t x = v[r], y = v[r | j];
                const uint32_t lo = x < y ? x : y, hi = x < y ? y : x;
                v[r] = asc ? lo : hi;
                v[r | j] = asc ? hi : lo;
            }
        } else {
            const int m = j / R;
            const bool upper = (lane & m) != 0;
#pragma unroll
            for (int r = 0; r < R; r++) {
                const uint32_t o = (uint32_t)__shfl_xor((int)v[r], m, 64);
                const uint32_t lo = v[r] < o ? v[r] : o, hi = v[r] < o ? o : v[r];
                v[r] = (upper != asc) ? lo : hi;
            }
        }
    }
    wave_sync();
#pragma unroll
    for (int r = 0; r < R; r++) a[lane * R + r] = v[r];
    wave_sync();
}
// Bitonic sort of a[0..n2) (n2 a power of two >= 1024, e.g. the contested list of a big grid in
// global scratch) with 512-key blocks in registers: every block sorted in its direction, then per
// k >= 1024 only the stages with j >= 512 cross blocks through memory (8 compare-exchanges per
// lane in flight) and the rest run in registers -- 10 memory passes at 4096 keys instead of the
// 78 stages of wave_sort, one wave fence each (cfg4's heaviest envs: ~3 M cycles of sorting).
template <typename T>
__device__ __forceinline__ void wave_sort_big(T* a, int n2) {
    const int lane = (int)(threadIdx.x & 63);
    constexpr int NB = 512;
    for (int b = 0; b < n2 / NB; b++) {
        wave_sort_reg<8>(a + b * NB);
        if (b & 1) {  // descending block: reverse it
            const uint32_t x[4] = {a[b * NB + lane], a[b * NB + 64 + lane], a[b * NB + 128 + lane], a[b * NB + 192 + lane]};
            const uint32_t y[4] = {a[b * NB + NB - 1 - lane], a[b * NB + NB - 65 - lane], a[b * NB + NB - 129 - lane],
                                   a[b * NB + NB - 193 - lane]};
            wave_sync();
#pragma unroll
            for (int q = 0; q < 4; q++) {
                a[b * NB + 64 * q + lane] = y[q];
                a[b * NB + NB - 1 - 64 * q - lane] = x[q];
            }
            wave_sync();
        }
    }
    for (int k = 2 * NB; k <= n2; k <<= 1) {
        for (int j = k >> 1; j >= NB; j >>= 1) {
            for (int q0 = 0; q0 < (n2 >> 1); q0 += 64 * 8) {
                uint32_t xs[8], ys[8];
                int is[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int q = q0 + 64 * u + lane;
                    is[u] = ((q & ~(j - 1)) << 1) | (q & (j - 1));
                    xs[u] = a[is[u]];
                    ys[u] = a[is[u] | j];
                }
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int i = is[u];
                    if ((xs[u] > ys[u]) == ((i & k) == 0)) {
                        a[i] = ys[u];
                        a[i | j] = xs[u];
                    }
                }
            }
            wave_sync();
        }
        for (int b = 0; b < n2 / NB; b++) wave_merge_reg<8>(a + b * NB, ((b * NB) & k) == 0);
    }
}

// Sort a[0..n) ascending (distinct keys): n <= 64 by rank (each lane counts the
// keys below its own, readlane broadcast); power-of-two padded n2 <= 512 (the caller
// pads with 0xffffffff) by a register bitonic network, larger by wave_sort_big.
template <typename T>
__device__ __forceinline__ void wave_sort_keys(T* a, int n, int n2) {
    const int lane = (int)(threadIdx.x & 63);
    if (n <= 64) {
        uint32_t k = 0xffffffffu;
        if (lane < n) k = a[lane];
        int rank = 0;
        for (int j = 0; j < n; j++) rank += (uint32_t)__builtin_amdgcn_readlane((int)k, j) < k;
        wave_sync();
        if (lane < n) a[rank] = k;
        wave_sync();
    } else if (n2 == 128) {
        wave_sort_reg<2>(a);
    } else if (n2 == 256) {
        wave_sort_reg<4>(a);
    } else if (n2 == 512) {
        wave_sort_reg<8>(a);
    } else {
        wave_sort_big(a, n2);
    }
}

__host__ __device__ __forceinline__ int pow2_ceil(int n) {
    int m = 1;
    while (m < n) m <<= 1;
    return m;
}

// Contested targets of move_plan (envs/people.py:284-297): L[0..n) holds
// (target << pb | person) of every planner whose target has >= 2 planners.
// Sort -> groups (one per target, movers in person order); group heads sorted
// by first planner = dict insertion order; Lib/random.py shuffle per group on
// the Python stream (positions found wave-uniformly, shuffles lane-parallel);
// the losers are marked.
__device__ __forceinline__ int doff_of(uint32_t d, int GY) { return move_dx((int)d) * GY + move_dy((int)d); }

template <typename T>
__device__ __forceinline__ void contested_groups(T* Lp, T* heads, T* gstart, int& n, int pb, uint32_t* pyring, int& py_front,
                                 int& py_head, uint32_t* lost, uint32_t* grp, int& err, long long* prof, uint32_t* gst) {
    const int lane = (int)(threadIdx.x & 63);
#ifdef EVX_PROFILE
    long long tq = __builtin_amdgcn_s_memtime();
#define CG_T(i)                                          \
    do {                                                 \
        const long long t2 = __builtin_amdgcn_s_memtime(); \
        prof[i] += t2 - tq;                              \
        tq = t2;                                         \
    } while (0)
#else
#define CG_T(i)
#endif
    const uint32_t pmask = (1u << pb) - 1u;
    const int n2 = pow2_ceil(n);
    for (int i = n + lane; i < n2; i += 64) Lp[i] = 0xffffffffu;
    wave_sync();
    wave_sort_keys(Lp, n, n2);
    // candidates alone on their target (their cell pair held a contested target: the contested
    // bitmap is at half resolution) are dropped, in order: the groups are then the contested
    // targets exactly (>= 2 movers each, so at most n / 2 of them)
    {
        int nn = 0;
        uint32_t prevlast = 0xffffffffu;
        for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + lane;
            const uint32_t key = i < n ? (uint32_t)Lp[i] : 0xffffffffu;
            const uint32_t nxt = i + 1 < n ? (uint32_t)Lp[i + 1] : 0xffffffffu;  // read before this chunk writes
            uint32_t prv = (uint32_t)__shfl_up((int)key, 1, 64);
            if (lane == 0) prv = prevlast;
            const uint32_t tk = key >> pb;
            const bool keep = i < n && ((i > 0 && (prv >> pb) == tk) || (i + 1 < n && (nxt >> pb) == tk));
            prevlast = (uint32_t)__builtin_amdgcn_readlane((int)key, 63);
            const unsigned long long m = __ballot(keep);
            wave_fence();
            if (keep) Lp[nn + lanes_below(m)] = (T)key;
            nn += __popcll(m);
        }
        n = nn;
        wave_sync();
    }
    int ngrp = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        bool st = false;
        uint32_t key = 0;
        if (i < n) {
            key = Lp[i];
            st = (i == 0) || ((Lp[i - 1] >> pb) != (key >> pb));
        }
        const unsigned long long m = __ballot(st);
        if (st) {
            const int gi = ngrp + lanes_below(m);
            gstart[gi] = (uint32_t)i;
            heads[gi] = ((key & pmask) << GBITS) | (uint32_t)gi;
        }
        ngrp += __popcll(m);
    }
    if (lane == 0) gstart[ngrp] = (uint32_t)n;
    const int h2 = pow2_ceil(ngrp);
    for (int i = ngrp + lane; i < h2; i += 64) heads[i] = 0xffffffffu;
    wave_sync();
    wave_sort_keys(heads, ngrp, h2);
    CG_T(1);
    // group descriptors in dict order: (first mover's position in Lp << 8) | size
    for (int k = lane; k < ngrp; k += 64) {
        const int gi = (int)(heads[k] & ((1u << GBITS) - 1u));
        const int s0 = (int)gstart[gi], cnt = (int)gstart[gi + 1] - s0;
        heads[k] = ((uint32_t)s0 << 8) | (uint32_t)min(cnt, 255);
        if (cnt > GRP_MAX) err |= 1;  // > GRP_MAX movers on one target: not representable, flagged
    }
    err = __ballot(err != 0) ? (err | 1) : err;
    wave_sync();
    // Pass 1 (wave-uniform): where each group's random.shuffle starts on the Python
    // stream. _randbelow(b) accepts a word iff its top bit_length(b) bits are < b;
    // per 64-word window the acceptance sets of b = 2..8 are ballots (lane b of
    // mlo/mhi), so consuming one bound is a shift + count-trailing-zeros.
    // Pass 2 (lane per group): every shuffle of the chunk runs in parallel from its
    // recorded start word; only the winner (position 0 afterwards) moves.
    int pos = py_head;
    int B = -(1 << 30);  // window of the end tables: attempts may start at [B, B + 64)
    // end[c-2] (lane j): where the shuffle of a group of c <= 8 movers starting at word
    // B + j ends (relative to B), 255 if it needs words beyond B + 128
    uint32_t endt[7];
#pragma unroll
    for (int c = 0; c < 7; c++) endt[c] = 255u;
    uint32_t need = 0;  // bit c: the current chunk has groups of c <= 8 movers (only their tables are built)
    auto build_window = [&](int b0) {
#ifdef EVX_PROFILE
        prof[4] += 1;
        const long long tb0 = __builtin_amdgcn_s_memtime();
#endif
        B = b0;
        py_ensure(pyring, py_front, B + 128, gst, B);
        const uint32_t t0 = mt_temper(pyring[np_slot(B + lane)]), t1 = mt_temper(pyring[np_slot(B + 64 + lane)]);
        unsigned long long lo[7], hi[7];  // acceptance of bound 2..8 over the 128 words
#pragma unroll
        for (int bb = 2; bb <= 8; bb++) {
            const int kbb = bb < 4 ? 2 : (bb < 8 ? 3 : 4);
            lo[bb - 2] = __ballot((t0 >> (32 - kbb)) < (uint32_t)bb);
            hi[bb - 2] = __ballot((t1 >> (32 - kbb)) < (uint32_t)bb);
        }
        auto next_acc = [&](int bi, int s0) -> int {  // first accepted word >= s0 for bound bi+2, else 128
            if (s0 < 64) {
                const unsigned long long m = lo[bi] >> s0;
                if (m) return s0 + __builtin_ctzll(m);
                return hi[bi] ? 64 + __builtin_ctzll(hi[bi]) : 128;
            }
            if (s0 >= 128) return 128;
            const unsigned long long m = hi[bi] >> (s0 - 64);
            return m ? s0 + __builtin_ctzll(m) : 128;
        };
#pragma unroll
        for (int c = 2; c <= 8; c++) {
            if (!((need >> c) & 1u)) continue;
            int sp = lane;
#pragma unroll
            for (int bb = c; bb >= 2; bb--) sp = sp < 128 ? next_acc(bb - 2, sp) + 1 : 129;
            endt[c - 2] = sp <= 128 ? (uint32_t)sp : 255u;
        }
#ifdef EVX_PROFILE
        prof[6] += __builtin_amdgcn_s_memtime() - tb0;
#endif
    };
#ifdef EVX_PROFILE
    prof[5] = ngrp;
#endif
    int k = 0;
    while (k < ngrp) {
        const int k0 = k, W0 = pos;
        uint32_t desc = 0;
        if (k0 + lane < ngrp) desc = heads[k0 + lane];
        {
            uint32_t nd = 0;
#pragma unroll
            for (int c = 2; c <= 8; c++)
                if (__ballot(k0 + lane < ngrp && (desc & 255u) == (uint32_t)c)) nd |= 1u << c;
            if (nd & ~need) B = -(1 << 30);  // tables of the new counts are missing: rebuild at first use
            need |= nd;
        }
        int wv = 0;
        int nk = 0;
        while (nk < 64 && k < ngrp && pos - W0 < SHUF_WORDS) {
            const uint32_t dsc = (uint32_t)__builtin_amdgcn_readlane((int)desc, nk);
            const int cnt = (int)(dsc & 255u);
            // a group of more than 8 movers (rare) runs alone in its chunk and is shuffled here, by lane
            // 0 as the words are made (its words need not stay in the ring for pass 2)
            if (cnt > 8 && nk > 0) break;
            wv = lane == nk ? pos : wv;
            if (cnt == 1) {
                // a lone mover (its cell pair held a contested target, its own target is not
                // contested): random.shuffle of one element draws nothing, the mover wins
            } else if (cnt <= 8) {
                while (true) {
                    if (pos - B >= 64 || pos < B) build_window(pos);
                    const uint32_t tab = cnt == 2 ? endt[0] : cnt == 3 ? endt[1] : cnt == 4 ? endt[2] : cnt == 5 ? endt[3]
                                       : cnt == 6 ? endt[4] : cnt == 7 ? endt[5] : endt[6];
                    const uint32_t en = (uint32_t)__builtin_amdgcn_readlane((int)tab, pos - B);
                    if (en != 255u) {
                        pos = B + (int)en;
                        break;
                    }
                    build_window(pos);  // the group runs past B + 128 from here: restart the window at it
                    const uint32_t tab2 = cnt == 2 ? endt[0] : cnt == 3 ? endt[1] : cnt == 4 ? endt[2] : cnt == 5 ? endt[3]
                                        : cnt == 6 ? endt[4] : cnt == 7 ? endt[5] : endt[6];
                    const uint32_t en2 = (uint32_t)__builtin_amdgcn_readlane((int)tab2, 0);
                    if (en2 != 255u) {
                        pos = B + (int)en2;
                        break;
                    }
                    err |= 2;  // > 128 words for <= 8 movers: not a sane stream
                    break;
                }
            } else {  // large group: Lib/random.py shuffle word by word (rare)
                const int s0 = (int)(dsc >> 8);
                const bool rep = cnt <= GRP_MAX;  // larger: flagged above, not representable
                if (rep)
                    for (int q = lane; q < cnt; q += 64) grp[q] = Lp[s0 + q] & pmask;
                wave_fence();
                for (int i = cnt - 1; i >= 1; i--) {
                    const uint32_t bound = (uint32_t)(i + 1);
                    const int kb = bit_length(bound);
                    while (true) {
                        if (py_front < pos + 1) py_ensure(pyring, py_front, pos + 64, gst, pos);
                        const uint32_t r = mt_temper(pyring[np_slot(pos)]) >> (32 - kb);
                        pos++;
                        if (r < bound) {
                            if (lane == 0 && rep) {
                                const uint32_t t = grp[i];
                                grp[i] = grp[r];
                                grp[r] = t;
                            }
                            break;
                        }
                    }
                }
                wave_fence();
                if (rep)
                    for (int q = 1 + lane; q < cnt; q += 64) atomicOr(&lost[grp[q] >> 5], 1u << (grp[q] & 31));
                B = -(1 << 30);  // end tables are stale
                nk++;
                k++;
                break;
            }
            nk++;
            k++;
        }
        CG_T(2);
        wave_sync();  // ring words [W0, pos) are in place
        // Pass 2: lane j shuffles group k0 + j (Lib/random.py shuffle, in registers)
        if (lane < nk) {
            const int s0 = (int)(desc >> 8), cnt = (int)(desc & 255u);
            int head = wv;
            if (cnt <= 8) {
                uint32_t a[8];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    a[j] = 0u;
                    if (j < cnt) a[j] = Lp[s0 + j] & pmask;
                }
#pragma unroll
                for (int i = 7; i >= 1; i--) {
                    if (i < cnt) {
                        const uint32_t bound = (uint32_t)(i + 1);
                        const int kb = bit_length(bound);
                        uint32_t r;
                        do {
                            r = mt_temper(pyring[np_slot(head++)]) >> (32 - kb);
                        } while (r >= bound);
                        uint32_t ar = a[0];
#pragma unroll
                        for (int j = 1; j < i; j++) ar = (r == (uint32_t)j) ? a[j] : ar;
                        const uint32_t ai = a[i];
#pragma unroll
                        for (int j = 0; j < i; j++) a[j] = (r == (uint32_t)j) ? ai : a[j];
                        a[i] = (r == (uint32_t)i) ? ai : ar;
                    }
                }
#pragma unroll
                for (int j = 1; j < 8; j++)
                    if (j < cnt) atomicOr(&lost[a[j] >> 5], 1u << (a[j] & 31));
            }
        }
        wave_sync();
        CG_T(3);
    }
    py_head = pos;
#undef CG_T
}

// First planner of contested target t (the group's smallest person index); p when t is not
// contested (a candidate of the half-resolution bitmap alone on its target: its own first planner).
__device__ __forceinline__ int find_pf(const uint32_t* Lp, int n, int t, int pb, int p) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int)(Lp[mid] >> pb) < t) lo = mid + 1;
        else hi = mid;
    }
    if (lo >= n || (int)(Lp[lo] >> pb) != t) return p;
    return (int)(Lp[lo] & ((1u << pb) - 1u));
}

struct WaveLds {  // word offsets into dynamic LDS
    int pyring, npring, aux, rmapb, tbits, cbits, vac, nearc, lost, robots, misc, total;
};

// Big grids (bitmaps of more than WR words: beyond ~181x181 cells, e.g. cfg4's 256x256): the
// target / contested / vacated bitmaps live in the env's global step scratch (L2) instead of LDS,
// which leaves the occupancy map as the only grid-sized LDS table (44 -> 21 KB per env at 256x256:
// 3 -> 7 envs per CU).
#ifndef EVX_BIGG_RW
#define EVX_BIGG_RW WR  // experiment builds: -DEVX_BIGG_RW=0 puts every grid's bitmaps in global scratch
#endif
__host__ __device__ inline bool big_grid(int L, int W) { return ((L + 2) * (W + 2) + 31) / 32 > EVX_BIGG_RW; }

__host__ __device__ inline int cbits_words(int G) { return ((G + 1) / 2 + 31) / 32; }
__host__ __device__ inline WaveLds wave_lds(int L, int W, int P, int R, bool bigg = false) {
    WaveLds s;
    const int G = (L + 2) * (W + 2);
    const int RW = (G + 31) / 32;
    const int NCW = (((L + 2 + 3) >> 2) * ((W + 2 + 3) >> 2) + 31) / 32;
    int o = 0;
    s.pyring = o; o += MT_N;               // after the shuffles: vacated-cell bitmap; reward: leaf sums | leaf buffer
    s.npring = o; o += MT_N;               // the numpy ring (np_ensure); after the rows: contested list
    s.aux = o; o += 512 + 16;              // planner queue + health group; events; leaf table
    s.rmapb = o; o += RW;
    if (bigg) {
        s.tbits = s.cbits = s.vac = -1;  // global scratch (env_scratch_words)
    } else {
        s.tbits = o; o += RW;
        // contested targets at half resolution (cell pairs t >> 1): a set bit marks a pair holding a
        // contested target; the exact test happens when the candidates are grouped by target (a
        // mover alone on its target forms a group of one, which shuffles nothing and wins)
        s.cbits = o; o += cbits_words(G);
        if (RW <= MT_N) {
            s.vac = s.pyring;
        } else {
            s.vac = o; o += RW;
        }
    }
    if (bigg) {
        s.lost = -1;  // global scratch, after the three bitmaps
    } else {
        s.lost = o; o += (P + 31) / 32;
    }
    o = (o + 3) & ~3;
    s.robots = o; o += (R + 3) & ~3;  // 16-B aligned: read 4 robots at a time
    o = (o + 1) & ~1;
    s.misc = o; o += GRP_MAX + 16;         // shuffle group; event counter; pairwise stacks
    // the near-robot block map is read only by the rows (dir_prep), before misc is first written
    // (the contested groups): it overlays misc when it fits (256x256: 16.6 -> 16.1 KB per env, 9 -> 10
    // envs per CU by LDS; 128x128 stays at 12, its VGPR limit)
    if (NCW <= GRP_MAX + 16) {
        s.nearc = s.misc;
    } else {
        s.nearc = o; o += NCW;
    }
    s.total = (o + 3) & ~3;
    return s;
}

// per env: move plan [P] uint2 | not-dead list [P] uint2 | spill: contested list,
// group heads, group starts (each a power of two >= P) | healths [P] double
__host__ __device__ inline int64_t wave_hv_offset(int P) {
    const int n2 = pow2_ceil(P < 64 ? 64 : P);
    return ((int64_t)4 * P + 3 * (int64_t)n2 + 2 + 1) & ~(int64_t)1;
}
// ... | health of every not-dead person after update_health, list order (wide rows)
__host__ __device__ inline int64_t wave_scratch_words(int P) { return wave_hv_offset(P) + 2 * (int64_t)P; }
// ... | big grids: target, contested and vacated bitmaps [3][RW], contest losers [P/32] (the
// per-env stride)
// ... | the light path's lists, kept from one step to the next: header [8] (LISTS_VALID, not-dead
// count, in-play count, -, the health total as a double at [4..5], -) | the not-dead persons'
// healths in list order [P] double (the in-play list itself stays in the wide path's health
// region, which a light step does not otherwise use)
__host__ __device__ inline int64_t persist_offset(const evx_layout& l) {
    const int RW = ((l.L + 2) * (l.W + 2) + 31) / 32;
    const int64_t o = wave_scratch_words(l.P) + (big_grid(l.L, l.W) ? 3 * (int64_t)RW + (l.P + 31) / 32 : 0);
    return (o + 1) & ~(int64_t)1;
}
constexpr int LHDR = 8;  // words of the kept lists' header
__host__ __device__ inline int64_t env_scratch_words(const evx_layout& l) { return persist_offset(l) + LHDR + 2 * (int64_t)l.P; }
constexpr uint32_t LISTS_VALID = 0x4c495354u;

__device__ __forceinline__ int pb_bits(int P) { return P > 1 ? bit_length((uint32_t)(P - 1)) : 1; }

// Diagnostic phase stamps (evx_step_out.stamps; off when NULL): slots 0-8 shader
// clock, 9/10 constant-rate clock at start/end, 11-14 counters.
#define EVX_STAMP(i)                                                                                   \
    do {                                                                                               \
        if (out.stamps && (threadIdx.x & 63) == 0)                                                            \
            out.stamps[(size_t)e * 48 + (i)] = (int64_t)__builtin_amdgcn_s_memtime();         \
    } while (0)
#define EVX_RSTAMP(i)                                                                                  \
    do {                                                                                               \
        if (out.stamps && (threadIdx.x & 63) == 0)                                                            \
            out.stamps[(size_t)e * 48 + (i)] = (int64_t)__builtin_amdgcn_s_memrealtime();     \
    } while (0)
#define EVX_COUNT(i, v)                                                                                \
    do {                                                                                               \
        if (out.stamps && (threadIdx.x & 63) == 0) out.stamps[(size_t)e * 48 + (i)] = (v);           \
    } while (0)

// EVX_PROFILE builds only: cycle accumulators of sub-phases, stored to slots 16..31
#ifdef EVX_PROFILE
#define PT_DECL(n) long long pt_##n = 0, pt0_##n = __builtin_amdgcn_s_memtime()
#define PT_BEGIN(n) pt0_##n = __builtin_amdgcn_s_memtime()
#define PT_END(n) pt_##n += __builtin_amdgcn_s_memtime() - pt0_##n
#define PT_STORE(n, slot) EVX_COUNT(slot, pt_##n)
#else
#define PT_DECL(n)
#define PT_BEGIN(n)
#define PT_END(n)
#define PT_STORE(n, slot)
#endif

// Pin a loaded value: the wait for its load happens here, before any later load
// is issued (vmcnt waits are in-order, so a first use placed after the next
// prefetch would also wait for that prefetch).
__device__ __forceinline__ void pin(uint32_t v) { asm volatile("" ::"v"(v)); }
__device__ __forceinline__ void pin(uint2 v) { asm volatile("" ::"v"(v.x), "v"(v.y)); }
__device__ __forceinline__ void pin(double v) { asm volatile("" ::"v"(v)); }

__device__ __forceinline__ double readlane_d(double v, int k) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), k);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), k);
    return __hiloint2double(hi, lo);
}

// the class byte of an env (evx_state.perm_ws; see env_orders_kernel)
__device__ __forceinline__ uint8_t env_class(const evx_layout& lay, int fs, int evac, int dead) {
    const int P = lay.P, rem = P - evac - dead;
    const int b = 15 - min(15, max(0, rem) * 16 / (P + 1));
    const int hmin = max(1, P / 4);  // heavy_cap's threshold
    return (uint8_t)(b | (fs >= lay.t_max ? 0x10 : 0) | (rem >= hmin ? 0x20 : 0));
}
template <bool BIGG = false>
__device__ __forceinline__ void reset_one(const evx_layout& lay, const evx_state& st, const int e, uint32_t* smem,
                                          evx_obs* obs, int32_t* err);

struct ResetLds {
    int pyring, validb, rmapb, total;
};
// bigg: the validity bitmap is read from the layout's table (L2) instead of an LDS copy, so a
// big grid's fused reset needs no more LDS than its step (cfg4: 20.7 -> 19.3 KB per env)
__host__ __device__ inline ResetLds reset_lds(int G, int P, bool bigg = false) {
    ResetLds s;
    const int RW = (G + 31) / 32;
    int o = 0;
    s.pyring = o; o += WR;
    if (bigg) {
        s.validb = -1;
    } else {
        s.validb = o; o += RW;
    }
    s.rmapb = o; o += RW;
    s.total = (o + 3) & ~3;
    return s;
}

// dynamic LDS words of one env's wave: the step's layout, which also hosts a fused reset
__host__ __device__ inline int step_lds_words(const evx_layout& l, bool bigg = false) {
    const int G = (l.L + 2) * (l.W + 2);
    const int a = wave_lds(l.L, l.W, l.P, l.R, bigg).total, b = reset_lds(G, l.P, bigg).total;
    return ((a > b ? a : b) + 3) & ~3;
}

// People.find_best_direction (envs/people.py:232-262) for one planner per lane, split
// in two: dir_prep gathers the operands (floor deltas, robot distances), dir_score
// consumes the planner's Python-stream words (uniform(-0.1, 0.1) per candidate, in
// direction order) from ring[(idx - base) & mask].
struct DirPrep {
    double f[8];     // (floor[c] - floor[c + MoveTO[d]]) * 5.0
    int md2[8];      // squared distance to the nearest robot (only where nearm)
    uint32_t nearm;  // candidates inside a near-robot block
};
__device__ __forceinline__ void dir_prep(DirPrep& d, bool has, int x, int y, uint32_t cand, int GY,
                                         const double* __restrict__ fd5, const uint32_t* nearc, int BY,
                                         const uint32_t* robots, int R, int rb) {
#pragma unroll
    for (int k = 0; k < 8; k++) d.f[k] = 0.0;
    if (has) {
        const double2* fr = reinterpret_cast<const double2*>(fd5 + (size_t)(x * GY + y) * 8);
#pragma unroll
        for (int q2 = 0; q2 < 4; q2++) {
            const double2 v = fr[q2];
            d.f[2 * q2] = v.x;
            d.f[2 * q2 + 1] = v.y;
        }
    }
    // squared distance to the nearest robot for the 8 neighbours, only when some
    // candidate lies in a near-robot block (robots outer: 4 per LDS read)
    uint32_t nearm = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int nx = x + move_dx(k), ny = y + move_dy(k);
        if (((cand >> k) & 1u) && bit_get(nearc, (nx >> 2) * BY + (ny >> 2))) nearm |= 1u << k;
    }
    d.nearm = nearm;
#pragma unroll
    for (int k = 0; k < 8; k++) d.md2[k] = 0x7fffffff;
    if (__ballot(nearm != 0)) {
        const uint4* r4 = reinterpret_cast<const uint4*>(robots);
        for (int r0 = 0; r0 < R; r0 += 4) {
            const uint4 q4 = r4[r0 >> 2];
            const uint32_t rq[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int rx = rp_x(rq[j]), ry = rp_y(rq[j]);
                // robots no lane is near cannot be the nearest within range: skipped
                if (r0 + j < R && __ballot(abs(x - rx) <= rb && abs(y - ry) <= rb)) {
#pragma unroll
                    for (int k = 0; k < 8; k++) {
                        const int dx = x + move_dx(k) - rx, dy = y + move_dy(k) - ry;
                        d.md2[k] = min(d.md2[k], dx * dx + dy * dy);
                    }
                }
            }
        }
    }
}
__device__ __forceinline__ uint32_t dir_score(const DirPrep& d, uint32_t cand, int idx, const uint32_t* ring, int base,
                                              int mask, double repel_k, int rd2) {
    double maxs = -INFINITY;
    uint32_t best = NODIR;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if ((cand >> k) & 1u) {
            double effect = 0.0;
            if (((d.nearm >> k) & 1u) && d.md2[k] < rd2) effect = repel_k / (sqrt((double)d.md2[k]) + 0.1);
            // mask 0: the step's 624-slot Python ring; else a power-of-two ring or a linear buffer
            const double u = -0.1 + (0.1 - -0.1) * (mask ? mt_double(ring, mask, idx - base) : np_double(ring, idx));
            idx += 2;
            const double score = d.f[k] + effect + u;  // delta_p * 5.0 + robot_effect + uniform
            if (score > maxs) {
                maxs = score;
                best = (uint32_t)k;
            }
        }
    }
    return best;
}

// ============================================ wide rows: one heavy env, WNW waves
// An env-step early in an episode has thousands of persons in play, and one wave
// per env makes the launch wait for the heaviest. For the heaviest envs (listed
// first by evx_env_order) the rows phase (update_health, accumulate, planning,
// find_best_direction) runs on all WNW waves of a workgroup: the not-dead list is
// dealt out in 64-person groups round-robin (group g to wave g % WNW), each
// group's numpy / Python stream offsets follow from per-group counts (the reference
// consumes both streams in person order), the MT19937 words are generated
// cooperatively (227 per round, one block barrier per round) into a linear LDS
// buffer, and the planners are scored in word windows that every wave shares in.
// Wave 0 then carries on alone (contested targets, execute, reward), while wave 1
// folds the health total (CPython's sequential sum) in parallel.
constexpr int WNW = 4;
struct WideCtl {
    int nnd, np_head, py_head, fs;  // in: published by wave 0
    int ndc[WNW];                   // deaths per wave
    int any_cont, nplan, n_died, py_front, py_head_out, pad0;
    double total;  // health total (wave 1)
    int total_ready, pad1;
};
// Workgroup LDS (WNW waves): WNW env regions of step_lds_words, then WideCtl. A heavy
// env keeps wave 0's region; the rows buffers overlay regions 1.. (dead once the
// rows are done, when waves 1.. go on with other envs) and may run past them; WideCtl
// follows whichever ends later.
struct WideLds {
    int ctl, grp, NGmax, lin, LINW, lists, CHmax, end, total;
};
__host__ __device__ inline WideLds wide_lds(const evx_layout& l) {
    WideLds s;
    const int LW = step_lds_words(l);
    s.NGmax = (l.P + 63) / 64;
    s.grp = LW;                 // per group: numpy words | Python words | movers | Python offset
    s.lin = s.grp + ((4 * s.NGmax + 3) & ~3);
    s.LINW = ((2 * l.P + 1280) + 3) & ~3;  // numpy words of the step + MT history + slack
    s.lists = s.lin + s.LINW;
    s.CHmax = ((s.NGmax + WNW - 1) / WNW) * 64;  // planners per wave
    s.end = s.lists + WNW * s.CHmax * 3;
    s.ctl = ((WNW * LW > s.end ? WNW * LW : s.end) + 3) & ~3;
    s.total = s.ctl + 32;
    return s;
}

// Extend the raw MT sequence held linearly (word n at lin[n - base]) to upto; all
// WNW waves, uniform arguments, one block barrier per 227-word round.
__device__ __forceinline__ void coop_gen(uint32_t* lin, int base, int& front, int upto) {
    const int tid = (int)threadIdx.x;
    while (front < upto) {
        const int cnt = min(MT_LAG, upto - front);
        for (int j = tid; j < cnt; j += 64 * WNW) {
            const int n = front + j - base;
            lin[n] = mt_twist1(lin[n - MT_LAG], lin[n - MT_N], lin[n - MT_N + 1]);
        }
        front += cnt;
        __syncthreads();
    }
}

// sum of cnt[0..g) (wave-uniform g)
__device__ __forceinline__ int group_prefix(const int* cnt, int g) {
    int acc = 0;
    for (int i = (int)(threadIdx.x & 63); i < g; i += 64) acc += cnt[i];
    return wave_sum(acc);
}

// People.run phases 1+2 of env e on all WNW waves (wave 0 has published WideCtl and
// its LDS tables: rmap snapshot, near map, robots, zeroed target bitmaps, the two MT
// states at ring positions [0, 624)). Outputs in WideCtl; the plan list and person
// writes in HBM; the numpy state stored; the Python stream handed back to wave 0's
// ring.
__device__ __forceinline__ void rows_wide(const evx_layout& lay, const evx_state& st, const int e, uint32_t* smem,
                                          int64_t* prof = nullptr) {
    const int tid = (int)threadIdx.x, lane = tid & 63, w = tid >> 6;
#ifdef EVX_PROFILE
    long long wt = __builtin_amdgcn_s_memtime(), wacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#define WT(i)                                              \
    do {                                                   \
        const long long t2 = __builtin_amdgcn_s_memtime(); \
        wacc[i] += t2 - wt;                                \
        wt = t2;                                           \
    } while (0)
#else
#define WT(i)
#endif
    const int P = lay.P, R = lay.R, GY = lay.W + 2, G = (lay.L + 2) * (lay.W + 2);
    const WaveLds S = wave_lds(lay.L, lay.W, P, R);
    const WideLds WL = wide_lds(lay);
    WideCtl* ctl = reinterpret_cast<WideCtl*>(smem + WL.ctl);
    int* npg = reinterpret_cast<int*>(smem + WL.grp);  // numpy words per group
    int* pyg = npg + WL.NGmax;                          // Python words per group
    int* mvg = pyg + WL.NGmax;                          // movers per group
    int* pyo = mvg + WL.NGmax;                          // first Python word per group (owner wave only)
    uint32_t* lin = smem + WL.lin;
    // this wave's planners: (person | cand << 16 | best << 24, x | y << 12 | group << 24, first word)
    uint32_t* myl = smem + WL.lists + w * WL.CHmax * 3;
    const uint32_t* rmapb = smem + S.rmapb;
    uint32_t* tbits = smem + S.tbits;
    const uint32_t* nearc = smem + S.nearc;
    const uint32_t* robots = smem + S.robots;
    uint32_t* pyring = smem + S.pyring;
    const uint32_t* npring = smem + S.npring;
    const int nnd = ctl->nnd, np_head0 = ctl->np_head, py_head0 = ctl->py_head, fs = ctl->fs;

    uint32_t* pk_g = st.pk + (size_t)e * P;
    double* h_g = st.health + (size_t)e * P;
    double* a_g = st.acc + (size_t)e * P;
    uint32_t* scr = st.scratch + (size_t)e * env_scratch_words(lay);
    uint32_t* cbits = smem + S.cbits;  // contested cell pairs (LDS)
    uint2* plan = reinterpret_cast<uint2*>(scr);
    const uint2* ndl = reinterpret_cast<const uint2*>(scr + 2 * P);
    double* hv = reinterpret_cast<double*>(scr + wave_hv_offset(P));
    const double* __restrict__ dpt = lay.danger_p + (size_t)fs * G;
    const double* __restrict__ fd5 = lay.floor_d5;
    const uint8_t* __restrict__ nbv = lay.nbr_valid;
    int doff[8];
#pragma unroll
    for (int d = 0; d < 8; d++) doff[d] = move_dx(d) * GY + move_dy(d);
    const int rd2 = lay.repel_d2;
    const int BY = (GY + 3) >> 2;
    int rr = 0;
    while ((rr + 1) * (rr + 1) < rd2) rr++;
    const int rb = rr + 1;

    const int NG = (nnd + 63) >> 6;
    const uint2 NOONE = make_uint2(0u, DONEPK);
    constexpr int GS = 4 * WNW;  // groups per iteration of a pass: w, w + WNW, w + 2 WNW, w + 3 WNW

    // pass 1: numpy draws per group (alive, not safe, danger > 0)
    for (int g0 = w; g0 < NG; g0 += GS) {
        uint2 en[4];
        double dg[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int i = 64 * (g0 + WNW * j) + lane;
            en[j] = NOONE;
            if (i < nnd) en[j] = ndl[i];
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            dg[j] = 0.0;
            if (!((en[j].y >> 24) & 3u)) dg[j] = dpt[pk_x(en[j].y) * GY + pk_y(en[j].y)];
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int c = 2 * __popcll(__ballot(!((en[j].y >> 24) & 3u) && dg[j] > 0));
            if (lane == 0 && g0 + WNW * j < NG) {
                npg[g0 + WNW * j] = c;
                mvg[g0 + WNW * j] = 0;
            }
        }
    }
    WT(0);
    for (int i = tid; i < MT_N; i += 64 * WNW) lin[i] = npring[i];
    __syncthreads();
    WT(1);
    const int Tnp = group_prefix(npg, NG);
    int front = MT_N;
    coop_gen(lin, 0, front, np_head0 + Tnp);
    WT(2);

    // pass 2: health, accumulate, candidates; planners into this wave's list
    int nq = 0, nd = 0;
    for (int g0 = w; g0 < NG; g0 += GS) {
        uint2 en[4];
        double hh[4], ac[4], dg[4];
        uint32_t nv[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int i = 64 * (g0 + WNW * j) + lane;
            en[j] = NOONE;
            if (i < nnd) en[j] = ndl[i];
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int i = 64 * (g0 + WNW * j) + lane;
            hh[j] = 0.0;
            ac[j] = 0.0;
            dg[j] = 0.0;
            nv[j] = 0u;
            if (i < nnd) {
                hh[j] = h_g[en[j].x];
                if (!((en[j].y >> 24) & 3u)) {
                    const int c = pk_x(en[j].y) * GY + pk_y(en[j].y);
                    ac[j] = a_g[en[j].x];
                    dg[j] = dpt[c];
                    nv[j] = nbv[c];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int gi = g0 + WNW * j;
            if (gi >= NG) break;
            const int off = np_head0 + group_prefix(npg, gi);
            const int i = 64 * gi + lane;
            const bool inr = i < nnd;
            const int p = (int)en[j].x;
            const uint32_t v = en[j].y;
            const bool act = inr && !((v >> 24) & 3u);
            const int x = pk_x(v), y = pk_y(v), cold = x * GY + y;
            double h = hh[j], a = ac[j];
            const bool need = act && dg[j] > 0;
            const unsigned long long nm = __ballot(need);
            bool alive = act, died = false;
            if (need) {
                const double u = mt_double(lin, -1, off + 2 * lanes_below(nm));
                if (update_health(h, dg[j], u)) {
                    died = true;
                    alive = false;
                }
            }
            nd += __popcll(__ballot(died));
            if (inr) hv[i] = died ? 0.0 : h;  // +0.0 leaves CPython's running sum unchanged
            bool planner = false;
            if (alive) {
                a += person_speed(h) * 0.5;
                if (a >= 1.0) {
                    a -= 1.0;
                    planner = true;
                }
            }
            uint32_t cand = 0;
            if (planner) {
                uint32_t occ = 0;
#pragma unroll
                for (int d = 0; d < 8; d++) occ |= (uint32_t)bit_get(rmapb, cold + doff[d]) << d;
                cand = nv[j] & ~occ;
            }
            // Python words: exclusive prefix of 2 * |cand| within the group (bit-sliced ballots)
            const int nc = __popc(cand);
            int off2 = 0, tot2 = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const unsigned long long m = __ballot((nc >> b) & 1);
                off2 += lanes_below(m) << (b + 1);
                tot2 += __popcll(m) << (b + 1);
            }
            const unsigned long long qm = __ballot(cand != 0);
            if (cand) {
                const int k = nq + lanes_below(qm);
                myl[3 * k] = (uint32_t)p | (cand << 16) | (NODIR << 24);
                myl[3 * k + 1] = (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)gi << 24);
                myl[3 * k + 2] = (uint32_t)off2;
            }
            nq += __popcll(qm);
            if (lane == 0) pyg[gi] = tot2;
            if (need) h_g[p] = h;
            if (alive) a_g[p] = a;
            if (died) pk_g[p] = v | (2u << 24);
        }
    }
    WT(3);
    if (lane == 0) ctl->ndc[w] = nd;
    // the numpy stream is finished for this step: store its state (mt_store_w)
    {
        const int head = np_head0 + Tnp;
        uint32_t* gst = st.np_mt + (size_t)e * EVX_MT_WORDS;
        if (head <= MT_N) {
            if (tid == 0) gst[MT_N] = (uint32_t)head;
        } else {
            const int b = MT_N * ((head - 1) / MT_N);
            coop_gen(lin, 0, front, b + MT_N);
            for (int i = tid; i < MT_N; i += 64 * WNW) gst[i] = lin[b + i];
            if (tid == 0) gst[MT_N] = (uint32_t)(head - b);
        }
    }
    WT(4);
    __syncthreads();  // pass 2 done everywhere: the buffer takes the Python stream
    for (int i = tid; i < MT_N; i += 64 * WNW) lin[i] = pyring[i];
    const int Tpy = group_prefix(pyg, NG);
    int nd_all = 0;
    for (int v = 0; v < WNW; v++) nd_all += ctl->ndc[v];
    // absolute first words of this wave's planners (its own groups only: no barrier)
    for (int gi = w; gi < NG; gi += WNW) {
        const int o = py_head0 + group_prefix(pyg, gi);
        if (lane == 0) pyo[gi] = o;
    }
    wave_fence();
    for (int k = lane; k < nq; k += 64) myl[3 * k + 2] += (uint32_t)pyo[myl[3 * k + 1] >> 24];
    __syncthreads();
    WT(5);

    // find_best_direction in word windows of the linear buffer
    front = MT_N;
    int base = 0, cursor = 0;
    const int pend = py_head0 + Tpy;
    bool anyc = false;
    while (true) {
        const int whi = min(pend, base + WL.LINW - 16);
        coop_gen(lin, base, front, min(whi + 16, pend));
        WT(6);
        while (cursor < nq) {  // this wave's planners whose first word lies below whi
            const int k = cursor + lane;
            const bool has = k < nq;
            uint32_t e0 = 0, e1 = 0;
            int sidx = 0x7fffffff;
            if (has) {
                e0 = myl[3 * k];
                e1 = myl[3 * k + 1];
                sidx = (int)myl[3 * k + 2];
            }
            const bool in = has && sidx < whi;
            const int nin = __popcll(__ballot(in));
            if (nin == 0) break;
            const uint32_t cand = (e0 >> 16) & 0xffu;
            const int x = pk_x(e1), y = pk_y(e1);
            DirPrep dp;
            dir_prep(dp, in, x, y, in ? cand : 0u, GY, fd5, nearc, BY, robots, R, rb);
            uint32_t best = NODIR;
            if (in) best = dir_score(dp, cand, sidx, lin, base, -1, lay.repel_k, rd2);
            if (in) {
                myl[3 * k] = (e0 & 0x00ffffffu) | (best << 24);
                if (best != NODIR) {
                    const int t = x * GY + y + doff_of(best, GY);
                    const uint32_t bit = 1u << (t & 31);
                    const uint32_t old = atomicOr(&tbits[t >> 5], bit);
                    if (old & bit) {
                        atomicOr(&cbits[(t >> 1) >> 5], 1u << ((t >> 1) & 31));
                        anyc = true;
                    }
                }
            }
            cursor += nin;
            if (nin < 64) break;
        }
        WT(7);
        if (whi >= pend) break;
        __syncthreads();  // every wave is done with this window
        const int nb = max(0, front - 1040);  // keep 1040 words: MT history + wave 0's ring
        if (nb > base) {
            const int cnt = front - nb;
            uint32_t tmp[(1040 + 64 * WNW - 1) / (64 * WNW)];
#pragma unroll
            for (int q = 0; q < (1040 + 64 * WNW - 1) / (64 * WNW); q++) {
                const int j = tid + 64 * WNW * q;
                if (j < cnt) tmp[q] = lin[nb - base + j];
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < (1040 + 64 * WNW - 1) / (64 * WNW); q++) {
                const int j = tid + 64 * WNW * q;
                if (j < cnt) lin[j] = tmp[q];
            }
            base = nb;
            __syncthreads();
        }
    }
    WT(8);
    if (__ballot(anyc) && lane == 0) atomicOr(&ctl->any_cont, 1);
    // the movers of People.move_plan in person order: per-group counts, then offsets
    for (int k0 = 0; k0 < nq; k0 += 64) {
        const int k = k0 + lane;
        if (k < nq && (myl[3 * k] >> 24) != NODIR) atomicAdd(&mvg[myl[3 * k + 1] >> 24], 1);
    }
    __syncthreads();
    const int nplan = group_prefix(mvg, NG);
    {
        int gcur = -1, pos = 0;
        for (int k0 = 0; k0 < nq; k0 += 64) {
            const int k = k0 + lane;
            const bool has = k < nq;
            uint32_t e0 = NODIR << 24, e1 = 0;
            if (has) {
                e0 = myl[3 * k];
                e1 = myl[3 * k + 1];
            }
            const uint32_t best = e0 >> 24;
            const bool mover = has && best != NODIR;
            const int gk = (int)(e1 >> 24);
            int dst = 0;
            unsigned long long left = __ballot(has);
            while (left) {  // the batch's groups in order (this wave's groups only)
                const int gsel = __builtin_amdgcn_readlane(gk, __builtin_ctzll(left));
                const bool ing = has && gk == gsel;
                if (gsel != gcur) {
                    gcur = gsel;
                    pos = group_prefix(mvg, gsel);
                }
                const unsigned long long mm = __ballot(ing && mover);
                if (ing && mover) dst = pos + lanes_below(mm);
                pos += __popcll(mm);
                left &= ~__ballot(ing);
            }
            if (mover) plan[dst] = make_uint2(e0 & 0xffffu, (uint32_t)(pk_x(e1) * GY + pk_y(e1)) | (best << 24));
        }
    }
    // hand the Python stream back to wave 0's 624-slot ring: words [front - 624, front)
    for (int n = max(0, front - MT_N) + tid; n < front; n += 64 * WNW) pyring[np_slot(n)] = lin[n - base];
    if (tid == 0) {
        ctl->nplan = nplan;
        ctl->n_died = nd_all;
        ctl->py_front = front;
        ctl->py_head_out = pend;
    }
    __syncthreads();
    WT(9);
#ifdef EVX_PROFILE
    if (prof && tid == 0)
        for (int i = 0; i < 10; i++) prof[36 + i] = wacc[i];
#endif
#undef WT
}

// Wave 1 after rows_wide: sum(p.health for p in people if not p.dead), in list order.
__device__ __forceinline__ void wide_health_sum(const evx_layout& lay, const evx_state& st, const int e, uint32_t* smem) {
    const int lane = (int)(threadIdx.x & 63);
    const int P = lay.P;
    WideCtl* ctl = reinterpret_cast<WideCtl*>(smem + wide_lds(lay).ctl);
    const int nnd = ctl->nnd;
    const double* hv = reinterpret_cast<const double*>(st.scratch + (size_t)e * env_scratch_words(lay) + wave_hv_offset(P));
    double total = 0.0;
    double cur = lane < nnd ? hv[lane] : 0.0;
    for (int i0 = 0; i0 < nnd; i0 += 64) {
        const double nxt = i0 + 64 + lane < nnd ? hv[i0 + 64 + lane] : 0.0;
        const int n = min(64, nnd - i0);
        for (int j = 0; j < n; j++) total += readlane_d(cur, j);
        cur = nxt;
    }
    if (lane == 0) {
        ctl->total = total;
        __hip_atomic_store(&ctl->total_ready, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// One env-step of env e by the calling wave (smem: its wave_lds region).
// WIDE: wave 0 of a heavy env's workgroup; the rows phase runs on all its waves.
template <bool WIDE, bool BIGG = false>
__device__ __forceinline__ void step_env(const evx_layout& lay, const evx_state& st, const int32_t* __restrict__ actions,
                                         const evx_step_out& out, const int e, uint32_t* smem) {
    const int lane = (int)(threadIdx.x & 63);
    EVX_RSTAMP(9);
    EVX_STAMP(0);
    Geo g;
    g.L = lay.L; g.W = lay.W; g.GY = lay.W + 2; g.G = (lay.L + 2) * (lay.W + 2);
    g.RW = (g.G + 31) / 32; g.P = lay.P; g.R = lay.R;
    const int P = g.P, R = g.R, GY = g.GY;
    const int NR = (P + 63) >> 6;
    const int pb = pb_bits(P);
    const WaveLds S = wave_lds(g.L, g.W, P, R, BIGG);
    uint32_t* pyring = smem + S.pyring;
    uint32_t* npring = smem + S.npring;
    uint32_t* aux = smem + S.aux;
    uint32_t* rmapb = smem + S.rmapb;
    const int64_t SW = env_scratch_words(lay);
    uint32_t* scr = st.scratch + (size_t)e * SW;
    uint32_t *tbits, *cbits, *vac;
    if constexpr (BIGG) {  // global (L2): read with agent-scope atomic loads, past the L1
        tbits = scr + wave_scratch_words(P);
        cbits = tbits + g.RW;
        vac = cbits + g.RW;
    } else {
        tbits = smem + S.tbits;
        cbits = smem + S.cbits;  // contested cell pairs (half resolution, see wave_lds)
        vac = smem + S.vac;
    }
    auto tc_get = [&](const uint32_t* b, int i) -> bool {
        if constexpr (BIGG)
            return (__hip_atomic_load(b + (i >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (i & 31)) & 1u;
        else
            return bit_get(b, i);
    };
    // contested target t (big grids: exact, global; others: its cell pair, LDS)
    auto cb_idx = [&](int t) -> int { return BIGG ? t : t >> 1; };
    auto cb_get = [&](int t) -> bool { return tc_get(cbits, cb_idx(t)); };
    uint32_t* nearc = smem + S.nearc;
    const int NCW = (((g.L + 2 + 3) >> 2) * ((GY + 3) >> 2) + 31) / 32;
    uint32_t* lost = BIGG ? vac + g.RW : smem + S.lost;  // BIGG: set by atomics, read by tc_get
    uint32_t* robots = smem + S.robots;
    uint32_t* misc = smem + S.misc;
    const uint32_t* __restrict__ validg = lay.valid_bits;

    uint32_t* pk_g = st.pk + (size_t)e * P;
    double* h_g = st.health + (size_t)e * P;
    double* a_g = st.acc + (size_t)e * P;
    uint2* plan = reinterpret_cast<uint2*>(scr);           // (person, cell | dir << 24) of every mover
    uint2* ndl = reinterpret_cast<uint2*>(scr + 2 * P);    // (person, person word) of the not-dead
    // light path: the persons in play (not safe, not dead) as (person | not-dead index << 16, word)
    // in the wide path's health region, and every not-dead person's health in list order
    // (frozen for the safe ones, updated by the rows for those in play) in the spill region
    uint2* ipl = reinterpret_cast<uint2*>(scr + wave_hv_offset(P));
    // kept between light steps (persist_offset): the lists' header and the list-order healths
    uint32_t* lhdr = scr + persist_offset(lay);
    double* hl = reinterpret_cast<double*>(lhdr + LHDR);
    const int n2P = pow2_ceil(P < 64 ? 64 : P);
    uint32_t* Lg = scr + 4 * P;                             // spill: contested list
    uint32_t* Hg = Lg + n2P;                                // spill: group heads
    uint32_t* Sg = Hg + n2P;                                // spill: group starts

    // ---------------------------------------------------------------- load
    const int* scal_g = st.scal + (size_t)e * 4;
    const int fs = scal_g[0], cur_step = scal_g[1], prev_evac = scal_g[2], prev_dead = scal_g[3];
    // light path: the in-play list and the list-order healths left by this env's previous (light)
    // step replace the scan of every person word and health (reset or a wide step invalidate them)
    const uint32_t lh_valid = lhdr[0], lh_nnd = lhdr[1], lh_nip = lhdr[2];  // (8-byte aligned only)
    const bool kept = !WIDE && __builtin_amdgcn_readfirstlane((int)(lh_valid == LISTS_VALID));
    uint32_t view = st.view[e];
    PT_DECL(ld1);
    PT_DECL(ld2);
    PT_DECL(ld3);
    PT_BEGIN(ld1);
    // every global read of this phase is issued before any of it is used
    uint32_t rp_pre = 0u;  // this lane's robot (Map.move_robot below)
    int a_pre = -1;
    if (lane < R) {
        rp_pre = st.robots[(size_t)e * R + lane];
        a_pre = actions[(size_t)e * R + lane];
    }
    const uint32_t* gpy = st.py_mt + (size_t)e * EVX_MT_WORDS;
    const uint32_t* gnp = st.np_mt + (size_t)e * EVX_MT_WORDS;
    uint32_t* gpyw = st.py_mt + (size_t)e * EVX_MT_WORDS;  // py_ensure / py_store (read above first)
    uint32_t wpy[10], wnp[10];
#pragma unroll
    for (int j = 0; j < 10; j++) {
        wpy[j] = 0u;
        wnp[j] = 0u;
        if (lane + 64 * j < EVX_MT_WORDS) {
            wpy[j] = gpy[lane + 64 * j];
            wnp[j] = gnp[lane + 64 * j];
        }
    }
    // the first rows of person words, in flight with the MT and rmap loads (the not-dead scan
    // below prefetches each next batch while it processes one)
    // light path: the rows' healths too (contiguous, all persons: no dependence on the words)
    constexpr int PKB = WIDE ? 12 : 8;
    uint32_t vv[PKB];
    double hr[WIDE ? 1 : PKB];
#pragma unroll
    for (int j = 0; j < PKB; j++) {
        const int p = j * 64 + lane;
        vv[j] = 2u << 24;
        if (!kept && p < P) vv[j] = pk_g[p];
        if constexpr (!WIDE) hr[j] = !kept && p < P ? h_g[p] : 0.0;
    }
    // kept lists: the rows' first in-play entries, in flight with the state loads (read past the
    // list's end only within the buffer; entries >= nip are dropped below)
    uint2 pre_e[2 * GQ];
#pragma unroll
    for (int j = 0; j < 2 * GQ; j++) {
        pre_e[j] = make_uint2(0u, DONEPK);
        if (!WIDE && kept && 64 * j + lane < P) pre_e[j] = ipl[64 * j + lane];
    }
    // Map.move_robot (envs/map.py:160-201): a robot's candidate cell and whether it may move there
    // (action in 0..4, inside the robots' range and the map); the cell's validity word is the one
    // read that depends on the state loads -- issued here, ahead of the MT / rmap LDS stores
    auto robot_cand = [&](uint32_t rp, int a, int& nx, int& ny) -> bool {
        const int x = rp_x(rp), y = rp_y(rp);
        nx = x;
        ny = y;
        if (a == 0) nx = x + 1;
        else if (a == 1) ny = y - 1;
        else if (a == 2) nx = x - 1;
        else if (a == 3) ny = y + 1;
        return a >= 0 && a <= 4 && lay.rx_lo <= nx && nx <= lay.rx_hi && 0 <= ny && ny <= g.W && nx >= 1 &&
               nx <= g.L && ny >= 1 && ny <= g.W;
    };
    int nx_pre = 0, ny_pre = 0;
    bool ok_pre = false;
    uint32_t vw_pre = 0u;
    if (lane < R) {
        ok_pre = robot_cand(rp_pre, a_pre, nx_pre, ny_pre);
        if (ok_pre) vw_pre = validg[(nx_pre * GY + ny_pre) >> 5];
    }
    const uint32_t* grm = st.rmap + (size_t)e * g.RW;
    for (int i0 = 0; i0 < g.RW; i0 += 16 * 64) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            w[j] = 0u;
            if (i0 + 64 * j + lane < g.RW) w[j] = grm[i0 + 64 * j + lane];
        }
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int i = i0 + 64 * j + lane;
            if (i < g.RW) {
                rmapb[i] = w[j];
                tbits[i] = 0;
                if constexpr (BIGG) cbits[i] = 0;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 10; j++) {
        if (lane + 64 * j < MT_N) {
            pyring[lane + 64 * j] = wpy[j];
            npring[lane + 64 * j] = wnp[j];
        }
    }
    int py_head = __builtin_amdgcn_readlane((int)wpy[9], MT_N - 576);  // word 624 = index
    int np_head = __builtin_amdgcn_readlane((int)wnp[9], MT_N - 576);
    for (int i = lane; i < (P + 31) / 32; i += 64) lost[i] = 0;
    if constexpr (!BIGG)
        for (int i = lane; i < cbits_words(g.G); i += 64) cbits[i] = 0;
    for (int i = lane; i < NCW; i += 64) nearc[i] = 0;
    int py_front = MT_N, np_front = MT_N;
    // Map.move_robot for every robot (envs/map.py:160-201); robots never interact.
    bool valid_a0 = false;
    for (int r = lane; r < R; r += 64) {
        uint32_t rp = r == lane ? rp_pre : st.robots[(size_t)e * R + r];
        const int a = r == lane ? a_pre : actions[(size_t)e * R + r];
        int nx = nx_pre, ny = ny_pre;
        bool ok = ok_pre;
        uint32_t vw = vw_pre;
        if (r != lane) {  // robots beyond the first 64 (R > 64)
            ok = robot_cand(rp, a, nx, ny);
            if (ok) vw = validg[(nx * GY + ny) >> 5];
        }
        if (ok && ((vw >> ((nx * GY + ny) & 31)) & 1u)) rp = rp_pack(nx, ny);
        robots[r] = rp;
        st.robots[(size_t)e * R + r] = rp;
        if (r == 0) valid_a0 = (a >= 0 && a <= 4);
    }
    PT_END(ld1);
    PT_BEGIN(ld2);
    // the not-dead persons in person order (sum(... if not p.dead) and the movers
    // never look at anyone else)
    int nnd = 0, n_safe = 0, nip = 0;
    if (kept) {
        nnd = __builtin_amdgcn_readfirstlane((int)lh_nnd);
        nip = __builtin_amdgcn_readfirstlane((int)lh_nip);
    }
    for (int r0 = 0; r0 < (kept ? 0 : NR); r0 += PKB) {  // PKB rows processed while the next PKB are in flight
        uint32_t nx[PKB];
        double hn[WIDE ? 1 : PKB];
#pragma unroll
        for (int j = 0; j < PKB; j++) {
            const int p = (r0 + PKB + j) * 64 + lane;
            nx[j] = 2u << 24;
            if (p < P) nx[j] = pk_g[p];
            if constexpr (!WIDE) hn[j] = p < P ? h_g[p] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < PKB; j++) {
            pin(vv[j]);
            const int p = (r0 + j) * 64 + lane;
            const bool nd = !pk_dead(vv[j]);
            const unsigned long long m = __ballot(nd);
            const int k = nnd + lanes_below(m);
            if constexpr (WIDE) {
                if (nd) ndl[k] = make_uint2((uint32_t)p, vv[j]);
                n_safe += __popcll(__ballot(nd && pk_safe(vv[j])));
            } else {  // the light path needs only the in-play list and the list-order healths
                if (nd) hl[k] = hr[j];
                const bool ip = nd && !pk_safe(vv[j]);
                const unsigned long long mi = __ballot(ip);
                if (ip) ipl[nip + lanes_below(mi)] = make_uint2((uint32_t)p | ((uint32_t)k << 16), vv[j]);
                nip += __popcll(mi);
            }
            nnd += __popcll(m);
        }
#pragma unroll
        for (int j = 0; j < PKB; j++) {
            vv[j] = nx[j];
            if constexpr (!WIDE) hr[j] = hn[j];
        }
    }
    if constexpr (!WIDE) n_safe = nnd - nip;
    wave_fence();
    PT_END(ld2);
    PT_BEGIN(ld3);
    if (__shfl((int)valid_a0, 0)) view = robots[0];  // robot_position refreshed only after a valid action
    // Coarse near-robot map: 4x4-cell blocks that may hold a cell within the repel
    // range of some robot; only there does find_best_direction's robot loop run.
    const int rd2 = lay.repel_d2;
    const int BY = (GY + 3) >> 2;
    int rr = 0;
    while ((rr + 1) * (rr + 1) < rd2) rr++;
    const int rb = rr + 1;  // a neighbour within range of a robot lies within rb of it in x and y
    if (rd2 > 0) {  // 16 robots per pass, 4 lanes each (a robot's range spans few blocks)
        for (int r0 = 0; r0 < R; r0 += 16) {
            const int r = r0 + (lane >> 2), sub = lane & 3;
            if (r < R) {
                const uint32_t rp = robots[r];
                const int bx0 = max(rp_x(rp) - rr, 0) >> 2, bx1 = min(rp_x(rp) + rr, g.L + 1) >> 2;
                const int by0 = max(rp_y(rp) - rr, 0) >> 2, by1 = min(rp_y(rp) + rr, g.W + 1) >> 2;
                if (bx1 >= bx0 && by1 >= by0) {
                    const int nby = by1 - by0 + 1;
                    const float inv = 1.0f / (float)nby;
                    for (int c = sub; c < (bx1 - bx0 + 1) * nby; c += 4) {
                        const int q = (int)(((float)c + 0.5f) * inv);  // c / nby, exact for c < 2^20
                        const int b = (bx0 + q) * BY + by0 + (c - q * nby);
                        atomicOr(&nearc[b >> 5], 1u << (b & 31));
                    }
                }
            }
        }
    }
    wave_sync();  // not-dead list and LDS tables complete
    PT_END(ld3);
    PT_STORE(ld1, 27);
    PT_STORE(ld2, 28);
    PT_STORE(ld3, 29);
    EVX_STAMP(1);

    // --------------------- People.run phases 1+2 (health, accumulate, plan)
    const double* __restrict__ dpt = lay.danger_p + (size_t)fs * g.G;
    const double* __restrict__ fd5 = lay.floor_d5;
    const uint8_t* __restrict__ nbv = lay.nbr_valid;
    int doff[8];
#pragma unroll
    for (int d = 0; d < 8; d++) doff[d] = move_dx(d) * GY + move_dy(d);

    int nplan = 0, n_died = 0;
    bool any_hit = false;  // some person in play took damage this step (wave-uniform)
#ifdef EVX_FCX
    int fcx = 0x7fffffff;  // diagnostic: the first not-dead-list index whose health changes this step
#endif
    // the persons in play that survive update_health, compacted in list order over the in-play
    // list's consumed entries: the reward pass walks them (light path; the wide rows: the
    // not-dead list, nrl = nnd)
    int nrl = nnd;
    const uint2* rl = ndl;
    bool any_cont = false;
    PT_DECL(np);
    PT_DECL(hsum);
    PT_DECL(plan);
    PT_DECL(drain);
    PT_DECL(top);
    PT_DECL(rew);
    PT_DECL(leaf);
    PT_DECL(rtop);
    PT_DECL(sbl);
    PT_DECL(sbm);
    PT_DECL(sbs);
    PT_DECL(sbt);
    double total = 0.0;  // CPython sum(p.health for p in self.people.list if not p.dead): sequential
    int fold_kept = 0;   // light path: entries of the kept list-order healths after this step
    // a light step whose planners were scored in one batch keeps its move plan in registers (lane k:
    // the batch's planner k, its target's cell info loaded at scoring time): no plan round trip
    uint2 rp_en = make_uint2(0u, 0u);
    uint32_t rp_ci = 0u;
    bool rp_mov = false;
    int nbatch = 0;
    if constexpr (WIDE) {
        WideCtl* ctl = reinterpret_cast<WideCtl*>(smem + wide_lds(lay).ctl);
        if (lane == 0) {
            ctl->nnd = nnd;
            ctl->np_head = np_head;
            ctl->py_head = py_head;
            ctl->fs = fs;
            ctl->any_cont = 0;
            ctl->total_ready = 0;
        }
        wave_sync();
        __syncthreads();  // the other waves of the workgroup join here
        rows_wide(lay, st, e, smem, out.stamps ? out.stamps + (size_t)e * 48 : nullptr);
        nplan = ctl->nplan;
        n_died = ctl->n_died;
        any_cont = ctl->any_cont != 0;
        py_front = ctl->py_front;
        py_head = ctl->py_head_out;
        EVX_COUNT(11, nplan);
    } else {
    // Planners wait in an LDS queue and are scored 64 at a time (scoring is the
    // heavy part and only a few persons per row plan).
    uint32_t* qa = aux;        // person | candidate mask << 16   (<= 127 queued)
    uint32_t* qb = aux + 128;  // x | y << 12
    int* qc = reinterpret_cast<int*>(aux + 256);        // first Python-stream word
    int qn = 0;
    int nal = 0;  // alive persons in play so far (see nrl)
    auto score_batch = [&](int n, bool only) {  // People.find_best_direction for queue entries [0, n)
        // (only: the step's one batch -- its plan stays in registers, not in HBM)
        PT_BEGIN(sbl);
        const bool has = lane < n;
        uint32_t ea = 0, eb = 0;
        int off = 0;
        if (has) {
            ea = qa[lane];
            eb = qb[lane];
            off = qc[lane];
        }
        const int p = (int)(ea & 0xffffu);
        const uint32_t cand = ea >> 16;
        const int x = pk_x(eb), y = pk_y(eb), cold = x * GY + y;
        const int first = __builtin_amdgcn_readfirstlane(off);
        const int end = __builtin_amdgcn_readlane(off + 2 * __popc(cand), n - 1);
        DirPrep dp;
        dir_prep(dp, has, x, y, cand, GY, fd5, nearc, BY, robots, R, rb);
#ifdef EVX_PROFILE
#pragma unroll
        for (int d = 0; d < 8; d++) pin(dp.f[d]);
#endif
        PT_END(sbl);
        uint32_t best = NODIR;
        for (int lo = first; lo < end; lo += WWIN) {  // windowed: a batch may need more words than the ring
            PT_BEGIN(sbm);
            py_ensure(pyring, py_front, min(end, lo + WWIN + 16), gpyw, end);
            PT_END(sbm);
            PT_BEGIN(sbs);
            if (has && off >= lo && off < lo + WWIN) best = dir_score(dp, cand, off, pyring, 0, 0, lay.repel_k, rd2);
            PT_END(sbs);
        }
        PT_BEGIN(sbt);
        const bool mover = best != NODIR;
        const unsigned long long mm = __ballot(mover);
        nbatch++;
        rp_mov = mover;
        if (mover) {
            const int t = cold + doff_of(best, GY);
            rp_en = make_uint2((uint32_t)p, (uint32_t)cold | (best << 24));
            rp_ci = lay.cellinfo[t];
            const uint32_t bit = 1u << (t & 31);
            const uint32_t old = atomicOr(&tbits[t >> 5], bit);
            if (old & bit) {
                const int ci = cb_idx(t);
                atomicOr(&cbits[ci >> 5], 1u << (ci & 31));
                any_cont = true;
            }
            if (!only) plan[nplan + lanes_below(mm)] = make_uint2((uint32_t)p, (uint32_t)cold | (best << 24));
        }
        nplan += __popcll(mm);
        PT_END(sbt);
    };
    // one group (64 list entries, in person order) of People.run phases 1+2
    // one group (64 entries of the in-play list, in person order) of People.run phases 1+2
    auto person_half = [&](int i, uint2 en, double hh, double ac, double dg, uint32_t nv) {
        PT_BEGIN(np);
        const bool inr = i < nip;
        const int p = (int)(en.x & 0xffffu);
        const uint32_t v = en.y;
        const bool act = inr;
        const int x = pk_x(v), y = pk_y(v), cold = x * GY + y;
        // phase 1: Person.update_state -> update_health (numpy stream)
        const bool need = act && dg > 0;
        const unsigned long long nm = __ballot(need);
        any_hit |= nm != 0ull;
        const int tot = 2 * __popcll(nm);
        bool alive = act, died = false;
        if (tot) {
            np_ensure(npring, np_front, np_head + tot);
            if (need) {
                const double u = np_double(npring, np_head + 2 * lanes_below(nm));
                if (update_health(hh, dg, u)) {
                    died = true;
                    alive = false;
                }
            }
            np_head += tot;
        }
        const unsigned long long dm = __ballot(died);
        n_died += __popcll(dm);
#ifdef EVX_FCX
        if (need) fcx = min(fcx, (int)(en.x >> 16));
#endif
        {
            // entry i of the not-dead list was read two iterations ago: the compacted alive list
            // (index <= i) overwrites only consumed entries. Each keeps its index in the not-dead
            // list as it will stand after this step's deaths are dropped (deaths only happen among
            // the persons in play, so those before it are the deaths earlier in this list)
            const unsigned long long am = __ballot(alive);
            const uint32_t knew = (en.x >> 16) - (uint32_t)(n_died - __popcll(dm) + lanes_below(dm));
            if (alive) ipl[nal + lanes_below(am)] = make_uint2((uint32_t)p | (knew << 16), v);
            nal += __popcll(am);
        }
        PT_END(np);
        // the list-order health the fold reads; a death leaves -0.0 (adds nothing to the running
        // sum, which is >= +0.0) and marks the slot the fold drops from the kept list
        if (need) hl[en.x >> 16] = died ? -0.0 : hh;  // the others' kept entries are unchanged
        PT_BEGIN(plan);
        // phase 2: accumulate; candidates of find_best_direction
        bool planner = false;
        if (alive) {
            ac += person_speed(hh) * 0.5;
            if (ac >= 1.0) {
                ac -= 1.0;
                planner = true;
            }
        }
        uint32_t cand = 0;
        if (planner) {
            uint32_t occ = 0;
#pragma unroll
            for (int d = 0; d < 8; d++) occ |= (uint32_t)bit_get(rmapb, cold + doff[d]) << d;
            cand = nv & ~occ;
        }
        // queue the planners with >= 1 candidate; their Python-stream words are
        // assigned here, in person order (exclusive prefix of 2*|cand| by bit-sliced ballots)
        const int ncand = __popc(cand);
        int off2 = 0, tot2 = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const unsigned long long m = __ballot((ncand >> b) & 1);
            off2 += lanes_below(m) << (b + 1);
            tot2 += __popcll(m) << (b + 1);
        }
        const unsigned long long qm = __ballot(cand != 0);
        if (cand) {
            const int k = qn + lanes_below(qm);
            qa[k] = (uint32_t)p | (cand << 16);
            qb[k] = (uint32_t)x | ((uint32_t)y << 12);
            qc[k] = py_head + off2;
        }
        py_head += tot2;
        qn += __popcll(qm);
        if (need) h_g[p] = hh;
        if (alive) a_g[p] = ac;
        if (died) pk_g[p] = v | (2u << 24);
        PT_END(plan);
    };
    // Four 64-person groups per iteration: the next iteration's data and the
    // list entries of the one after are in flight while this one computes. The
    // per-group body exists once (a group is picked by selects), as does the scorer.
    const uint2 NOONE = make_uint2(0u, DONEPK);
    auto load_entry = [&](int i) -> uint2 {
        uint2 en = NOONE;
        if (i < nip) en = ipl[i];
        return en;
    };
    auto load_data = [&](int i, uint2 en, double& h, double& a, double& dg, uint32_t& nv) {
        h = 0.0; a = 0.0; dg = 0.0; nv = 0u;
        if (i < nip) {
            const uint32_t pe = en.x & 0xffffu;
            const int c = pk_x(en.y) * GY + pk_y(en.y);
            h = h_g[pe];
            a = a_g[pe];
            dg = dpt[c];
            nv = nbv[c];
        }
    };
    uint2 nxe[GQ], nne[GQ];
    double nxh[GQ], nxa[GQ], nxg[GQ];
    uint32_t nxv[GQ];
#pragma unroll
    for (int k = 0; k < GQ; k++) {
        if (kept) {  // loaded with the state
            nxe[k] = 64 * k + lane < nip ? pre_e[k] : NOONE;
            nne[k] = 64 * (GQ + k) + lane < nip ? pre_e[GQ + k] : NOONE;
        } else {
            nxe[k] = load_entry(64 * k + lane);
            nne[k] = load_entry(64 * (GQ + k) + lane);
        }
    }
#pragma unroll
    for (int k = 0; k < GQ; k++) load_data(64 * k + lane, nxe[k], nxh[k], nxa[k], nxg[k], nxv[k]);
    const int NIT = (nip + 64 * GQ - 1) / (64 * GQ);
    for (int it = 0; it <= NIT; it++) {  // the extra iteration only drains the planner queue
        PT_BEGIN(top);
        const int i0 = it * 64 * GQ + lane;
        uint2 ce[GQ];
        double chh[GQ], caa[GQ], cgg[GQ];
        uint32_t cvv[GQ];
#pragma unroll
        for (int k = 0; k < GQ; k++) {
            ce[k] = nxe[k];
            chh[k] = nxh[k];
            caa[k] = nxa[k];
            cgg[k] = nxg[k];
            cvv[k] = nxv[k];
            nxe[k] = nne[k];
            pin(ce[k]);
            pin(chh[k]);
            pin(caa[k]);
            pin(cgg[k]);
            pin(cvv[k]);
            pin(nxe[k]);
        }
#pragma unroll
        for (int k = 0; k < GQ; k++) load_data(i0 + 64 * (GQ + k), nxe[k], nxh[k], nxa[k], nxg[k], nxv[k]);
#pragma unroll
        for (int k = 0; k < GQ; k++) nne[k] = load_entry(i0 + 64 * (2 * GQ + k));
#pragma clang loop unroll(disable)
        for (int k = 0; k < GQ; k++) {
            uint2 en = ce[0];
            double hh = chh[0], ac = caa[0], dg = cgg[0];
            uint32_t nv = cvv[0];
#pragma unroll
            for (int j = 1; j < GQ; j++) {
                if (k == j) {
                    en = ce[j];
                    hh = chh[j];
                    ac = caa[j];
                    dg = cgg[j];
                    nv = cvv[j];
                }
            }
            PT_END(top);
            person_half(i0 + 64 * k, en, hh, ac, dg, nv);
            const bool fin = it == NIT && k == GQ - 1;
            PT_BEGIN(drain);
            while (qn >= 64 || (fin && qn > 0)) {
                wave_fence();
                const int n = min(qn, 64);
                score_batch(n, fin && nbatch == 0 && qn == n);
                const int rest = qn - n;  // move entries [n, qn) to the front (rest <= 126)
                uint32_t ta[2] = {0u, 0u}, tb[2] = {0u, 0u};
                int tc[2] = {0, 0};
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    if (lane + 64 * j < rest) {
                        ta[j] = qa[n + lane + 64 * j];
                        tb[j] = qb[n + lane + 64 * j];
                        tc[j] = qc[n + lane + 64 * j];
                    }
                }
                wave_fence();
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    if (lane + 64 * j < rest) {
                        qa[lane + 64 * j] = ta[j];
                        qb[lane + 64 * j] = tb[j];
                        qc[lane + 64 * j] = tc[j];
                    }
                }
                qn = rest;
                wave_fence();
            }
            PT_END(drain);
            PT_BEGIN(top);
        }
        PT_END(top);
    }
    // the numpy stream is finished for this step
    np_store(npring, np_front, np_head, st.np_mt + (size_t)e * EVX_MT_WORDS);
#ifdef EVX_FCX
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) fcx = min(fcx, __shfl_xor(fcx, o, 64));
    EVX_COUNT(36, fcx);
    EVX_COUNT(37, nnd);
#endif
    nrl = nal;
    rl = ipl;
    EVX_COUNT(13, np_head);
    EVX_COUNT(11, nplan);
    }  // !WIDE
    any_cont = __ballot(any_cont) != 0;
    wave_sync();  // plan[] and the person writes are visible to every lane
    // No one in play took damage: every health and the not-dead list are as the previous step left
    // them (a death needs damage), so CPython's sum is the previous step's total, bit for bit. That
    // holds for ~60 % of the envs at the stationary mix, and the fold (a dependent f64 add chain
    // over ~720 persons, ~16 k cycles) is skipped for them.
    const bool same_total = !WIDE && kept && !any_hit;
    if (same_total) {
        total = *reinterpret_cast<const double*>(lhdr + 4);
        fold_kept = nnd;
    }
    if (!WIDE && !same_total) {
        // CPython's sum(p.health for p in self.people.list if not p.dead): lane 0 folds the
        // not-dead list's healths (after update_health; +0.0 for this step's deaths, which leaves
        // the running sum unchanged) in list order, staged 64 at a time through LDS; the loads of
        // the next 4 groups are in flight while a group is folded
        PT_BEGIN(hsum);
        double* hc = reinterpret_cast<double*>(aux + 384);
        constexpr int FB = 4;
        int nkeep = 0;  // the kept list for the next step: this step's deaths (-0.0) dropped, in place
        double fv[FB];
#pragma unroll
        for (int k = 0; k < FB; k++) fv[k] = 64 * k + lane < nnd ? hl[64 * k + lane] : 0.0;
        for (int i0 = 0; i0 < nnd; i0 += 64 * FB) {
            double fn[FB];
#pragma unroll
            for (int k = 0; k < FB; k++) {
                const int i = i0 + 64 * (FB + k) + lane;
                fn[k] = i < nnd ? hl[i] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < FB; k++) {
                if (i0 + 64 * k >= nnd) break;
                pin(fv[k]);
                hc[lane] = fv[k];
                {
                    const bool keep = i0 + 64 * k + lane < nnd && !signbit(fv[k]);
                    const unsigned long long km = __ballot(keep);
                    const int dst = nkeep + lanes_below(km);  // <= read index: a consumed entry
                    if (keep && dst != i0 + 64 * k + lane) hl[dst] = fv[k];  // only entries behind a death move
                    nkeep += __popcll(km);
                }
                wave_fence();
                if (lane == 0) {
                    const double2* h2 = reinterpret_cast<const double2*>(hc);
                    double2 q0 = h2[0], q1 = h2[1], q2 = h2[2], q3 = h2[3];
                    double2 r0 = h2[4], r1 = h2[5], r2 = h2[6], r3 = h2[7];
#pragma unroll
                    for (int c = 0; c < 8; c++) {
                        double2 s0 = q0, s1 = q1, s2 = q2, s3 = q3;
                        if (c + 2 < 8) {
                            s0 = h2[4 * (c + 2)];
                            s1 = h2[4 * (c + 2) + 1];
                            s2 = h2[4 * (c + 2) + 2];
                            s3 = h2[4 * (c + 2) + 3];
                        }
                        total += q0.x; total += q0.y; total += q1.x; total += q1.y;
                        total += q2.x; total += q2.y; total += q3.x; total += q3.y;
                        q0 = r0; q1 = r1; q2 = r2; q3 = r3;
                        r0 = s0; r1 = s1; r2 = s2; r3 = s3;
                    }
                }
                wave_fence();
            }
#pragma unroll
            for (int k = 0; k < FB; k++) fv[k] = fn[k];
        }
        fold_kept = nkeep;
        PT_END(hsum);
    }
    EVX_STAMP(2);

    // The move plan in HBM is walked 4 x 64 entries at a time, loads first (or, one batch, from
    // the registers its scoring left: lane k's entry is valid iff it moves).
    const bool preg = !WIDE && nbatch <= 1;

    // ------------------------- contested targets: groups, shuffle, losers
    int err = 0;
    if (!WIDE && fold_kept != nnd - n_died) err |= 32;  // kept list out of step with the counts
    int ncont = 0;
    PT_DECL(lp);
    PT_DECL(grp);
    PT_DECL(mts);
    long long cgp[7] = {0, 0, 0, 0, 0, 0, 0};  // EVX_PROFILE: sort, heads, pass 1, pass 2, windows, groups, window cycles
    PT_BEGIN(lp);
    uint32_t* Lp = npring;  // the numpy ring is free now
    // the (candidate) contested movers, their contested-bitmap words loaded 4 x 64 at a time before
    // any is used (big grids: from L2)
    auto cont_pass = [&](auto&& fn) {
        auto one = [&](const uint2 en, bool ok, uint32_t cw) {
            const int t = (int)(en.y & 0xffffffu) + doff_of(en.y >> 24, GY);
            const bool c = ok && ((cw >> (cb_idx(t) & 31)) & 1u);
            fn(c, ((uint32_t)t << pb) | en.x);
        };
        auto cword = [&](const uint2 en, bool ok) -> uint32_t {
            if (!ok) return 0u;
            const int t = (int)(en.y & 0xffffffu) + doff_of(en.y >> 24, GY);
            if constexpr (BIGG)
                return __hip_atomic_load(cbits + (t >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                return cbits[cb_idx(t) >> 5];
        };
        if (preg) {
            one(rp_en, rp_mov, cword(rp_en, rp_mov));
            return;
        }
        for (int i0 = 0; i0 < nplan; i0 += 256) {
            uint2 en[4];
            uint32_t cw[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                en[j] = make_uint2(0u, 0u);
                if (i0 + 64 * j + lane < nplan) en[j] = plan[i0 + 64 * j + lane];
            }
#pragma unroll
            for (int j = 0; j < 4; j++) cw[j] = cword(en[j], i0 + 64 * j + lane < nplan);
#pragma unroll
            for (int j = 0; j < 4; j++) one(en[j], i0 + 64 * j + lane < nplan, cw[j]);
        }
    };
    if (any_cont) {
        cont_pass([&](bool c, uint32_t key) {
            const unsigned long long m = __ballot(c);
            const int pos = ncont + lanes_below(m);
            if (c && pos < CL_CAP) Lp[pos] = key;
            ncont += __popcll(m);
        });
        PT_END(lp);
        PT_BEGIN(grp);
        if (ncont <= CL_CAP) {
            contested_groups(Lp, aux, aux + 256, ncont, pb, pyring, py_front, py_head, lost, misc, err, cgp, gpyw);
        } else {  // rare: sort in this env's global scratch
            Lp = Lg;
            int k = 0;
            cont_pass([&](bool c, uint32_t key) {
                const unsigned long long m = __ballot(c);
                if (c) Lg[k + lanes_below(m)] = key;
                k += __popcll(m);
            });
            wave_sync();
            contested_groups(Lg, Hg, Sg, ncont, pb, pyring, py_front, py_head, lost, misc, err, cgp, gpyw);
        }
    }
    PT_END(grp);
    PT_BEGIN(mts);
    EVX_COUNT(14, ncont);
    // py_ensure stores a block only while the stream's final head may lie in it; once the front runs
    // 2 blocks past the head's block, a later crossing has overwritten that stored copy: flag it
    if (py_head > MT_N && py_front > MT_N * ((py_head - 1) / MT_N) + 2 * MT_N) err |= 64;
    py_store(pyring, py_front, py_head, gpyw);
    EVX_COUNT(12, py_head);
    // the Python stream is stored: its ring becomes the "vacated by a winner" bitmap
    for (int i = lane; i < g.RW; i += 64) vac[i] = 0;
    if constexpr (BIGG) wave_sync(); else wave_fence();  // LDS (big grids: global); the state stores drain later
    PT_END(mts);
    PT_STORE(lp, 24);
    PT_STORE(grp, 25);
    PT_STORE(mts, 26);
#ifdef EVX_PROFILE
    EVX_COUNT(32, cgp[0]);
    EVX_COUNT(33, cgp[1]);
    EVX_COUNT(34, cgp[2]);
    EVX_COUNT(35, cgp[3]);
    EVX_COUNT(46, cgp[4] * 65536 + cgp[5]);
    EVX_COUNT(47, cgp[6]);
#endif
    EVX_STAMP(3);

    // the reward's first list entries (the rows phase left the list final) are loaded here, so
    // their latency runs under execute_move's (the person words they index are read after it)
    auto load_idx = [&](int i) -> uint32_t {  // person | (list index << 16)
        uint32_t p = 0u;
        if (i < nrl) p = rl[i].x;
        return p;
    };
    uint32_t nxj[GQ], nnj[GQ];
#pragma unroll
    for (int k = 0; k < GQ; k++) {
        nxj[k] = load_idx(64 * k + lane);
        nnj[k] = load_idx(64 * (GQ + k) + lane);
    }

    // --------------------------------------------- execute_move, in order
    // The word of bitmap b holding bit i. Big grids keep the contested / loser / target / vacated
    // bitmaps in L2 (agent-scope loads past the L1): both passes below load every word an entry
    // needs for all (up to 4 x 64) entries of a block before using any -- one round trip per block
    // instead of two or three per 64 entries.
    auto bit_w = [&](const uint32_t* b, int i) -> uint32_t {
        if constexpr (BIGG)
            return __hip_atomic_load(b + (i >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            return b[i >> 5];
    };
    auto vac_entry = [&](const uint2 en, bool ok, uint32_t wc, uint32_t wl) {
        if (ok) {
            const int cold = (int)(en.y & 0xffffffu);
            const int t = cold + doff_of(en.y >> 24, GY);
            const bool cont = any_cont && ((wc >> (cb_idx(t) & 31)) & 1u);
            const bool win = !cont || !((wl >> ((int)en.x & 31)) & 1u);
            if (win) atomicOr(&vac[cold >> 5], 1u << (cold & 31));
            if (st.thmap) atomicAdd(&st.thmap[(size_t)e * g.G + (win ? t : cold)], 1);
        }
    };
    if (preg) {
        uint32_t wc = 0u, wl = 0u;
        if (rp_mov) {
            const int t = (int)(rp_en.y & 0xffffffu) + doff_of(rp_en.y >> 24, GY);
            if (any_cont) wc = bit_w(cbits, cb_idx(t));
            wl = bit_w(lost, (int)rp_en.x);
        }
        vac_entry(rp_en, rp_mov, wc, wl);
    } else {
        for (int i0 = 0; i0 < nplan; i0 += 256) {
            uint2 en[4];
            uint32_t wc[4], wl[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                en[j] = make_uint2(0u, 0u);
                if (i0 + 64 * j + lane < nplan) en[j] = plan[i0 + 64 * j + lane];
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                wc[j] = wl[j] = 0u;
                if (i0 + 64 * j + lane < nplan) {
                    const int t = (int)(en[j].y & 0xffffffu) + doff_of(en[j].y >> 24, GY);
                    if (any_cont) wc[j] = bit_w(cbits, cb_idx(t));
                    wl[j] = bit_w(lost, (int)en[j].x);
                }
            }
#pragma unroll
            for (int j = 0; j < 4; j++) vac_entry(en[j], i0 + 64 * j + lane < nplan, wc[j], wl[j]);
        }
    }
    if (lane == 0) misc[0] = 0;
    if constexpr (BIGG) wave_sync(); else wave_fence();  // vac: LDS (big grids: global)
    uint32_t* ev = aux;  // (cell, key) pairs; groups are done
    int n_evac_new = 0;
    // a step with <= 64 movers writes back only the rmap words its winners changed (cold, t)
    const bool rm_dirty = nplan <= 64;
    int dw0 = -1, dw1 = -1;
    // bits: the words of the contested, loser, target (cold) and vacated (t) bitmaps (bit_w)
    auto exec_entry = [&](const uint2 en, const uint32_t ci, const bool valid, const uint4 wb) {
        bool exw = false;
        if (valid) {
            const int p = (int)en.x;
            const int cold = (int)(en.y & 0xffffffu);
            const int dd = (int)(en.y >> 24);
            const int t = cold + doff_of((uint32_t)dd, GY);
            const bool cont = any_cont && ((wb.x >> (cb_idx(t) & 31)) & 1u);
            if (!cont || !((wb.y >> (p & 31)) & 1u)) {
                const bool ex = (ci >> 1) & 1u;
                exw = ex;
                const bool ev_old = (wb.z >> (cold & 31)) & 1u, ev_new = (wb.w >> (t & 31)) & 1u;
                int pf = p;
                if ((ev_old || ev_new) && cont) pf = find_pf(Lp, ncont, t, pb, p);
                if (ev_old) {
                    const int s = atomicAdd((int*)&misc[0], 1);
                    if (s < EV_CAP) {
                        ev[2 * s] = (uint32_t)cold;
                        ev[2 * s + 1] = ((uint32_t)pf << 2) | 0u;  // sub-step 0: leave, value 0
                    }
                } else {
                    atomicAnd(&rmapb[cold >> 5], ~(1u << (cold & 31)));
                }
                if (ev_new) {
                    const int s = atomicAdd((int*)&misc[0], 1);
                    if (s < EV_CAP) {
                        ev[2 * s] = (uint32_t)t;
                        ev[2 * s + 1] = ((uint32_t)pf << 2) | 2u | (ex ? 0u : 1u);
                    }
                } else if (ex) {
                    atomicAnd(&rmapb[t >> 5], ~(1u << (t & 31)));
                } else {
                    atomicOr(&rmapb[t >> 5], 1u << (t & 31));
                }
                const int ox = cold / GY, oy = cold - ox * GY;
                pk_g[p] = (uint32_t)(ox + move_dx(dd)) | ((uint32_t)(oy + move_dy(dd)) << 12) | (ex ? (1u << 24) : 0u);
                dw0 = cold >> 5;
                dw1 = t >> 5;
            }
        }
        n_evac_new += __popcll(__ballot(exw));
    };
    auto exec_words = [&](const uint2 en) -> uint4 {
        const int cold = (int)(en.y & 0xffffffu);
        const int t = cold + doff_of(en.y >> 24, GY);
        return make_uint4(any_cont ? bit_w(cbits, cb_idx(t)) : 0u, bit_w(lost, (int)en.x), bit_w(tbits, cold),
                          bit_w(vac, t));
    };
    if (preg) {
        exec_entry(rp_en, rp_ci, rp_mov, rp_mov ? exec_words(rp_en) : make_uint4(0u, 0u, 0u, 0u));
    } else {
        for (int i0 = 0; i0 < nplan; i0 += 256) {
            uint2 en4[4];
            uint32_t ci4[4];
            uint4 wb4[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                en4[j] = make_uint2(0u, 0u);
                if (i0 + 64 * j + lane < nplan) en4[j] = plan[i0 + 64 * j + lane];
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {  // exit bits and bitmap words of the targets, all in flight
                ci4[j] = 0u;
                wb4[j] = make_uint4(0u, 0u, 0u, 0u);
                if (i0 + 64 * j + lane < nplan) {
                    ci4[j] = lay.cellinfo[(int)(en4[j].y & 0xffffffu) + doff_of(en4[j].y >> 24, GY)];
                    wb4[j] = exec_words(en4[j]);
                }
            }
#pragma unroll
            for (int j = 0; j < 4; j++) exec_entry(en4[j], ci4[j], i0 + 64 * j + lane < nplan, wb4[j]);
        }
    }
    // LDS hand-offs only (the person words are drained below); big grids' bitmaps are global
    if constexpr (BIGG) wave_sync(); else wave_fence();
    {
        const int nev = (int)misc[0];
        if (nev > EV_CAP) err |= 16;
        const int ne = min(nev, EV_CAP);
        for (int i = lane; i < ne; i += 64) {  // last writer = largest (first planner, sub-step)
            const uint32_t c = ev[2 * i], kv = ev[2 * i + 1];
            bool top = true;
            for (int j = 0; j < ne; j++)
                if (ev[2 * j] == c && ev[2 * j + 1] > kv) top = false;
            if (top) {
                if (kv & 1u) atomicOr(&rmapb[c >> 5], 1u << (c & 31));
                else atomicAnd(&rmapb[c >> 5], ~(1u << (c & 31)));
            }
        }
    }
    wave_sync();  // the person words of the movers and the rmap bits complete
    EVX_STAMP(4);

    // ---------------------------------- fire update (both fire models)
    const int fs1 = fs < lay.t_max ? fs + 1 : fs;

    // ------------------------------------ _calculate_reward + counters
    const int evac = n_safe + n_evac_new, dead = (P - nnd) + n_died;
    const int nrem = P - evac - dead;
    int* ltab = reinterpret_cast<int*>(aux);  // leaf offsets | lengths
    double* leafsum = reinterpret_cast<double*>(pyring);
    // the remaining persons' robot distances, in list order, go to the numpy ring's LDS (free since
    // the contested lists) when they fit -- the leaf sums then read LDS after a wave fence -- else
    // to the move-plan scratch (P doubles; the plan is dead once executed, but the leaf sums must
    // wait for the stores to drain); the numpy leaves are summed after the pass
    const bool dist_lds = nrem <= MT_N / 2;
    double* dist = dist_lds ? reinterpret_cast<double*>(npring) : reinterpret_cast<double*>(plan);
    int nleaf = 0;
    if (lane == 0 && nrem > 0)
        nleaf = np_pairwise_leaves(nrem, ltab, ltab + LEAF_CAP, LEAF_CAP, reinterpret_cast<int*>(misc));
    nleaf = __shfl(nleaf, 0);
    if (nleaf > LEAF_CAP) {
        err |= 8;
        nleaf = 0;
    }
    wave_fence();
    const int vx = rp_x(view), vy = rp_y(view);
    double gq_t = 0.0;
    int q = 0;
    // remaining persons = the list nrl (the alive persons in play, or the whole not-dead list)
    // minus this step's deaths and evacuations
    auto reward_half = [&](int i, uint32_t v, double hv, uint32_t px) {
        PT_BEGIN(rew);
        const bool rem = i < nrl && !pk_safe(v) && !pk_dead(v);
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
        const unsigned long long rm = __ballot(rem);
        if (rem) dist[q + lanes_below(rm)] = 0.5 * sqrt((double)n4);
        // light path: the persons still in play are the next step's in-play list (entry i was
        // read two groups ago: index <= i overwrites only consumed entries)
        if (!WIDE && rem) ipl[q + lanes_below(rm)] = make_uint2(px, v);
        q += __popcll(rm);
        PT_END(rew);
    };
    auto load_pw = [&](int i, uint32_t px, uint32_t& w, double& h) {
        w = DONEPK;
        h = 0.0;
        if (i < nrl) {
            const uint32_t p = px & 0xffffu;
            w = pk_g[p];
            h = h_g[p];
        }
    };
    uint32_t nxw[GQ];
    double nxhv[GQ];
#pragma unroll
    for (int k = 0; k < GQ; k++) load_pw(64 * k + lane, nxj[k], nxw[k], nxhv[k]);
    // People.rmap back to HBM only now: stores issued before those loads would hold their waits
    // (vmcnt counts loads and stores in issue order)
    if (rm_dirty) {  // the words a winner changed (repeats store the same final value)
        if (dw0 >= 0) st.rmap[(size_t)e * g.RW + dw0] = rmapb[dw0];
        if (dw1 >= 0 && dw1 != dw0) st.rmap[(size_t)e * g.RW + dw1] = rmapb[dw1];
    } else {
        for (int i = lane; i < g.RW; i += 64) st.rmap[(size_t)e * g.RW + i] = rmapb[i];
    }
    const int NITR = (nrl + 64 * GQ - 1) / (64 * GQ);
    for (int it = 0; it < NITR; it++) {
        PT_BEGIN(rtop);
        const int i0 = it * 64 * GQ + lane;
        uint32_t cw[GQ];
        double ch[GQ];
        uint32_t cj[GQ];
#pragma unroll
        for (int k = 0; k < GQ; k++) {
            cw[k] = nxw[k];
            ch[k] = nxhv[k];
            cj[k] = nxj[k];
            nxj[k] = nnj[k];
            pin(cw[k]);
            pin(ch[k]);
            pin(nxj[k]);
        }
#pragma unroll
        for (int k = 0; k < GQ; k++) load_pw(i0 + 64 * (GQ + k), nxj[k], nxw[k], nxhv[k]);
#pragma unroll
        for (int k = 0; k < GQ; k++) nnj[k] = load_idx(i0 + 64 * (2 * GQ + k));
#pragma clang loop unroll(disable)
        for (int k = 0; k < GQ; k++) {
            uint32_t w = cw[0], px = cj[0];
            double h = ch[0];
#pragma unroll
            for (int j = 1; j < GQ; j++) {
                if (k == j) {
                    w = cw[j];
                    h = ch[j];
                    px = cj[j];
                }
            }
            PT_END(rtop);
            reward_half(i0 + 64 * k, w, h, px);
            PT_BEGIN(rtop);
        }
        PT_END(rtop);
    }
    PT_BEGIN(leaf);
    if (dist_lds)
        wave_fence();  // the distances (LDS) are visible to every lane
    else
        wave_sync();   // the distances (global scratch) are visible to every lane
    // numpy's pairwise leaves (<= 128 elements), 8 at a time: lane = 8 * leaf + chain j;
    // chain j sums a[j], a[j + 8], ... (numpy's r[j]), the 8 chains meet as
    // ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) by xor-shuffles, and the leaf's
    // chain-0 lane adds the len % 8 tail in order (or sums a short leaf from 0.0)
    for (int l0 = 0; l0 < nleaf; l0 += 8) {
        const int li = l0 + (lane >> 3), j = lane & 7;
        int o = 0, len = 0;
        if (li < nleaf) {
            o = ltab[li];
            len = ltab[LEAF_CAP + li];
        }
        const int len8 = len >= 8 ? len - (len % 8) : 0;
        double a[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            a[k] = 0.0;  // padding: d + 0.0 == d for the non-negative distances
            if (8 * k < len8) a[k] = dist[o + 8 * k + j];
        }
        double r = a[0];
#pragma unroll
        for (int k = 1; k < 16; k++) r += a[k];
        r += __shfl_xor(r, 1, 64);
        r += __shfl_xor(r, 2, 64);
        r += __shfl_xor(r, 4, 64);
        if (j == 0 && li < nleaf) {
            double res = len >= 8 ? r : 0.0;
            for (int k = len8; k < len; k++) res += dist[o + k];
            leafsum[li] = res;
        }
    }
    wave_fence();
    PT_END(leaf);
    const double gq = wave_sum_d(gq_t);  // multiples of 0.5: exact in any order
    PT_STORE(np, 16);
    PT_STORE(hsum, 17);
    PT_STORE(plan, 18);
    PT_STORE(drain, 19);
    PT_STORE(top, 20);
    PT_STORE(rew, 21);
    PT_STORE(leaf, 22);
    PT_STORE(rtop, 23);
    PT_STORE(sbl, 30);
    PT_STORE(sbm, 31);
    PT_STORE(sbs, 15);
    PT_STORE(sbt, 7);
    EVX_STAMP(5);
    if constexpr (WIDE) {  // the health total folded by wave 1
        WideCtl* ctl = reinterpret_cast<WideCtl*>(smem + wide_lds(lay).ctl);
        while (__hip_atomic_load(&ctl->total_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
            __builtin_amdgcn_s_sleep(4);
        total = ctl->total;
    }
    if (lane == 0) {
        const int remaining = nrem;
        double reward = 0.0;
        reward += (evac - prev_evac) * lay.evac_reward;
        reward += gq;
        if (remaining > 0 && nleaf > 0) {
            const double avg = np_pairwise_combine(nrem, leafsum, reinterpret_cast<int*>(misc),
                                                   reinterpret_cast<double*>(misc + 64)) /
                               (double)nrem;
            const double dr = 2.0 - fabs(avg - 8.0) * 0.2;
            reward += dr > 0 ? dr : 0.0;
        }
        if (remaining > 0) {
            const double urgency = (double)remaining / (double)P;
            reward += -0.05 - (urgency * 0.1);
        } else {
            reward -= 0.02;
        }
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
        if (st.perm_ws) st.perm_ws[e] = env_class(lay, fs1, evac, dead);  // a fused reset rewrites it
        if (err && out.err) atomicOr(out.err, err);
        // the lists the next light step starts from (a wide step's are not kept; a fused reset
        // below invalidates them again)
        lhdr[0] = WIDE ? 0u : LISTS_VALID;
        lhdr[1] = (uint32_t)(nnd - n_died);
        lhdr[2] = (uint32_t)q;
        *reinterpret_cast<double*>(lhdr + 4) = total;
    }

    EVX_STAMP(6);
    // ------------------------------------------------- observations
    // People.rmap is only ever set on valid cells, so Check_Valid reduces to the
    // interior range test here (no table reads).
    // with auto-reset, a finished env's terminal observation goes to obs_term and
    // the env is reset right here (its wave is light by then: few persons left)
    const bool fin = __builtin_amdgcn_readfirstlane((int)((evac + dead == P) || (0.5 * (double)(cur_step + 1) >= 600.0)));
    const bool ar = out.obs_term != nullptr && fin;
    evx_obs* obs_dst = ar ? out.obs_term : out.obs;
    // robot 0's observation is centred on Map.robot_position (view), the others on their own positions
    const uint32_t lid = st.layout_idx ? (uint32_t)st.layout_idx[e] : 0u;
#ifndef EVX_PROFILE
    EVX_STAMP(15);
#endif
    for (int r0 = 0; r0 < R; r0 += 16) write_obs16(g, rmapb, robots, view, r0, R, fs1, lid, obs_dst + (size_t)e * R);
#ifndef EVX_PROFILE
    EVX_STAMP(7);
#endif
    EVX_STAMP(8);
    if (ar) {
        __threadfence();  // this wave's state writes complete and visible before the reset reads them
        wave_sync();
        reset_one<BIGG>(lay, st, e, smem, out.obs, out.err);
    }
    EVX_RSTAMP(10);
}

// ------------------------------------------------------------------ reset
// One wave per env. People.__init__ placement (envs/people.py:183-194) is a
// sequential rejection sampler on the Python stream: x = randint(1, L-2),
// y = randint(1, W-2) (each _randbelow: top bit_length bits of a word, retried
// while >= the bound), retried while the cell is not valid. Over a window of 128
// stream words, lane j evaluates the attempt that would START at word B+j
// (acceptance masks by ballot, ctz jumps, word values by lane shuffle, validity
// from the bitmap) -> (end, success, cell). The wave then follows the chain of
// attempts from the stream head with readlanes: a few scalar ops per attempt.

// Reset of env e by the calling wave; smem: >= reset_lds(G, P, BIGG).total words.
template <bool BIGG>
__device__ __forceinline__ void reset_one(const evx_layout& lay, const evx_state& st, const int e, uint32_t* smem,
                                          evx_obs* obs, int32_t* err) {
    const int lane = (int)(threadIdx.x & 63);
    Geo g;
    g.L = lay.L; g.W = lay.W; g.GY = lay.W + 2; g.G = (lay.L + 2) * (lay.W + 2);
    g.RW = (g.G + 31) / 32; g.P = lay.P; g.R = lay.R;
    const int P = g.P, R = g.R;
    // fresh people: the light path's kept lists no longer describe this env
    if (lane == 0) st.scratch[(size_t)e * env_scratch_words(lay) + persist_offset(lay)] = 0u;
    const ResetLds S = reset_lds(g.G, P, BIGG);
    uint32_t* pyring = smem + S.pyring;
    const uint32_t* validb;
    uint32_t* rmapb = smem + S.rmapb;
    if constexpr (BIGG) {
        validb = lay.valid_bits;
        for (int i = lane; i < g.RW; i += 64) rmapb[i] = 0;
    } else {
        uint32_t* vb = smem + S.validb;
        for (int i = lane; i < g.RW; i += 64) {
            vb[i] = lay.valid_bits[i];
            rmapb[i] = 0;
        }
        validb = vb;
    }
    const uint32_t* gpy = st.py_mt + (size_t)e * EVX_MT_WORDS;
    for (int i = lane; i < MT_N; i += 64) pyring[i] = gpy[i];
    const int head0 = (int)gpy[MT_N];
    int py_front = MT_N;
    wave_fence();
#ifdef EVX_PROFILE
    long long tr0 = __builtin_amdgcn_s_memtime(), tw = 0, tc = 0, te = 0, tx;
    int nwin = 0;
#endif
    uint32_t* pk_o = st.pk + (size_t)e * P;
    double* h_o = st.health + (size_t)e * P;
    double* a_o = st.acc + (size_t)e * P;
    const uint32_t nx = (uint32_t)(g.L - 2), ny = (uint32_t)(g.W - 2);
    const int kx = bit_length(nx), ky = bit_length(ny);
    constexpr uint32_t UNKNOWN = 1u << 9, SUCC = 1u << 8;
    int pos = head0, placed = 0;
    int guard = 0;
    while (placed < P) {
        const int B = pos;
#ifdef EVX_PROFILE
        tx = __builtin_amdgcn_s_memtime();
#endif
        if (py_front < B + 128) mt_ensure_w(pyring, py_front, max(B + 128, py_front + MT_LAG));  // full rounds
#ifdef EVX_PROFILE
        te += __builtin_amdgcn_s_memtime() - tx;
        tx = __builtin_amdgcn_s_memtime();
        nwin++;
#endif
        const uint32_t t0 = mt_temper(pyring[(B + lane) & WRM]), t1 = mt_temper(pyring[(B + 64 + lane) & WRM]);
        const unsigned long long ax0 = __ballot((t0 >> (32 - kx)) < nx), ax1 = __ballot((t1 >> (32 - kx)) < nx);
        const unsigned long long ay0 = __ballot((t0 >> (32 - ky)) < ny), ay1 = __ballot((t1 >> (32 - ky)) < ny);
        // first set bit >= k of the 128-bit mask (m0, m1); 128 = none
        auto next_set = [](unsigned long long m0, unsigned long long m1, int k) -> int {
            if (k < 64) {
                const unsigned long long a = m0 >> k;
                if (a) return k + __builtin_ctzll(a);
                return m1 ? 64 + __builtin_ctzll(m1) : 128;
            }
            if (k >= 128) return 128;
            const unsigned long long b = m1 >> (k - 64);
            return b ? k + __builtin_ctzll(b) : 128;
        };
        uint32_t dend = UNKNOWN, dxy = 0;
        {
            const int jx = next_set(ax0, ax1, lane);
            const int jy = jx < 127 ? next_set(ay0, ay1, jx + 1) : 128;
            const uint32_t wx0 = __shfl(t0, jx & 63), wx1 = __shfl(t1, jx & 63);
            const uint32_t wy0 = __shfl(t0, jy & 63), wy1 = __shfl(t1, jy & 63);
            if (jy < 128) {
                const int x = 1 + (int)(((jx < 64) ? wx0 : wx1) >> (32 - kx));
                const int y = 1 + (int)(((jy < 64) ? wy0 : wy1) >> (32 - ky));
                dend = (uint32_t)(jy + 1) | (check_valid(g, validb, x, y) ? SUCC : 0u);
                dxy = (uint32_t)x | ((uint32_t)y << 12);
            }
        }
        // Follow the chain of attempts from lane 0. Almost every attempt is 2 words,
        // so the chain runs along one parity and only irregular attempts (other
        // lengths, or not evaluable in this window) need a scalar step.
#ifdef EVX_PROFILE
        tw += __builtin_amdgcn_s_memtime() - tx;
        tx = __builtin_amdgcn_s_memtime();
#endif
        const bool known = !(dend & UNKNOWN);
        const unsigned long long irr = __ballot(!known || (int)(dend & 0xffu) - lane != 2);
        constexpr unsigned long long EVEN = 0x5555555555555555ull;
        unsigned long long vis = 0;
        int rel = 0;
        while (rel < 64) {
            const unsigned long long par = (rel & 1) ? ~EVEN : EVEN;
            const unsigned long long from = par & (~0ull << rel);
            const unsigned long long cand = irr & from;
            if (!cand) {  // regular to the end of the window
                vis |= from;
                rel = ((63 - rel) & 1) ? 64 : 65;  // last visited 62 or 63, then +2
                break;
            }
            const int q = __builtin_ctzll(cand);
            vis |= from & ((1ull << q) - 1);
            const uint32_t de = (uint32_t)__builtin_amdgcn_readlane((int)dend, q);
            if (de & UNKNOWN) {
                rel = q;
                break;
            }
            vis |= 1ull << q;
            rel = (int)(de & 0xffu);
        }
        // emit the successful visited attempts in order; stop exactly at person P
        const bool emit = ((vis >> lane) & 1ull) && (dend & SUCC);
        const unsigned long long em = __ballot(emit);
        const int nem = __popcll(em);
        if (placed + nem >= P) {  // the P-th person ends this reset: its attempt's end is the stream head
            unsigned long long m2 = em;
            for (int t = 0; t < P - placed - 1; t++) m2 &= m2 - 1;
            const int last = __builtin_ctzll(m2);
            rel = (int)((uint32_t)__builtin_amdgcn_readlane((int)dend, last) & 0xffu);
        }
        const int k = placed + lanes_below(em);
        if (emit && k < P) {
            pk_o[k] = dxy;
            const int c = (int)(dxy & 0xfff) * g.GY + (int)((dxy >> 12) & 0xfff);
            atomicOr(&rmapb[c >> 5], 1u << (c & 31));
        }
        placed = min(P, placed + nem);
        pos = B + rel;
#ifdef EVX_PROFILE
        tc += __builtin_amdgcn_s_memtime() - tx;
#endif
        if (rel == 0) {  // an attempt longer than 128 words: cannot happen with a sane stream
            if (++guard > 4) {
                if (lane == 0 && err) atomicOr(err, 4);
                break;
            }
            pos = B + 64;
        }
    }
    for (int p = lane; p < P; p += 64) {
        h_o[p] = 100.0;
        a_o[p] = 0.0;
    }
    wave_sync();  // person words and rmap bits complete
    if (st.thmap) {
        int32_t* th = st.thmap + (size_t)e * g.G;
        for (int i = lane; i < g.G; i += 64) th[i] = (rmapb[i >> 5] >> (i & 31)) & 1u;
    }
    for (int i = lane; i < g.RW; i += 64) st.rmap[(size_t)e * g.RW + i] = rmapb[i];
    uint32_t view;
    if (lay.reset_robots) {
        for (int r = lane; r < R; r += 64)
            st.robots[(size_t)e * R + r] = rp_pack(lay.robot_init[2 * r], lay.robot_init[2 * r + 1]);
        view = rp_pack(lay.robot_init[0], lay.robot_init[1]);
    } else {
        view = rp_pack(lay.reset_view_x, lay.reset_view_y);
    }
    wave_sync();
    if (lane == 0) {
        st.view[e] = view;
        int* sg = st.scal + (size_t)e * 4;
        sg[1] = 0;
        sg[2] = 0;
        sg[3] = 0;
    }
    const int fs = st.scal[(size_t)e * 4];
    if (lane == 0 && st.perm_ws) st.perm_ws[e] = env_class(lay, fs, 0, 0);
    if (obs) {
        for (int r = 0; r < R; r++) {
            const uint32_t c = (r == 0) ? view : st.robots[(size_t)e * R + r];
            write_obs(g, validb, rmapb, rp_x(c), rp_y(c), fs, st.layout_idx ? (uint32_t)st.layout_idx[e] : 0u,
                      obs + (size_t)e * R + r);
        }
    }
    mt_store_w(pyring, py_front, pos, st.py_mt + (size_t)e * EVX_MT_WORDS);
#ifdef EVX_PROFILE
    if (lane == 0 && e == 0)
        printf("reset env0: total %lld cycles, windows %d, ensure %lld, window eval %lld, chain %lld, words %d\n",
               __builtin_amdgcn_s_memtime() - tr0, nwin, te, tw, tc, pos - head0);
#endif
}

// The layout of env e: the launch's own (MULTI == false), or its entry of the layout set,
// read through the constant address space (scalar loads, like the kernel argument's).
typedef __attribute__((address_space(4))) const evx_layout ConstLayout;
template <bool MULTI>
__device__ __forceinline__ const evx_layout& lay_of(const evx_layout& lay, const evx_state& st, int e) {
    if constexpr (MULTI) {
        const int li = __builtin_amdgcn_readfirstlane(st.layout_idx[e]);
        const ConstLayout* p = (const ConstLayout*)(reinterpret_cast<const evx_layout*>(lay.layout_set) + li);
        return *(const evx_layout*)p;
    } else {
        return lay;
    }
}

template <bool MULTI>
__global__ __launch_bounds__(64) void env_reset_kernel(evx_layout lay, evx_state st, const uint8_t* __restrict__ mask,
                                                       evx_obs* obs, int32_t* err) {
    const int e = blockIdx.x;
    if (mask && !mask[e]) return;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    reset_one(lay_of<MULTI>(lay, st, e), st, e, smem, obs, err);
}

// NWB waves per workgroup, one env per wave, no block barrier between envs, in the
// dispatch order evx_env_order chose (heavy envs first). With NWB == WNW the first H
// workgroups take one heavy env each (its rows phase on all waves); once the rows
// are done, waves 1.. of heavy workgroup b take the light envs at the tail of the
// order (3 per heavy env), the remaining envs go 4 per workgroup.
// pslots > 0: the launch ends with its heaviest envs, so their waves issue ahead of
// the light envs' waves sharing a SIMD (s_setprio): the heavy workgroups' waves while
// they work on their heavy env, and single-wave envs at order slots < H + pslots.
#ifndef EVX_ENV_MINW
#define EVX_ENV_MINW 3
#endif
// BIGG: big_grid layouts (target / contested / vacated bitmaps in global scratch, no heavy
// workgroups).
template <int NWB, bool MULTI, bool BIGG = false>
__global__ __launch_bounds__(64 * NWB, EVX_ENV_MINW) void env_step_kernel(evx_layout lay, evx_state st,
                                                            const int32_t* __restrict__ actions, evx_step_out out,
                                                            int hcap, int pslots, int part) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int w = (int)(threadIdx.x >> 6);
    const int words = step_lds_words(lay, BIGG);
    const int H = (NWB == WNW && st.order && hcap > 0) ? min(hcap, st.order[st.E]) : 0;
    // light envs order[H, E): the last nt of them go to the heavy workgroups' spare waves
    // (only when one launch steps them all: part 0). Each step_env variant has ONE call site:
    // every inlined copy of its body costs instruction-cache space.
    const int nt = part == 0 ? min((NWB - 1) * H, st.E - H) : 0;
    const bool heavy = !BIGG && part != 2 && (int)blockIdx.x < H;
    if (part == 1 && !heavy) return;  // heavy envs only
    int slot = -1;                    // this wave's light env slot in the order
    if constexpr (BIGG) {
    } else if (heavy) {
        const int e = st.order[blockIdx.x];
        if (pslots > 0) __builtin_amdgcn_s_setprio(2);
        if (w == 0) {
            step_env<true>(lay_of<MULTI>(lay, st, e), st, actions, out, e, smem);
        } else {
            __syncthreads();  // wave 0 has published the rows inputs
            rows_wide(lay_of<MULTI>(lay, st, e), st, e, smem);
            if (w == 1) wide_health_sum(lay_of<MULTI>(lay, st, e), st, e, smem);
            const int t = (int)blockIdx.x * (NWB - 1) + (w - 1);
            if (t < nt) slot = st.E - nt + t;
        }
        if (pslots > 0) __builtin_amdgcn_s_setprio(0);
    }
    if (!heavy) {
        slot = part == 2 ? H + (int)blockIdx.x * NWB + w : H + ((int)blockIdx.x - H) * NWB + w;
        if (slot >= (part == 2 ? st.E : st.E - nt)) {
            slot = -1;
        } else if (part != 2 && __builtin_amdgcn_readfirstlane(slot) < H + pslots) {
            // s_setprio ignores EXEC: the condition must be provably wave-uniform (readfirstlane)
            __builtin_amdgcn_s_setprio(1);
        }
    }
    if (slot < 0) return;
    const int e = st.order ? st.order[slot] : slot;
    step_env<false, BIGG>(lay_of<MULTI>(lay, st, e), st, actions, out, e, smem + (size_t)w * words);
}

// ------------------------------------------------------- dispatch order
// A step's cost grows with the persons still in play, and one env is one wave:
// the launch ends with its slowest env. Dispatching envs by descending remaining
// persons (16 buckets, stable counting sort in one workgroup) starts the heavy
// ones first so the light ones fill in around them.
// order[E] = H: the first H envs of the order (at most hcap, each with >= hmin persons
// in play) run their rows phase on a whole workgroup (rows_wide).
// Every env's bucket is read from the state ONCE, into LDS (bk[E]): with the lagged
// training schedule this kernel runs while an env.step may be updating the counters,
// and a bucket that changed between the counting and the ranking pass would break the
// permutation.
__global__ __launch_bounds__(1024) void env_order_kernel(evx_layout lay, evx_state st, int hcap, int hmin) {
    // wave w owns the contiguous slice [w * S, (w + 1) * S) of the envs, so a stable rank is
    // bucket start + the same-bucket envs of lower waves + those earlier in the wave's slice
    __shared__ int wcnt[16][16], woff[16][16], nheavy;
    extern __shared__ uint8_t bk[];  // [E] bucket (0 = most persons remaining)
    const int tid = threadIdx.x, E = st.E, P = lay.P;
    const int lane = tid & 63, w = tid >> 6;
    const int S = ((E + 16 * 64 - 1) / (16 * 64)) * 64;  // slice length, a multiple of 64
    if (tid < 256) wcnt[tid >> 4][tid & 15] = 0;
    if (tid == 0) nheavy = 0;
    __syncthreads();
    int nh = 0;
    uint32_t mycnt = 0;  // lane b < 16: this wave's count of bucket b
    // (prev_evacuated, prev_dead) of every env in one 8-byte load, up to 8 loads in flight
    constexpr int LPT = 8;
    for (int i0 = 0; i0 < S; i0 += LPT * 64) {
        unsigned long long v[LPT];
#pragma unroll
        for (int j = 0; j < LPT; j++) {
            const int i = i0 + j * 64 + lane, e = w * S + i;
            v[j] = (i < S && e < E) ? __hip_atomic_load(reinterpret_cast<const unsigned long long*>(st.scal + (size_t)e * 4 + 2),
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                    : 0ull;
        }
#pragma unroll
        for (int j = 0; j < LPT; j++) {
            const int i = i0 + j * 64 + lane, e = w * S + i;
            int b = -1;
            if (i < S && e < E) {
                const int rem = P - (int)(uint32_t)v[j] - (int)(uint32_t)(v[j] >> 32);
                b = 15 - min(15, max(0, rem) * 16 / (P + 1));
                bk[e] = (uint8_t)b;
                nh += rem >= hmin;
            }
            if (__ballot(b >= 0)) {
#pragma unroll
                for (int bb = 0; bb < 16; bb++) {
                    const uint32_t c = (uint32_t)__popcll(__ballot(b == bb));
                    mycnt += lane == bb ? c : 0u;
                }
            }
        }
    }
    if (lane < 16) wcnt[w][lane] = (int)mycnt;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) nh += __shfl_xor(nh, o, 64);
    if (lane == 0 && nh) atomicAdd(&nheavy, nh);
    __syncthreads();
    if (tid < 16) {  // bucket tid: start of every wave's run
        int below = 0;
        for (int b = 0; b < tid; b++)
            for (int ww = 0; ww < 16; ww++) below += wcnt[ww][b];
        for (int ww = 0; ww < 16; ww++) {
            woff[ww][tid] = below;
            below += wcnt[ww][tid];
        }
    }
    if (tid == 0) st.order[E] = min(hcap, nheavy);
    __syncthreads();
    int run = lane < 16 ? woff[w][lane] : 0;  // lane b < 16: next rank of bucket b in this wave
    for (int i0 = 0; i0 < S; i0 += 64) {
        const int i = i0 + lane, e = w * S + i;
        const int b = e < E ? (int)bk[e] : -1;
        if (!__ballot(b >= 0)) break;
#pragma unroll
        for (int bb = 0; bb < 16; bb++) {
            const unsigned long long m = __ballot(b == bb);
            const int r0 = __shfl(run, bb, 64);
            if (b == bb)
                st.order[r0 + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = e;
            run += lane == bb ? __popcll(m) : 0;
        }
    }
}

// ------------------------------------------------------- act permutation
// The two scheduling permutations (results never depend on them) from one class byte per env
// (evx_state.perm_ws): bits 0-3 the bucket of persons remaining (0 = most), bit 4 fire step >=
// t_max (the x3 act's table path), bit 5 heavy (>= P/4 persons remaining). The step and reset
// kernels write an env's byte as they finish with it, so the orders of the next step need no pass
// over the state (evx_env_classes rewrites every byte from the state words, for states written
// from the host).
// Each env's byte is computed against its own layout (a layout set: its entry), as the step and
// reset kernels write it.
__global__ __launch_bounds__(256) void env_classes_kernel(evx_layout lay, evx_state st) {
    const int e = (int)blockIdx.x * 256 + (int)threadIdx.x;
    if (e >= st.E) return;
    const int4 v = *reinterpret_cast<const int4*>(st.scal + (size_t)e * 4);
    const evx_layout* le = &lay;
    if (lay.layout_set && st.layout_idx) le = reinterpret_cast<const evx_layout*>(lay.layout_set) + st.layout_idx[e];
    st.perm_ws[e] = env_class(*le, v.x, v.z, v.w);
}
// One launch, workgroup c ranking the envs [1024 c, 1024 c + 1024) (stable: env order within a
// class):
//   order[0, E): the envs by bucket (most persons remaining first), order[E] = min(hcap, heavy);
//   perm[0, E): the envs at fire step >= t_max first, then the rest.
// Either output may be NULL. The class bytes are read more than once (the counts, then the ranks):
// this launch must not overlap a step or reset of the same envs (VecEnv.compute_order(ahead=True)
// runs env_order_kernel instead, which reads each env's counters once). Every workgroup counts the classes of all E envs (one byte each, L2)
// itself -- the totals set where each class starts, the chunks before c where this chunk's run of
// it starts -- so no second launch or workspace carries counts between workgroups. Per 64 envs a
// wave takes 7 ballots (4 bucket bits, valid, fire, heavy); lane k < 16 counts bucket k as the AND
// of the bit ballots that match k. Slots: 0-15 buckets, 16 fire class, 17 heavy, 18 valid.
constexpr int OSL = 19;
__device__ __forceinline__ unsigned long long bucket_eq(int k, const unsigned long long (&m)[4], unsigned long long v) {
#pragma unroll
    for (int j = 0; j < 4; j++) v &= ((k >> j) & 1) ? m[j] : ~m[j];
    return v;
}
// NW waves per workgroup, 64 NW envs ranked per workgroup (blk): env_orders_kernel and the orders
// blocks of env_orders_push_kernel (NW 16; smaller workgroups straddle the 1024-env scan chunks).
template <bool V16, int NW>  // V16: cls 16-B aligned -- the scan reads 16 class bytes per lane
__device__ __forceinline__ void orders_body(const uint8_t* __restrict__ cls, int E, int hcap, int32_t* __restrict__ order,
                                            int32_t* __restrict__ perm, int blk) {
    __shared__ int wt[NW][OSL], wp[NW][OSL], wc[NW][OSL];
    const int tid = (int)threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c0 = blk * 64 * NW;
    auto ballots = [&](int b, unsigned long long (&m)[4], unsigned long long& mv, unsigned long long& mf,
                       unsigned long long& mh) {
        mv = __ballot(b >= 0);
#pragma unroll
        for (int j = 0; j < 4; j++) m[j] = __ballot(b >= 0 && ((b >> j) & 1));
        mf = __ballot(b >= 0 && (b & 0x10));
        mh = __ballot(b >= 0 && (b & 0x20));
    };
    auto slot_count = [&](const unsigned long long (&m)[4], unsigned long long mv, unsigned long long mf,
                          unsigned long long mh) -> int {  // lane k < OSL: this block's count of slot k
        const int k = lane < 16 ? lane : 0;
        const unsigned long long sel = lane < 16 ? bucket_eq(k, m, mv) : lane == 16 ? mf : lane == 17 ? mh : mv;
        return lane < OSL ? __popcll(sel) : 0;
    };
    // every class byte of the launch: totals (t) and the envs before this workgroup's (pr)
    int t = 0, pr = 0;
    if constexpr (V16) {
        // wave w reads the 1024-env chunks w, w + NW, ..: lane l holds envs 16 l .. 16 l + 15 of one,
        // two chunks' loads in flight before either is counted (byte j of every lane: one ballot set)
        for (int q0 = w; q0 * 1024 < E; q0 += 2 * NW) {
            uint4 v[2];
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int e0 = (q0 + NW * i) * 1024 + 16 * lane;
                v[i] = make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);
                if (e0 < E) v[i] = *reinterpret_cast<const uint4*>(cls + e0);
            }
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int q = q0 + NW * i, e0 = q * 1024 + 16 * lane;
                const uint32_t wd[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
                // a chunk that straddles c0 (NW < 16) counts its envs below c0 separately
                const bool split = q * 1024 < c0 && c0 < q * 1024 + 1024;
                int n = 0, nb = 0;
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    const int b = e0 + j < E ? (int)((wd[j >> 2] >> (8 * (j & 3))) & 0xffu) : -1;
                    unsigned long long m[4], mv, mf, mh;
                    ballots(b, m, mv, mf, mh);
                    n += slot_count(m, mv, mf, mh);
                    if (split) {
                        ballots(e0 + j < c0 ? b : -1, m, mv, mf, mh);
                        nb += slot_count(m, mv, mf, mh);
                    }
                }
                t += n;
                pr += q * 1024 + 1024 <= c0 ? n : nb;
            }
        }
    } else {
        const int nb = (E + 63) / 64;
#pragma unroll 4
        for (int bk = w; bk < nb; bk += NW) {
            const int e = bk * 64 + lane;
            const int b = e < E ? (int)cls[e] : -1;
            unsigned long long m[4], mv, mf, mh;
            ballots(b, m, mv, mf, mh);
            const int n = slot_count(m, mv, mf, mh);
            t += n;
            pr += bk * 64 < c0 ? n : 0;
        }
    }
    if (lane < OSL) {
        wt[w][lane] = t;
        wp[w][lane] = pr;
    }
    // this workgroup's envs: the waves' counts (for the ranks across waves) and the in-wave masks
    const int e = c0 + tid;
    const int b = e < E ? (int)cls[e] : -1;
    unsigned long long m[4], mv, mf, mh;
    ballots(b, m, mv, mf, mh);
    const int n = slot_count(m, mv, mf, mh);
    if (lane < OSL) wc[w][lane] = n;
    __syncthreads();
    if (tid < OSL) {  // totals and prefix over the waves' partial counts (into wt[0], wp[0])
        int st = 0, sp = 0;
        for (int k = 0; k < NW; k++) {
            st += wt[k][tid];
            sp += wp[k][tid];
        }
        wt[0][tid] = st;
        wp[0][tid] = sp;
    }
    __syncthreads();
    if (b < 0) return;
    const unsigned long long lt = (1ull << lane) - 1ull;
    if (order) {
        const int bk = b & 15;
        int base = wp[0][bk];
        for (int k = 0; k < bk; k++) base += wt[0][k];
        for (int k = 0; k < w; k++) base += wc[k][bk];
        order[base + __popcll(bucket_eq(bk, m, mv) & lt)] = e;
        if (e == 0) order[E] = min(hcap, wt[0][17]);
    }
    if (perm) {
        const bool f = (b & 0x10) != 0;
        int base;
        if (f) {
            base = wp[0][16];
            for (int k = 0; k < w; k++) base += wc[k][16];
            base += __popcll(mf & lt);
        } else {  // after every fire-class env: the non-fire envs before this one
            base = wt[0][16] + (wp[0][18] - wp[0][16]);
            for (int k = 0; k < w; k++) base += wc[k][18] - wc[k][16];
            base += __popcll(mv & ~mf & lt);
        }
        perm[base] = e;
    }
}
template <bool V16>
__global__ __launch_bounds__(1024) void env_orders_kernel(const uint8_t* __restrict__ cls, int E, int hcap,
                                                          int32_t* __restrict__ order, int32_t* __restrict__ perm) {
    orders_body<V16, 16>(cls, E, hcap, order, perm, (int)blockIdx.x);
}
// DQNAgent.remember for every robot of the step (the replay push: evxq::replay_push_kernel's body)
// and the next step's orders in one launch: workgroups [0, nord) the orders (1024 envs each), the
// rest one transition per thread -- the orders then need no launch or cross-stream event of their
// own, and run beside the push's memory traffic. (256-env order workgroups of 4 waves, each
// scanning every class byte, made the launch 32 us.)
struct PushArgs {
    evx_replay rp;
    const evx_obs *s, *s2, *s2_term;
    const int32_t* a;
    const double* r_env;
    const uint8_t* done_env;
    int n, agents_per_env;
    int64_t pos;
};
// the learn step's batch drawn in the same launch (evx_replay_sample's draws over the ring as it
// stands after the push: a drawn slot inside the push window is read from the push's sources)
struct SampleArgs {
    int64_t size;  // ring size after the push
    int B;
    uint64_t seed, offset;
    evx_obs *s, *s2;
    int32_t* a;
    float* r;
    uint8_t* done;
};
template <bool V16>
__global__ __launch_bounds__(1024) void env_orders_push_kernel(const uint8_t* __restrict__ cls, int E, int hcap,
                                                               int32_t* __restrict__ order, int32_t* __restrict__ perm,
                                                               int nord, int nsmp, PushArgs pa, SampleArgs sa) {
    const int64_t cm = pa.rp.capacity - 1;  // power-of-two capacity (host-checked)
    if ((int)blockIdx.x < nsmp) {  // 256 draws per workgroup: the dependent draw-and-gather chains
                                   // spread over 4x the CUs (the other 12 waves leave at once)
        if (threadIdx.x >= 256) return;
        const int i = (int)blockIdx.x * 256 + (int)threadIdx.x;
        if (i >= sa.B) return;
        const evxd::perm_key pk = evxd::make_perm_key((uint64_t)sa.size, sa.seed, sa.offset, 0u);
        const int64_t j = (int64_t)evxd::perm_apply(pk, (uint64_t)i, (uint64_t)sa.size);  // base 0: the whole ring
        const int64_t off = (j - pa.pos) & cm;
        if (off < pa.n) {  // written by this launch's push: its source
            const int k = (int)off, e = k / pa.agents_per_env;
            sa.s[i] = pa.s[k];
            sa.s2[i] = (pa.s2_term && pa.done_env[e]) ? pa.s2_term[k] : pa.s2[k];
            sa.a[i] = pa.a[k];
            sa.r[i] = (float)pa.r_env[e];
            sa.done[i] = pa.done_env[e];
        } else {
            sa.s[i] = pa.rp.s[j];
            sa.s2[i] = pa.rp.s2[j];
            sa.a[i] = pa.rp.a[j];
            sa.r[i] = pa.rp.r[j];
            sa.done[i] = pa.rp.done[j];
        }
        return;
    }
    if ((int)blockIdx.x < nsmp + nord) {
        orders_body<V16, 16>(cls, E, hcap, order, perm, (int)blockIdx.x - nsmp);
        return;
    }
    const int i = ((int)blockIdx.x - nord - nsmp) * 1024 + (int)threadIdx.x;
    if (i >= pa.n) return;
    const int64_t slot = (pa.pos + i) & cm;
    const int e = i / pa.agents_per_env;
    pa.rp.s[slot] = pa.s[i];
    pa.rp.s2[slot] = (pa.s2_term && pa.done_env[e]) ? pa.s2_term[i] : pa.s2[i];
    pa.rp.a[slot] = pa.a[i];
    pa.rp.r[slot] = (float)pa.r_env[e];
    pa.rp.done[slot] = pa.done_env[e];
}

// ---------------------------------------------------- observation expand
// EvacuationEnv._get_state (envs/evacuation_env.py:84-120) from the compact form.
template <typename T>
__global__ __launch_bounds__(256) void obs_expand_kernel(evx_layout lay0, const evx_obs* __restrict__ obs, int64_t n,
                                                         T* __restrict__ out) {
    // one thread per (row, window cell): the cell's six channels from one observation load and one
    // cellinfo load, written as 6 consecutive values (was one thread per value)
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= n * 121) return;
    const int64_t o = gid / 121;
    const int c = (int)(gid - o * 121);
    const int i = c / 11, j = c - i * 11;
    const evx_obs ob = obs[o];
    const evx_layout& lay = lay0.layout_set ? reinterpret_cast<const evx_layout*>(lay0.layout_set)[ob.layout] : lay0;
    const int mx = ob.cx + i - 5, my = ob.cy + j - 5;
    const int GY = lay.W + 2;
    const bool inb = mx >= 0 && mx <= lay.L + 1 && my >= 0 && my <= lay.W + 1;
    const uint8_t ci = inb ? lay.cellinfo[mx * GY + my] : (uint8_t)0;
    const bool valid = mx >= 1 && mx <= lay.L && my >= 1 && my <= lay.W && (ci & 1u);
    T v[6];
    v[0] = 0;
    v[1] = ((ob.occ[c >> 5] >> (c & 31)) & 1u) ? (T)1 : (T)0;
    v[2] = 0;
    const int ti = mx - lay.ox0, tj = my - lay.oy0;
    if (ti >= 0 && ti < lay.OX && tj >= 0 && tj < lay.OY) {
        const size_t idx = ((size_t)ob.fire_step * lay.OX + ti) * lay.OY + tj;
        if constexpr (sizeof(T) == 8) v[2] = (T)lay.danger_o[idx];
        else v[2] = (T)lay.danger_o32[idx];
    }
    v[3] = (!valid || (inb && ((ci >> 2) & 1u))) ? (T)1 : (T)0;
    v[4] = (mx == lay.exit_x && my == lay.exit_y) ? (T)1 : (T)0;
    v[5] = (i == 5 && j == 5) ? (T)1 : (T)0;
    T* dst = out + o * 726 + c * 6;
#pragma unroll
    for (int ch = 0; ch < 6; ch++) dst[ch] = v[ch];
}

}  // namespace evx

// ===================================================================== C-ABI
// the step kernel's dynamic LDS also hosts a fused auto-reset
static size_t step_lds_bytes(const evx_layout& l, bool bigg = false) {
    return (size_t)evx::step_lds_words(l, bigg) * 4;
}
// dynamic LDS of a step workgroup of nwb waves: nwb envs, or (nwb == 4) one heavy env
static size_t step_launch_lds(const evx_layout& l, int nwb, bool bigg = false) {
    if (bigg || nwb != evx::WNW) return step_lds_bytes(l, bigg) * nwb;
    return (size_t)evx::wide_lds(l).total * 4;  // WNW env regions + WideCtl
}
// Heavy envs per step (rows_wide workgroups): at most the cap, each with >= *hmin
// persons in play; 0 when the 4-wave workgroup does not fit in LDS. EVX_HEAVY_CAP /
// EVX_HEAVY_MIN override (tuning). Cap 176 (tools/tune_heavy_train.sh, tune_heavy_cfgs.sh):
// with 256 heavy workgroups (one per CU) the light envs' waves start late; 160-192 is a
// plateau in the training step (cfg3 lagged 9.63 -> 10.07 M, strict 7.44 -> 7.75 M,
// env-only 13.3 -> 13.9 M, cfg2 17.9 -> 18.3 M, cfg5 8.72 -> 8.88 M env-steps/s).
static int heavy_cap(const evx_layout& l, int* hmin) {
    *hmin = std::max(1, l.P / 4);
    if (evx::big_grid(l.L, l.W)) return 0;  // BIGG kernels: no heavy workgroups
    const evx::WideLds wl = evx::wide_lds(l);
    if (step_launch_lds(l, evx::WNW) > 160 * 1024 || wl.end > wl.ctl) return 0;
    static const int cap_env = [] {
        const char* v = getenv("EVX_HEAVY_CAP");
        return v ? atoi(v) : -1;
    }();
    static const int min_env = [] {
        const char* v = getenv("EVX_HEAVY_MIN");
        return v ? atoi(v) : -1;
    }();
    if (min_env > 0) *hmin = min_env;
    return cap_env >= 0 ? cap_env : 176;
}

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
    return (int64_t)step_lds_bytes(*l, evx::big_grid(l->L, l->W));
}

int64_t evx_step_scratch_words(const evx_layout* l) {
    if (check_layout(l)) return -1;
    return evx::env_scratch_words(*l);
}

int evx_env_step(const evx_layout* l, const evx_state* s, const int32_t* actions, const evx_step_out* o, void* stream) {
    return evx_env_step_part(l, s, actions, o, 0, stream);
}

int evx_env_step_part(const evx_layout* l, const evx_state* s, const int32_t* actions, const evx_step_out* o,
                      int32_t part, void* stream) {
    if (part < 0 || part > 2) return fail(-22, "env_step: part must be 0, 1 or 2");
    int rc = check_layout(l);
    if (rc) return rc;
    if (!s || !o || !actions || !o->reward || !o->done || !o->obs) return fail(-22, "NULL argument");
    if (!s->scratch) return fail(-22, "state scratch is NULL (evx_step_scratch_words per env)");
    if (!l->nbr_valid || !l->floor_d5) return fail(-22, "missing table nbr_valid / floor_d5");
    if (s->E <= 0) return 0;
    const int G = (l->L + 2) * (l->W + 2);
    {  // contested-list keys are (target << bits(P-1)) | person in 32 bits
        int pb = 1, gb = 1;
        while ((1 << pb) < l->P) pb++;
        while ((1LL << gb) < (long long)G) gb++;
        if (pb + gb > 32) return fail(-22, "grid cells x people too large for 32-bit move keys");
    }
    const bool bigg = evx::big_grid(l->L, l->W);
    const size_t lds = step_lds_bytes(*l, bigg);
    if (lds > 160 * 1024) return fail(-7, "layout needs more than 160 KiB of LDS");
    const bool multi = l->layout_set && s->layout_idx;
    {
        static std::atomic<uint64_t> attr_done;
        const void* ks[10] = {(const void*)evx::env_step_kernel<1, false>, (const void*)evx::env_step_kernel<2, false>,
                              (const void*)evx::env_step_kernel<4, false>, (const void*)evx::env_step_kernel<1, true>,
                              (const void*)evx::env_step_kernel<2, true>, (const void*)evx::env_step_kernel<4, true>,
                              (const void*)evx::env_step_kernel<1, false, true>,
                              (const void*)evx::env_step_kernel<2, false, true>,
                              (const void*)evx::env_step_kernel<1, true, true>,
                              (const void*)evx::env_step_kernel<2, true, true>};
        evxh::max_lds_once(attr_done, ks, 10, 160 * 1024);
    }
    // Default: 4-wave workgroups with the heavy-env path while a launch is short enough for
    // its heaviest env to set its length (fewer than 64 envs per CU); one-wave workgroups
    // beyond, where throughput rules: a wave's VGPRs and LDS free the moment its env is done
    // instead of when the slowest of four is (32768 envs: env_step 1.50 -> 1.31 ms).
    const int ncu = evxh::cu_count();
    // (64 envs per CU: the 8192-env share of cfg5 keeps the heavy-env workgroups -- env_step 0.42 ->
    // 0.37 ms; big grids, which have no heavy path, switch at 32)
    int nwb = s->E >= (bigg ? 32 : 64) * ncu ? 1 : 4;
    if (bigg && nwb > 2) nwb = 2;  // BIGG kernels: 1 or 2 envs per workgroup
    while (nwb > 1 && step_launch_lds(*l, nwb, bigg) > 160 * 1024) nwb >>= 1;
    int hmin = 0;
    const int hcap = (nwb == evx::WNW && s->order) ? heavy_cap(*l, &hmin) : 0;
    // single-wave envs at order slots < H + pslots could run at raised wave priority: 0 (a sweep
    // of 0 / 1 / 256 / 768 / 1536 slots measured box noise in the training step)
    const int pslots = 0;
    const size_t blds = step_launch_lds(*l, nwb, bigg);
    // heavy envs take a workgroup each; part 1: only those, part 2: only the rest
    if (part == 1 && hcap == 0) return 0;  // no heavy workgroups for this layout: part 2 steps every env
    const int nblk = part == 1 ? hcap : (s->E + nwb - 1) / nwb + (part == 0 ? hcap : 0);
    hipStream_t hs = (hipStream_t)stream;
    if (bigg) {
        if (nwb == 2 && multi)
            hipLaunchKernelGGL((evx::env_step_kernel<2, true, true>), dim3(nblk), dim3(128), blds, hs, *l, *s, actions,
                               *o, 0, 0, (int)part);
        else if (nwb == 2)
            hipLaunchKernelGGL((evx::env_step_kernel<2, false, true>), dim3(nblk), dim3(128), blds, hs, *l, *s, actions,
                               *o, 0, 0, (int)part);
        else if (multi)
            hipLaunchKernelGGL((evx::env_step_kernel<1, true, true>), dim3(nblk), dim3(64), blds, hs, *l, *s, actions,
                               *o, 0, 0, (int)part);
        else
            hipLaunchKernelGGL((evx::env_step_kernel<1, false, true>), dim3(nblk), dim3(64), blds, hs, *l, *s, actions,
                               *o, 0, 0, (int)part);
    } else if (nwb == 4 && multi)
        hipLaunchKernelGGL((evx::env_step_kernel<4, true>), dim3(nblk), dim3(256), blds, hs, *l, *s, actions, *o, hcap,
                           pslots, (int)part);
    else if (nwb == 4)
        hipLaunchKernelGGL((evx::env_step_kernel<4, false>), dim3(nblk), dim3(256), blds, hs, *l, *s, actions, *o, hcap,
                           pslots, (int)part);
    else if (nwb == 2 && multi)
        hipLaunchKernelGGL((evx::env_step_kernel<2, true>), dim3(nblk), dim3(128), blds, hs, *l, *s, actions, *o, 0, 0,
                           (int)part);
    else if (nwb == 2)
        hipLaunchKernelGGL((evx::env_step_kernel<2, false>), dim3(nblk), dim3(128), blds, hs, *l, *s, actions, *o, 0, 0,
                           (int)part);
    else if (multi)
        hipLaunchKernelGGL((evx::env_step_kernel<1, true>), dim3(nblk), dim3(64), blds, hs, *l, *s, actions, *o, 0, 0,
                           (int)part);
    else
        hipLaunchKernelGGL((evx::env_step_kernel<1, false>), dim3(nblk), dim3(64), blds, hs, *l, *s, actions, *o, 0, 0,
                           (int)part);
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
    {
        static std::atomic<uint64_t> attr_done;
        const void* ks[2] = {(const void*)evx::env_reset_kernel<false>, (const void*)evx::env_reset_kernel<true>};
        evxh::max_lds_once(attr_done, ks, 2, 160 * 1024);
    }
    if (l->layout_set && s->layout_idx)
        hipLaunchKernelGGL(evx::env_reset_kernel<true>, dim3(s->E), dim3(64), lds, (hipStream_t)stream, *l, *s, mask,
                           obs, err);
    else
        hipLaunchKernelGGL(evx::env_reset_kernel<false>, dim3(s->E), dim3(64), lds, (hipStream_t)stream, *l, *s, mask,
                           obs, err);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "env_reset launch");
}

// The scheduling permutations' workspace in evx_state.perm_ws: the class byte of every env.
static int64_t perm_ws_need(int64_t E) { return (E + 255) / 256 * 256; }
constexpr int ORDERS_MAX_E = 160 * 1024 - 4096;  // env_order_kernel's LDS (no workspace): one byte per env

namespace evx {
// diagnostic / test entry (evx_diag_sort_keys): one wave sorts n distinct keys in place in global
// memory with the contested list's sort (wave_sort_keys), padding to a power of two in pad[]
__global__ __launch_bounds__(64) void diag_sort_kernel(uint32_t* keys, uint32_t* pad, int n) {
    const int lane = (int)threadIdx.x;
    const int n2 = pow2_ceil(n);
    for (int i = lane; i < n2; i += 64) pad[i] = i < n ? keys[i] : 0xffffffffu;
    wave_sync();
    wave_sort_keys(pad, n, n2);
    for (int i = lane; i < n; i += 64) keys[i] = pad[i];
}
}  // namespace evx
int evx_diag_sort_keys(uint32_t* keys, uint32_t* pad, int32_t n, void* stream) {
    if (!keys || !pad || n < 0) return fail(-22, "diag_sort_keys: bad argument");
    if (n == 0) return 0;
    hipLaunchKernelGGL(evx::diag_sort_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, keys, pad, n);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "diag_sort_keys launch");
}

static int launch_orders(const evx_layout* l, const evx_state* s, int32_t* order, int32_t* perm, hipStream_t st) {
    int hmin = 0;
    const int hcap = heavy_cap(*l, &hmin);
    const dim3 grid((unsigned)((s->E + 1023) / 1024));
    if (((uintptr_t)s->perm_ws & 15) == 0)
        hipLaunchKernelGGL(evx::env_orders_kernel<true>, grid, dim3(1024), 0, st, (const uint8_t*)s->perm_ws, s->E,
                           hcap, order, perm);
    else  // a part's slice of the class bytes at an unaligned offset
        hipLaunchKernelGGL(evx::env_orders_kernel<false>, grid, dim3(1024), 0, st, (const uint8_t*)s->perm_ws, s->E,
                           hcap, order, perm);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "env_orders launch");
}

int evx_env_order(const evx_layout* l, const evx_state* s, void* stream) {
    int rc = check_layout(l);
    if (rc) return rc;
    if (!s || !s->order) return fail(-22, "env_order: state.order is NULL");
    if (s->E <= 0) return 0;
    if (s->perm_ws) return launch_orders(l, s, s->order, nullptr, (hipStream_t)stream);
    if (s->E > ORDERS_MAX_E) return fail(-22, "env_order: too many envs for one workgroup's LDS");
    // no workspace: the one-workgroup kernel reads every env's counters from the state
    int hmin = 0;
    const int hcap = heavy_cap(*l, &hmin);
    {
        static std::atomic<uint64_t> attr_done;
        const void* ks[1] = {(const void*)evx::env_order_kernel};
        evxh::max_lds_once(attr_done, ks, 1, ORDERS_MAX_E);
    }
    const size_t lds = ((size_t)s->E + 3) & ~(size_t)3;  // one bucket byte per env
    hipLaunchKernelGGL(evx::env_order_kernel, dim3(1), dim3(1024), lds, (hipStream_t)stream, *l, *s, hcap, hmin);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "env_order launch");
}

int64_t evx_perm_ws_bytes(int32_t E) { return E > 0 ? perm_ws_need(E) : 0; }

int evx_act_perm(const evx_layout* l, const evx_state* s, int32_t* perm, void* stream) {
    int rc = check_layout(l);
    if (rc) return rc;
    if (!s || !perm) return fail(-22, "act_perm: NULL argument");
    if (s->E <= 0) return 0;
    if (!s->perm_ws) return fail(-22, "act_perm: state.perm_ws is NULL (evx_perm_ws_bytes(E) bytes)");
    return launch_orders(l, s, nullptr, perm, (hipStream_t)stream);
}

int evx_env_orders(const evx_layout* l, const evx_state* s, int32_t* perm, void* stream) {
    int rc = check_layout(l);
    if (rc) return rc;
    if (!s || !s->order || !s->perm_ws) return fail(-22, "env_orders: state.order / state.perm_ws is NULL");
    if (s->E <= 0) return 0;
    return launch_orders(l, s, s->order, perm, (hipStream_t)stream);
}

int evx_env_orders_push(const evx_layout* l, const evx_state* s, int32_t* perm, const evx_replay* rp,
                        const evx_obs* s_obs, const evx_obs* s2, const evx_obs* s2_term, const int32_t* a,
                        const double* r_env, const uint8_t* done_env, int32_t n, int32_t agents_per_env, int64_t pos,
                        void* stream) {
    return evx_env_orders_push_sample(l, s, perm, rp, s_obs, s2, s2_term, a, r_env, done_env, n, agents_per_env, pos,
                                      0, 0, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
}

int evx_env_orders_push_sample(const evx_layout* l, const evx_state* s, int32_t* perm, const evx_replay* rp,
                               const evx_obs* s_obs, const evx_obs* s2, const evx_obs* s2_term, const int32_t* a,
                               const double* r_env, const uint8_t* done_env, int32_t n, int32_t agents_per_env,
                               int64_t pos, int32_t B, int64_t size, uint64_t seed, uint64_t offset, evx_obs* out_s,
                               evx_obs* out_s2, int32_t* out_a, float* out_r, uint8_t* out_done, void* stream) {
    if (B > 0) {
        if (!rp || size <= 0 || size > rp->capacity) return fail(-22, "env_orders_push_sample: bad ring size");
        if (B > size) return fail(-22, "env_orders_push_sample: sample larger than population (random.sample)");
        if (!out_s || !out_s2 || !out_a || !out_r || !out_done) return fail(-22, "env_orders_push_sample: NULL output");
        if (pos < 0 || n > rp->capacity) return fail(-22, "env_orders_push_sample: bad push window");
    }
    int rc = check_layout(l);
    if (rc) return rc;
    if (!s || !s->order || !s->perm_ws) return fail(-22, "env_orders_push: state.order / state.perm_ws is NULL");
    if (!rp || rp->capacity <= 0 || (rp->capacity & (rp->capacity - 1)))
        return fail(-22, "env_orders_push: replay capacity must be a power of two");
    if (n < 0 || agents_per_env <= 0 || (n > 0 && (!s_obs || !s2 || !a || !r_env || !done_env)))
        return fail(-22, "env_orders_push: bad push arguments");
    int hmin = 0;
    const int hcap = heavy_cap(*l, &hmin);
    const int nord = s->E > 0 ? (s->E + 1023) / 1024 : 0;
    const int nsmp = B > 0 ? (B + 255) / 256 : 0;
    const unsigned nblk = (unsigned)(nord + nsmp + (n + 1023) / 1024);
    if (nblk == 0) return 0;
    evx::PushArgs pa{*rp, s_obs, s2, s2_term, a, r_env, done_env, n, agents_per_env, pos & (rp->capacity - 1)};
    evx::SampleArgs sa{size, B, seed, offset, out_s, out_s2, out_a, out_r, out_done};
    if (((uintptr_t)s->perm_ws & 15) == 0)
        hipLaunchKernelGGL(evx::env_orders_push_kernel<true>, dim3(nblk), dim3(1024), 0, (hipStream_t)stream,
                           (const uint8_t*)s->perm_ws, s->E, hcap, s->order, perm, nord, nsmp, pa, sa);
    else
        hipLaunchKernelGGL(evx::env_orders_push_kernel<false>, dim3(nblk), dim3(1024), 0, (hipStream_t)stream,
                           (const uint8_t*)s->perm_ws, s->E, hcap, s->order, perm, nord, nsmp, pa, sa);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "env_orders_push launch");
}

int evx_env_classes(const evx_layout* l, const evx_state* s, void* stream) {
    int rc = check_layout(l);
    if (rc) return rc;
    if (!s || !s->scal || !s->perm_ws) return fail(-22, "env_classes: state.scal / state.perm_ws is NULL");
    if (s->E <= 0) return 0;
    hipLaunchKernelGGL(evx::env_classes_kernel, dim3((unsigned)((s->E + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       *l, *s);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "env_classes launch");
}

int evx_obs_expand_f32(const evx_layout* l, const evx_obs* obs, int64_t n, float* out, void* stream) {
    int rc = check_layout(l);
    if (rc) return rc;
    if (!l->danger_o32) return fail(-22, "danger_o32 missing");
    if (n <= 0) return 0;
    const int64_t total = n * 726;
    hipLaunchKernelGGL(evx::obs_expand_kernel<float>, dim3((unsigned)((total / 6 + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, *l, obs, n, out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "obs_expand launch");
}

int evx_obs_expand_f64(const evx_layout* l, const evx_obs* obs, int64_t n, double* out, void* stream) {
    int rc = check_layout(l);
    if (rc) return rc;
    if (n <= 0) return 0;
    const int64_t total = n * 726;
    hipLaunchKernelGGL(evx::obs_expand_kernel<double>, dim3((unsigned)((total / 6 + 255) / 256)), dim3(256), 0,
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
