/* evacx -- C-ABI of the MI355X-native evacuation CA + DQN hot path (libevacx.so).
 *
 * The reference (LX-530/DQN-MARL, Louvre_Evacuation/) has no FFI: its boundary
 * is the duck-typed Python API its runners call. Each entry point below names
 * the reference function it replaces (paths relative to
 * /root/reference/Louvre_Evacuation/); the Python mirror in
 * dqn-marl_amd/Louvre_Evacuation binds them through ctypes.
 *
 * Conventions
 *  - every call returns 0 or a negative errno-like code; evx_last_error() has text;
 *  - every buffer is caller-owned DEVICE memory unless the name says _host;
 *  - no hidden allocations, no internal threads, no host syncs; `stream` is a
 *    hipStream_t passed as void* (0 = the null stream);
 *  - plain pointers and sizes only (no torch types).
 */
#ifndef EVACX_H
#define EVACX_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EVX_MT_WORDS 625 /* 624 MT19937 words + index, CPython/numpy layout */
#define EVX_OBS_CELLS 121
#define EVX_OBS_CH 6

/* Static, read-only description of one layout (device tables built on the host
 * by evacx/layout.py: Map.__init__ + Init_Potential envs/map.py:38-148,
 * ProgressiveFireModel envs/fire_model.py:4-199). */
typedef struct {
    int32_t L, W;             /* interior; padded grid (L+2)x(W+2), cell = x*(W+2)+y */
    int32_t P, R;             /* people per env, robots per env */
    int32_t t_max;            /* fire max_steps (tables hold t = 0..t_max) */
    int32_t ox0, oy0, OX, OY; /* danger_o window origin / size */
    int32_t exit_x, exit_y;   /* EvacuationEnv.exit_location */
    int32_t rx_lo, rx_hi;     /* Map.robot_range (envs/map.py:75) */
    int32_t reset_view_x, reset_view_y; /* Map.robot_position set by reset (envs/evacuation_env.py:64) */
    int32_t reset_robots;     /* 1 = EvacuationEnvMulti.reset re-places robots */
    int32_t flags;            /* EVX_LAYOUT_* */
    int32_t repel_d2;         /* smallest integer n with sqrt(n) >= repel_range (host-computed) */
    int32_t pad0;
    double repel_k, repel_range;  /* People.ROBOT_REPEL_K / _RANGE (envs/people.py:94-95) */
    double evac_reward, death_penalty, death_acc_penalty, alive_bonus; /* envs/evacuation_env.py:16-19 */
    const double *floor;      /* [G] floor field */
    const uint8_t *cellinfo;  /* [G] bit0 valid, bit1 exit (checkSavefy), bit2 barrier_list */
    const uint32_t *valid_bits; /* [ceil(G/32)] bit0 of cellinfo as a bitmap */
    const double *danger_p;   /* [(t_max+1)*G] danger at person positions (x+.5,y+.5) */
    const double *danger_o;   /* [(t_max+1)*OX*OY] danger at integer obs coordinates */
    const float *danger_o32;  /* same, float32 (network input path) */
    const int32_t *robot_init;/* [R*2] robot positions after a multi-robot reset */
    const uint8_t *nbr_valid; /* [G] bit d: Check_Valid of the MoveTO[d] neighbour (envs/people.py:259-265) */
    const double *floor_d5;   /* [G][8] (floor[c] - floor[c + MoveTO[d]]) * 5.0 = getDeltaP * 5.0 (envs/people.py:268,282) */
    /* [(t_max+1)][L+2+2*EVX_FEAT_PAD][W+2+2*EVX_FEAT_PAD] static observation features of map
     * cell (x, y) at index (t, x + PAD, y + PAD): bf16(danger_o32) in bits 0-15, the
     * barrier channel (!valid || barrier_list) in bit 16, the exit channel in bit 17
     * (_get_state's channels 2-4, envs/evacuation_env.py:84-120); read by the MLP fast path */
    const uint32_t *obs_feat;
    /* Layout set (per-env layouts), or NULL: a device array of the evx_layout
     * descriptors of every layout of the set -- all of one size (L, W, P, R, t_max, OX, OY) --
     * indexed by evx_state.layout_idx[e] in the env kernels and by evx_obs.layout in the
     * observation readers; obs_feats is the device array of their obs_feat tables. */
    const void *layout_set;
    const uint32_t *const *obs_feats;
    /* f32-accurate MLP inputs (evx_qmlp_params.x3): the bf16 residual of the danger feature,
     * bf16(danger_o32 - bf16(danger_o32)), indexed as obs_feat; obs_feats_lo: per layout of a set */
    const uint16_t *obs_feat_lo;
    const uint16_t *const *obs_feats_lo;
} evx_layout;

#define EVX_FEAT_PAD 6

/* Structure-of-arrays state of E env instances (env-major). */
typedef struct {
    int32_t E;
    uint32_t *pk;      /* [E*P] person: x | y<<12 | safe<<24 | dead<<25 */
    double *health;    /* [E*P] Person.health */
    double *acc;       /* [E*P] Person.move_accumulator */
    uint32_t *rmap;    /* [E*ceil(G/32)] People.rmap as a bitmap */
    int32_t *thmap;    /* [E*G] People.thmap, or NULL (diagnostic heat map) */
    uint32_t *robots;  /* [E*R] Map.robot_positions: (uint16)x | (uint16)y<<16 */
    uint32_t *view;    /* [E]   Map.robot_position (same packing) */
    int32_t *scal;     /* [E*4] fire_step, current_step, prev_evacuated, prev_dead */
    uint32_t *py_mt;   /* [E*625] CPython `random` MT19937 state per env */
    uint32_t *np_mt;   /* [E*625] legacy numpy.random MT19937 state per env */
    uint32_t *scratch; /* [E*evx_step_scratch_words] step scratch: move plan, contested lists beyond LDS */
    int32_t *order;    /* [E+1] dispatch order of the step's envs (evx_env_order), or NULL = 0..E-1;
                        * order[E] = H: the first H of them are heavy (rows phase on a 4-wave workgroup) */
    const int32_t *layout_idx; /* [E] each env's layout in evx_layout.layout_set, or NULL (one layout) */
    uint8_t *perm_ws;  /* [evx_perm_ws_bytes(E)] one class byte per env for the scheduling
                        * permutations (persons-remaining bucket, fire step >= t_max, heavy),
                        * written by the step and reset kernels as they finish an env (or by
                        * evx_env_classes from the state words) and read by evx_env_order /
                        * evx_act_perm / evx_env_orders, one launch each. NULL: evx_env_order
                        * reads the state words itself, evx_act_perm / evx_env_orders fail */
} evx_state;

/* Compact per-robot observation (32 B). Expands to the reference's 11x11x6
 * _get_state tensor (envs/evacuation_env.py:84-120) given the layout. */
typedef struct {
    uint32_t occ[4];   /* bit c (c = i*11+j): People.rmap at (cx+i-5, cy+j-5) if valid */
    int32_t cx, cy;    /* window centre */
    int32_t fire_step; /* env fire model step the obs was taken at */
    int32_t layout;    /* the env's layout in evx_layout.layout_set (0 without a set) */
} evx_obs;

/* Per-step outputs. */
typedef struct {
    double *reward;    /* [E] EvacuationEnv._calculate_reward (envs/evacuation_env.py:174-288) */
    uint8_t *done;     /* [E] */
    int32_t *counts;   /* [E*2] evacuated, dead after the step (may be NULL) */
    evx_obs *obs;      /* [E*R] observation after the step */
    int32_t *err;      /* [1] sticky device error word (may be NULL); bits: 1 > 128 movers on one
                        * target, 2 a runaway Python-stream window, 4 reset placement, 8 / 16
                        * scratch or event-list overflow, 32 kept-list mismatch, 64 an MT block
                        * overwritten before the state store (any bit: results not bit-exact) */
    int64_t *stamps;   /* [E*48] diagnostic per-phase s_memtime stamps + counters (NULL = off) */
    /* Auto-reset (NULL = off, the reference's separate env.reset): envs that finish this
     * step are reset in the same launch (evx_env_reset semantics); their terminal
     * observations go to obs_term [E*R] and obs receives the post-reset ones. */
    evx_obs *obs_term;
} evx_step_out;

/* Replaces EvacuationEnv.step / EvacuationEnvMulti.step (envs/evacuation_env.py:122-172,
 * envs/evacuation_env_multi.py:55-89): robot moves (Map.move_robot envs/map.py:160-201),
 * People.run (envs/people.py:196-314), fire update, reward, counters, observation.
 * actions: [E*R] int32; values outside 0..4 are ignored as in the reference. */
int evx_env_step(const evx_layout *lay, const evx_state *st, const int32_t *actions,
                 const evx_step_out *out, void *stream);
/* The same step in two launches that may run concurrently on two streams: part 1 steps the
 * heavy envs of the dispatch order (order[0, order[E]), one workgroup each), part 2 every
 * other env; part 0 = evx_env_step. Both parts of one step must be launched with the same
 * state, order, actions and outputs; results are identical to the one-launch step. */
int evx_env_step_part(const evx_layout *l, const evx_state *s, const int32_t *actions, const evx_step_out *o,
                      int32_t part, void *stream);

/* Replaces EvacuationEnv.reset / EvacuationEnvMulti.reset (envs/evacuation_env.py:61-82,
 * envs/evacuation_env_multi.py:31-42) incl. People placement (envs/people.py:183-194).
 * mask: [E] uint8 (NULL = all envs); obs receives the reset observation of masked envs. */
int evx_env_reset(const evx_layout *lay, const evx_state *st, const uint8_t *mask, evx_obs *obs,
                  int32_t *err, void *stream);

/* Expands n compact observations to the reference tensor layout [n][11][11][6]. */
int evx_obs_expand_f32(const evx_layout *lay, const evx_obs *obs, int64_t n, float *out, void *stream);
int evx_obs_expand_f64(const evx_layout *lay, const evx_obs *obs, int64_t n, double *out, void *stream);

/* Host helper: MT19937 states for integer seeds as random.seed(s) (init_by_array)
 * and numpy.random.seed(s) (init_genrand) produce them. Host pointers. */
int evx_seed_host(const uint32_t *seeds_host, int32_t n, uint32_t *py_mt_host, uint32_t *np_mt_host);

/* Scheduling only (results do not depend on it): st->order = envs by descending
 * persons still in play, so the heaviest env-steps start first; order[E] = how many
 * of the first get a whole workgroup each (at most 256, each with >= P/4 persons in
 * play; EVX_HEAVY_CAP / EVX_HEAVY_MIN override). */
int evx_env_order(const evx_layout *lay, const evx_state *st, void *stream);
/* act row permutation for the x3 act fast path: perm[0..E) lists the envs whose fire step is >= the
 * layout's t_max (the static-table fire step) first, then the rest, each in env order (stable) */
int evx_act_perm(const evx_layout *l, const evx_state *s, int32_t *perm, void *stream);
/* Both of the above in one launch: st->order for the next step and perm for the
 * next act, from the class bytes the step just wrote. */
int evx_env_orders(const evx_layout *l, const evx_state *s, int32_t *perm, void *stream);
/* Rewrites every env's class byte in st->perm_ws from st->scal (a state written from the host). */
int evx_env_classes(const evx_layout *l, const evx_state *s, void *stream);
/* Bytes of evx_state.perm_ws for E envs. */
int64_t evx_perm_ws_bytes(int32_t E);

/* Bytes of dynamic LDS the step kernel needs for a layout (diagnostics). */
int64_t evx_step_lds_bytes(const evx_layout *lay);
/* 32-bit words of evx_state.scratch the step needs per env. */
int64_t evx_step_scratch_words(const evx_layout *lay);
/* Test entry (no reference counterpart): one wave sorts keys[0..n) (distinct u32) in place with
 * the step's contested-list sort (envs/people.py:284-297 groups movers by target through it);
 * pad: device scratch of the next power of two >= n words. */
int evx_diag_sort_keys(uint32_t *keys, uint32_t *pad, int32_t n, void *stream);

const char *evx_last_error(void);

/* ------------------------------------------------------------------ learner
 * DQNNetwork / DQNAgent (agents/dqn_agent.py:15-191) as device primitives. */

#define EVX_PREC_F32 0   /* exact f32 MFMA (v_mfma_f32_32x32x2_f32), parity path */
#define EVX_PREC_BF16 1  /* bf16 inputs, f32 accumulate (v_mfma_f32_32x32x16_bf16) */
#define EVX_PREC_X3 2    /* f32-accurate: bf16 hi + lo operand pairs, hi*hi + hi*lo + lo*hi on the bf16 MFMA */
#define EVX_GEMM_RELU 1
#define EVX_GEMM_ACCUM 2
/* X3 only. SPLIT_AB: A and B hold bf16 hi / lo planes (k-contiguous: sak = sbk = 1; A's lo plane
 * M*sam elements after its hi plane, B's N*sbn after) -- their staging copies 16-B pieces instead
 * of splitting f32 per element. OUT_SPLIT (evx_conv3x3_gemm forward, LDS-staged kernel only): C is
 * written as bf16 hi / lo planes, the lo plane M*ldc elements after the hi plane. */
#define EVX_GEMM_SPLIT_AB 4
#define EVX_GEMM_OUT_SPLIT 8

/* C[m][n] = epi(alpha * sum_k A(m,k) B(k,n) + bias[n]) with A(m,k) = A[m*sam + k*sak],
 * B(k,n) = B[k*sbk + n*sbn], C[m*ldc + n]; epilogue order: bias, ReLU, dropout mask
 * (mask[m*ldm+n] ? v*mask_scale : 0), ReLU-backward gate (gate[m*ldg+n] > 0 ? v : 0),
 * accumulate. Covers nn.Linear forward (A x W^T), its dX (dY W) and dW (dY^T X).
 * BF16 / X3 GEMMs with a long K and few 128x128 tiles (fewer than 256 without an epilogue, at
 * most 256 with one) may be split over K when the caller passes a workspace: each K slice
 * stores its raw partial into ws[z][M][N] and a second launch on the same stream adds the
 * slices in slice order and applies the epilogue (deterministic: the same bits on every call).
 * The slice count is capped by ws_elems / (M*N); ws = NULL runs the GEMM in one pass.
 * evx_gemm_ws_elems gives the workspace a descriptor's full split uses (0: never split).
 * EVX_PREC_F32 never splits. */
typedef struct {
    int32_t M, N, K;
    int32_t precision;         /* EVX_PREC_* */
    int32_t flags;             /* EVX_GEMM_* */
    float alpha;
    const float *A; int64_t sam, sak;
    const float *B; int64_t sbk, sbn;
    float *C; int64_t ldc;
    const float *bias;         /* [N] or NULL */
    const uint8_t *mask; int64_t ldm; float mask_scale;  /* or NULL */
    const float *gate; int64_t ldg;                        /* or NULL */
    float *ws; int64_t ws_elems;  /* split-K workspace (f32 elements) or NULL */
} evx_gemm_desc;

typedef struct {
    float lr, beta1, beta2, eps, weight_decay;
    int64_t step;  /* 1-based step count after increment (torch.optim.Adam state['step']) */
} evx_adam;

/* Uniform replay ring of compact observations (DQNAgent.memory, agents/dqn_agent.py:88-99). */
typedef struct {
    int64_t capacity;
    evx_obs *s, *s2;
    int32_t *a;
    float *r;
    uint8_t *done;
} evx_replay;

int evx_gemm(const evx_gemm_desc *g, void *stream);
int64_t evx_gemm_ws_elems(const evx_gemm_desc *g);
/* Implicit-GEMM 3x3 convolution, padding 1, on 11x11 maps (DQNNetwork conv1-3,
 * agents/dqn_agent.py:22-24,48-50, in place of im2col + evx_gemm; x3 precision only). The
 * activations are pixel-major [B*121][cs]; the operand they feed is gathered in the tile fetch:
 *   EVX_CONV_FWD: C[m][n] = sum_{tap,c} A[m shifted by tap][c] W[n][c][tap]; M = B*121, K = 9 cs,
 *                 B = W with sbk = 9 (c stride), sbn = 9 cs (n stride). Epilogue as evx_gemm.
 *   EVX_CONV_DX:  C[m][n] = sum_{tap,o} A[m shifted by -tap][o] W[o][n][tap] (dX of the layer,
 *                 A = dY [B*121][cs]); K = 9 cs, B = W with sbk = 9 N, sbn = 9; gate = the
 *                 layer input (ReLU backward of the layer below).
 *   EVX_CONV_DW:  C[o][c*9+tap] = sum_m A[m][o] B[m shifted by tap][c] (dW, A = dY with sam = 1,
 *                 sak = M; B = the layer input [B*121][cs]); N = 9 cs, K = B*121.
 * Out-of-map taps read 0. */
#define EVX_CONV_FWD 1
#define EVX_CONV_DX 2
#define EVX_CONV_DW 3
int evx_conv3x3_gemm(const evx_gemm_desc *g, int32_t mode, int32_t cs, void *stream);
/* Workspace floats (evx_gemm_desc.ws / ws_elems) an evx_conv3x3_gemm call can use: the LDS-staged
   forward (bias / ReLU epilogue) and dX (ReLU gate) kernels over cfg4's layer shapes pack the
   weights there as bf16 hi / lo MFMA fragments; otherwise the split-K partials of
   evx_gemm_ws_elems. Without it the call runs the generic implicit-GEMM kernel. */
int64_t evx_conv3x3_ws_elems(const evx_gemm_desc *g, int32_t mode, int32_t cs);
/* out[n] (+)= sum_m X[m*ld+n] (bias gradients), fixed summation order */
int evx_colsum(const float *X, int64_t ld, int32_t M, int32_t N, float *out, int32_t accum, float *scratch,
               int32_t scratch_elems, void *stream);
/* DQNAgent.learn TD step (agents/dqn_agent.py:143-151): loss = mean((Q[a] - (r + gamma*max Qt * !done))^2),
 * dQ = d loss / d Q. Q, Qt: [B][A]. ws: caller workspace of evx_td_loss_ws_floats(B, nets) floats
 * (the per-block partials of the loss, summed in block order by a second launch: deterministic,
 * no state in the library; calls on different streams need different workspaces). */
int64_t evx_td_loss_ws_floats(int32_t B, int32_t nets);
int evx_td_loss(const float *Q, const float *Qt, int32_t A, const int32_t *act, const float *rew,
                const uint8_t *done, float gamma, int32_t B, float *dQ, float *loss, float *ws, int64_t ws_floats,
                void *stream);
/* evx_td_loss with optional importance weights w [B] (prioritized replay: loss = mean(w (q - y)^2),
 * dQ scaled by w) and optional td_abs [B] = |q - y| (the new priorities); w = td_abs = NULL is
 * evx_td_loss. */
int evx_td_loss_w(const float *Q, const float *Qt, int32_t A, const int32_t *act, const float *rew,
                  const uint8_t *done, float gamma, int32_t B, const float *w, float *dQ, float *loss,
                  float *td_abs, float *ws, int64_t ws_floats, void *stream);
/* evx_td_loss_w plus clearing zero[0..nzero) (the gradient buffer the backward accumulates into)
 * in the same launch (extra workgroups) */
int evx_td_loss_zero(const float *Q, const float *Qt, int32_t A, const int32_t *act, const float *rew,
                     const uint8_t *done, float gamma, int32_t B, const float *w, float *dQ, float *loss, float *td_abs,
                     float *zero, int64_t nzero, float *ws, int64_t ws_floats, void *stream);
/* ||g||_2 into norm[0] (clip_grad_norm_'s total norm) */
int evx_sumsq_norm(const float *g, int64_t n, float *scratch, int32_t scratch_elems, float *norm, void *stream);
/* g *= min(1, max_norm/(norm+1e-6)) (skipped if norm NULL) then one torch.optim.Adam step */
int evx_clip_adam(float *p, float *g, float *m, float *v, int64_t n, const float *norm, float max_norm,
                  const evx_adam *h, void *stream);
/* nn.Dropout keep-mask (1 with probability 1-p), counter-based Philox4x32-10 */
int evx_dropout_mask(uint8_t *mask, int64_t n, float p, uint64_t seed, uint64_t offset, void *stream);
/* DQNAgent.act (agents/dqn_agent.py:101-124): epsilon-greedy over argmax_a Q[i][a] */
int evx_act(const float *Q, int32_t n, int32_t A, float epsilon, uint64_t seed, uint64_t offset,
            int32_t *actions, void *stream);
int evx_replay_push(const evx_replay *rp, const evx_obs *s, const evx_obs *s2, const int32_t *a,
                    const double *r_env, const uint8_t *done_env, int32_t n, int32_t agents_per_env, int64_t pos,
                    void *stream);
/* random.sample replacement for the vectorised learner: B uniform indices < size */
/* evx_replay_push with s2 = done_env[e] ? s2_term : s2 (the terminal observations of
 * envs that evx_env_step auto-reset) */
int evx_replay_push_term(const evx_replay *rp, const evx_obs *s, const evx_obs *s2, const evx_obs *s2_term,
                         const int32_t *a, const double *r_env, const uint8_t *done_env, int32_t n,
                         int32_t agents_per_env, int64_t pos, void *stream);
/* evx_replay_push_term and evx_env_orders (the next step's order and the next act's env order
 * `perm`, from the class bytes of state `s`) in one launch; the replay capacity must be a power of
 * two. Replaces DQNAgent.remember for every robot of a step (agents/dqn_agent.py:97-99) plus the
 * scheduling permutations. */
int evx_env_orders_push(const evx_layout *l, const evx_state *s, int32_t *perm, const evx_replay *rp,
                        const evx_obs *s_obs, const evx_obs *s2, const evx_obs *s2_term, const int32_t *a,
                        const double *r_env, const uint8_t *done_env, int32_t n, int32_t agents_per_env,
                        int64_t pos, void *stream);
/* ... and the learn step's batch (evx_replay_sample over the ring as it stands after the push:
 * size = the ring size after it; B = 0 draws nothing) in the same launch. */
int evx_env_orders_push_sample(const evx_layout *l, const evx_state *s, int32_t *perm, const evx_replay *rp,
                               const evx_obs *s_obs, const evx_obs *s2, const evx_obs *s2_term, const int32_t *a,
                               const double *r_env, const uint8_t *done_env, int32_t n, int32_t agents_per_env,
                               int64_t pos, int32_t B, int64_t size, uint64_t seed, uint64_t offset, evx_obs *out_s,
                               evx_obs *out_s2, int32_t *out_a, float *out_r, uint8_t *out_done, void *stream);
int evx_replay_sample(const evx_replay *rp, int64_t size, int32_t B, uint64_t seed, uint64_t offset, evx_obs *s,
                      evx_obs *s2, int32_t *a, float *r, uint8_t *done, int64_t *idx_out, void *stream);
/* B uniform indices over the ring window [base, base+count) mod capacity (same draws as
 * evx_replay_sample with base 0): lets a learn step sample the transitions already pushed
 * while the next push overwrites the slots outside the window (lagged-replay schedule) */
int evx_replay_sample_window(const evx_replay *rp, int64_t base, int64_t count, int32_t B, uint64_t seed,
                             uint64_t offset, evx_obs *s, evx_obs *s2, int32_t *a, float *r, uint8_t *done,
                             int64_t *idx_out, void *stream);
/* One memory per agent (runners/train_double_dqn.py:50-51: agent_i.remember / learn on its own
 * transitions): with pushes of whole envs (rows env * nets + agent, capacity % nets == 0) the
 * agent's transitions are the ring slots == agent (mod nets); B uniform draws among them
 * (among the first size slots) for every agent, into rows [agent B, (agent + 1) B). */
int evx_replay_sample_agents(const evx_replay *rp, int64_t size, int32_t B, int32_t nets, uint64_t seed,
                             uint64_t offset, evx_obs *s, evx_obs *s2, int32_t *a, float *r, uint8_t *done,
                             void *stream);
/* The joint memory of runners/train_qmix.py:36,78-96 (one entry per env-step, all agents'
 * observations and actions): draw i picks the same env-step for every agent (rows agent B + i
 * hold that agent's slot); counters offset + i. */
int evx_replay_sample_joint(const evx_replay *rp, int64_t size, int32_t B, int32_t nets, uint64_t seed,
                            uint64_t offset, evx_obs *s, evx_obs *s2, int32_t *a, float *r, uint8_t *done,
                            void *stream);
/* ------------------------------------------- prioritized replay
 * Proportional prioritized replay (Schaul et al. 2016) over the slots of an evx_replay
 * ring; the reference samples uniformly (random.sample, agents/dqn_agent.py:132), so
 * this is the build's own extension, pinned by oracle/prio_oracle.c. Two segment trees
 * in heap layout over capacity C = 2^k slots (node n = child 2n (op) child 2n+1, root 1,
 * slot i at leaf C + i): sums and minima of the leaf priorities p_i^alpha. Empty or
 * hidden slots hold 0 in the sum tree and +inf in the min tree. New transitions get the
 * largest leaf priority set so far (max_leaf, initially 1). */
typedef struct {
    int64_t capacity;   /* power of two, 2^10 <= C <= 2^26 */
    double *sum;        /* [2C] */
    double *mn;         /* [2C] */
    double *max_leaf;   /* [1] */
    int32_t *owner;     /* [C] scratch for evx_prio_update, all -1 (evx_prio_init sets it) */
} evx_prio;

/* all leaves empty (sum 0, min +inf), max_leaf = 1, owner = -1 */
int evx_prio_init(const evx_prio *t, void *stream);
/* Slots [pos, pos + n_new) mod C get priority max_leaf (newly pushed transitions) and
 * slots [pos + n_new, pos + n_new + n_hide) mod C get priority 0 (hidden: about to be
 * overwritten by a push running concurrently -- the lagged schedule); both trees are
 * rebuilt over the touched leaf blocks. n_new + n_hide <= C. */
int evx_prio_set_range(const evx_prio *t, int64_t pos, int64_t n_new, int64_t n_hide, void *stream);
/* Leaf idx[k] = (td_abs[k] + eps)^alpha for k = 0..B-1 (a later k wins over an earlier
 * one with the same slot, as a sequential loop), max_leaf updated, trees rebuilt. */
int evx_prio_update(const evx_prio *t, const int64_t *idx, const float *td_abs, int32_t B, double eps,
                    double alpha, void *stream);
/* Stratified proportional sampling: for k = 0..B-1, u = (k + U_k) * (total / B) with U_k a
 * 53-bit uniform from Philox4x32-10(counter offset + k, key seed); descend the sum tree
 * (left if u < sum[left] or sum[right] <= 0, else u -= sum[left] and right). Gathers the
 * transitions like evx_replay_sample and writes the importance weights
 * w_k = (p_k / p_min)^(-beta) (= (N P(k))^-beta / max_j (N P(j))^-beta). */
int evx_prio_sample(const evx_replay *rp, const evx_prio *t, int32_t B, double beta, uint64_t seed,
                    uint64_t offset, evx_obs *s, evx_obs *s2, int32_t *a, float *r, uint8_t *done,
                    int64_t *idx_out, float *w_out, void *stream);

const char *evx_prio_last_error(void);

/* ---- static floor field on the device ------------------------------------
 * Replaces Map.Init_Potential (envs/map.py:127-148) for n_layouts layouts of one padded grid
 * size GX x GY (= (L+2) x (W+2)), one workgroup each, bit-identical to the reference's heapq
 * Dijkstra. Per layout, row-major [GX][GY]:
 *   valid  u8  Map.Check_Valid on the pre-potential grid (1 <= x <= L, 1 <= y <= W, space != inf)
 *   source u8  the exits (Map.Exit: distance 1)
 *   pen    f64 200 * danger(t=0, (i, j)) ** 2 (envs/map.py:143-146; NULL = no fire term)
 *   floor  f64 out: Map.space after Init_Potential (inf where unreachable)
 *   passes i32 [n_layouts] relaxation passes used (may be NULL; diagnostics) */
int evx_floor_field(int32_t n_layouts, int32_t GX, int32_t GY, const uint8_t *valid, const uint8_t *source,
                    const double *pen, double *floor, int32_t *passes, void *stream);
const char *evx_floor_last_error(void);

int evx_gather_obs(const evx_obs *src, const int64_t *idx, int32_t n, evx_obs *dst, void *stream);
/* DQNNetwork conv layers (agents/dqn_agent.py:22-24) as im2col + GEMM on 11x11 maps */
int evx_im2col3x3(const float *x, int32_t B, int32_t C, int32_t nhwc, float *cols, void *stream);
int evx_col2im3x3(const float *dcols, int32_t B, int32_t C, float *dx, void *stream);
/* NCHW [B][C][121] f32 -> pixel-major [B][121*C] as bf16 hi / lo planes (lo B*121*C elements after
   hi): the x3 operand of an EVX_GEMM_SPLIT_AB GEMM (the conv net's fc1 weights), C <= 134 */
int evx_pix_split(const float *src, int32_t B, int32_t C, uint16_t *dst, void *stream);
/* [B*121][C] pixel-major <-> [B][C][121] NCHW (to_nchw): through LDS for C <= 134, element-wise
   beyond (any C) */
int evx_pix_nchw(const float *src, int32_t B, int32_t C, int32_t to_nchw, float *dst, void *stream);
int evx_relu_grad(float *dy, const float *y, int64_t n, void *stream);
const char *evx_q_last_error(void);

/* ------------------------------------------------- MLP Q-network fast path (bf16 MFMA)
 * DQNNetwork's fc stack (agents/dqn_agent.py:40-61; MLP variant 726-512-256-5) with the
 * observation expansion of EvacuationEnv._get_state (envs/evacuation_env.py:84-120)
 * generated inside fc1, and DQNAgent.act's epsilon-greedy (:101-124) fused after fc3.
 * Dropout keep bits are a counter hash of (seed, stream, row, col): the backward pass
 * regenerates them. */
typedef struct {
    const uint16_t *w1;   /* [512][512] bf16 fc1.weight over the compact K (evx_qmlp_pack), MFMA operand-tiled */
    const float *b1c;     /* [512] fc1.bias + bf16(fc1.weight[:, 365]) (the constant centre channel), evx_qmlp_pack */
    const uint16_t *w2;   /* [256][512] bf16 fc2.weight, MFMA operand-tiled (evx_qmlp_pack) */
    const uint16_t *w2t;  /* [512][256] bf16 fc2.weight transposed (backward), may be NULL for forward */
    const float *b2;      /* [256] */
    const float *w3;      /* [5][256] f32 fc3.weight */
    const float *b3;      /* [5] */
    /* act fast path (evx_qmlp_act), optional: fc1's occupancy columns [512][128] bf16 (evx_qmlp_pack's
     * w1o) and the pre-activation table of evx_qmlp_stat for observations at fire step stat_fs */
    const uint16_t *w1o;
    const float *stat;
    int32_t stat_fs;
    /* x3 = 1: f32-accurate arithmetic (the reference's fp32 DQNNetwork): every f32 operand v is
     * carried as bf16 hi = bf16(v) plus lo = bf16(v - hi) and a product as hi*hi + hi*lo + lo*hi
     * on the bf16 MFMA (exact 0/1 operands skip their lo); w1 then spans K = 640 (compact K +
     * one danger-residual slot per cell), w1l / w2l / w2tl hold the lo parts (evx_qmlp_pack3) */
    int32_t x3;
    const uint16_t *w1l, *w2l, *w2tl;
    /* x3 act fast path: the lo part of w1o (w1o then holds the hi part; evx_qmlp_pack3 / _adam_pack3) */
    const uint16_t *w1ol;
    /* the table's window centres: x in [stat_x0, stat_x0 + stat_nx) (Map.robot_range: robots never
     * leave it), every y in [0, W + 1], row (x - stat_x0) * (W + 2) + y; stat_nx = 0: all L + 2 */
    int32_t stat_x0, stat_nx;
    /* x3, optional: the table rows' fc1 inputs (evx_qmlp_expand_x3 of the table's observations, the X of
     * evx_qmlp_stat_x): the learner's X of a batch row on the table path is that row of it plus the
     * row's occupancy bits (copied instead of regenerated; the same bits) */
    const uint16_t *stat_xin;
} evx_qmlp_params;

typedef struct {
    uint32_t seed, stream; /* mask identity */
    float p;               /* drop probability; 0 = eval (no dropout) */
    uint32_t row0;         /* hash row of the batch's first row (even): a rank's act masks keyed by the
                            * global agent id, so trajectories do not depend on the GPU count */
    const uint8_t *mask;   /* optional explicit keep mask [n][512] (1 = keep; scale 1/(1-p)) in place of
                            * the hash: replays the reference's captured torch dropout masks */
} evx_qmlp_dropout;

typedef struct {
    uint16_t *h1;          /* [n][512] bf16 fc1 output after ReLU + dropout (required) */
    uint16_t *x;           /* [n][512] bf16 compact expanded observation, or NULL */
    float *h2;             /* [n][256] fc2 output after ReLU, or NULL */
    float *q;              /* [n][5] Q values, or NULL */
    int32_t *actions;      /* [n] epsilon-greedy actions (evx_act's rule and RNG), or NULL */
    float epsilon;
    uint64_t act_seed, act_offset;
    /* x3: h1 holds two planes [2][n][512] (hi, lo) and x spans [n][640] */
    /* act only, optional: batch row i is observation / action row perm[i / rows_per_env] * rows_per_env +
     * i % rows_per_env (evx_act_perm: envs at the table's fire step first, so act tiles are uniform);
     * dropout rows and epsilon draws stay keyed by that original row; rows_per_env even (dropout
     * row pairs stay together) */
    const int32_t *perm;
    int32_t rows_per_env;
    /* act only, optional: int32 workspace of evx_qmlp_act_ws_ints(n) elements, zeroed once by the
     * caller (every act leaves its two counters zeroed; one workspace per act in flight). With it the x3 persistent act lists
     * the 128-row tiles it leaves to the 64-row kernel (a row below stat_fs or a centre outside the
     * table), so that kernel runs only those instead of re-checking every row (NULL: it re-checks). */
    int32_t *act_ws;
} evx_qmlp_fwd_out;

/* elements of evx_qmlp_fwd_out.act_ws for an act of n rows */
int64_t evx_qmlp_act_ws_ints(int32_t n);

/* bf16 copies of fc1.weight [512][726] over fc1's compact K and fc2.weight [256][512]
 * (w2t may be NULL), and b1c. Compact K: 4 features per cell c < 121 at k = 4c + f for
 * the reference's channels f + 1 (occupancy, danger, barrier, exit), k >= 484 zero; the
 * reference's channel 0 is identically zero and channel 5 is the constant centre
 * one-hot, folded into b1c. */
int evx_qmlp_pack(const float *w1, const float *b1, const float *w2, uint16_t *w1b, float *b1c, uint16_t *w2b,
                  uint16_t *w2t, uint16_t *w1o, void *stream);
/* x3 (f32-accurate) operand copies: w1b [512][640] hi (compact K, then the danger column of cell
 * c at k = 512 + c, multiplying the danger residual), w1l [512][512] lo of the compact K, w2b / w2l
 * hi / lo of fc2.weight, w2t / w2tl of its transpose (may be NULL); b1c = b1 + W1[:, centre] in f32 */
int evx_qmlp_pack3(const float *w1, const float *b1, const float *w2, uint16_t *w1b, uint16_t *w1l, float *b1c,
                   uint16_t *w2b, uint16_t *w2l, uint16_t *w2t, uint16_t *w2tl, void *stream);
/* x3 act fast path operands: fc1's occupancy columns [512][128] as hi (w1o) and lo (w1ol) bf16, w1o_tile order */
int evx_qmlp_pack_occ3(const float *w1, uint16_t *w1o, uint16_t *w1ol, void *stream);
/* fc1's pre-activation (X W1^T + b1, f32, no ReLU / dropout) of n observations -> out [n][512]:
 * with obs = every window centre of the layout at one fire step and zero occupancy this is the
 * act fast path's table (evx_qmlp_params.stat; rebuild after every weight update) */
int evx_qmlp_stat(const evx_layout *lay, const evx_obs *obs, int32_t n, const evx_qmlp_params *p, float *out,
                  void *stream);
/* x3: the rows' compact fc1 inputs [n][640] bf16 (4 features per cell, then the cells' danger
 * residuals: the X of evx_qmlp_fwd_out.x) of n observations */
int evx_qmlp_expand_x3(const evx_layout *lay, const evx_obs *obs, int32_t n, uint16_t *x, void *stream);
/* evx_qmlp_stat (x3) from the rows' X of evx_qmlp_expand_x3 instead of their observations: the same
 * table bit for bit, with fc1's A operand read instead of generated (the act table's rows are fixed,
 * so their X is expanded once; x NULL: evx_qmlp_stat) */
int evx_qmlp_stat_x(const evx_layout *lay, const evx_obs *obs, const uint16_t *x, int32_t n, const evx_qmlp_params *p,
                    float *out, void *stream);
int evx_qmlp_forward(const evx_layout *lay, const evx_obs *obs, int32_t n, const evx_qmlp_params *p,
                     const evx_qmlp_dropout *drop, const evx_qmlp_fwd_out *out, void *stream);
/* DQNAgent.act (agents/dqn_agent.py:101-124) in one launch: the forward of
 * evx_qmlp_forward with H1 and H2 kept on chip (out->h1, x, h2 ignored), writing
 * out->q and/or out->actions; bit-identical to evx_qmlp_forward's, except that 128-row tiles
 * whose observations are all at p->stat_fs start fc1 from p->stat (when p->w1o / p->stat are
 * set): the same products summed in another order. */
int evx_qmlp_act(const evx_layout *lay, const evx_obs *obs, int32_t n, const evx_qmlp_params *p,
                 const evx_qmlp_dropout *drop, const evx_qmlp_fwd_out *out, void *stream);
/* The same act on the 64-row kernel only. x3 evx_qmlp_act runs a persistent kernel of 128-row tiles
 * (one workgroup per CU) when the table path is attached, the dropout is the hash or off and n
 * covers 4 tiles per CU; it gives the same bits as this one (tests compare the two). */
int evx_qmlp_act64(const evx_layout *lay, const evx_obs *obs, int32_t n, const evx_qmlp_params *p,
                   const evx_qmlp_dropout *drop, const evx_qmlp_fwd_out *out, void *stream);
/* Two forwards of n rows in one launch pair (the learner's online and target nets). */
int evx_qmlp_forward2(const evx_layout *lay, int32_t n, const evx_obs *obs0, const evx_qmlp_params *p0,
                      const evx_qmlp_dropout *drop0, const evx_qmlp_fwd_out *out0, const evx_obs *obs1,
                      const evx_qmlp_params *p1, const evx_qmlp_dropout *drop1, const evx_qmlp_fwd_out *out1,
                      void *stream);

/* fp32 gradient tensors (the reference's parameter shapes: fc1.weight [512][726], ...) */
typedef struct {
    float *w1, *b1, *w2, *b2, *w3, *b3;
    /* required scratch of the backward's partial sums, evx_qmlp_backward_part_floats(B) floats
     * (weight-gradient split-K tiles, fc3 / bias block rows): every gradient sum is added in a
     * fixed order -- the same bits on every run, no f32 atomics */
    float *part;
} evx_qmlp_grads;
int64_t evx_qmlp_backward_part_floats(int32_t B);

/* loss.backward() of DQNAgent.learn (agents/dqn_agent.py:150-158) for the saved online
 * forward (x, h1, h2 of evx_qmlp_forward) given dQ = d loss / d Q [B][5]. zero_grads != 0: the
 * gradients are overwritten (every element), else added to. dz2 [B][256] and dz1
 * [B][512] are bf16 scratch. Needs p->w2t. With p->x3 the activations are the x3 forward's
 * (h1 two planes, x 640 wide), dz2 / dz1 hold two planes each (hi, lo) and every product
 * is split as in the forward. */
int evx_qmlp_backward(const evx_qmlp_params *p, int32_t B, const float *dq, const uint16_t *x, const uint16_t *h1,
                      const float *h2, float drop_p, uint16_t *dz2, uint16_t *dz1, const evx_qmlp_grads *g,
                      int32_t zero_grads, void *stream);
/* evx_qmlp_backward that also leaves clip_grad_norm_'s squared-norm partials of the final gradients
 * in ss[0 .. evx_qmlp_norm_parts()) (the gradients one flat state_dict-order buffer: g->w1 .. g->b3
 * contiguous); with g->part the weight-gradient reductions and the partials share one launch. */
int evx_qmlp_backward_ss(const evx_qmlp_params *p, int32_t B, const float *dq, const uint16_t *x, const uint16_t *h1,
                         const float *h2, float drop_p, uint16_t *dz2, uint16_t *dz1, const evx_qmlp_grads *g,
                         int32_t zero_grads, float *ss, void *stream);
/* DQNAgent.learn's TD step and loss.backward() in one (agents/dqn_agent.py:143-158): dQ from the
 * online Q [B][5], the target Qt [B][5], actions, rewards, done flags and gamma (as evx_td_loss_w,
 * importance weights w or NULL) inside the backward's first kernel; loss[0] = the mean (weighted)
 * squared TD error, td_abs [B] = |TD error| (or NULL); the gradients overwritten; ss as in
 * evx_qmlp_backward_ss, or NULL (no norm partials: an all-reduce will change the gradients). */
int evx_qmlp_td_backward_ss(const evx_qmlp_params *p, int32_t B, const float *Q, const float *Qt, const int32_t *act,
                            const float *rew, const uint8_t *done, float gamma, const float *w, float *loss,
                            float *td_abs, const uint16_t *x, const uint16_t *h1, const float *h2, float drop_p,
                            uint16_t *dz2, uint16_t *dz1, const evx_qmlp_grads *g, float *ss, void *stream);
int32_t evx_qmlp_norm_parts(void);
int64_t evx_qmlp_nparams(void);
/* the same partials of a flat gradient buffer (after an all-reduce changed it) */
int evx_qmlp_sumsq_parts(const float *g, float *ss, void *stream);
/* clip_grad_norm_ + Adam (agents/dqn_agent.py:158-160) on the MLP's flat p / g / m / v (state_dict
 * order, evx_qmlp_nparams() elements) from the nss norm partials, with the x3 operand repack
 * (evx_qmlp_pack3's outputs) in the same launch; g receives the clipped gradients, norm_out (or
 * NULL) the total norm. Replaces evx_sumsq_norm + evx_clip_adam + evx_qmlp_pack3. */
int evx_qmlp_adam_pack3(float *p, float *g, float *m, float *v, float max_norm, const evx_adam *h, uint16_t *w1b,
                        uint16_t *w1l, float *b1c, uint16_t *w2b, uint16_t *w2l, uint16_t *w2t, uint16_t *w2tl,
                        uint16_t *w1o, uint16_t *w1ol, const float *ss, int32_t nss, float *norm_out, void *stream);
const char *evx_qmlp_last_error(void);

/* ---- Grouped independent nets: runners/train_double_dqn.py:35-56 trains one
 * DQNAgent per robot, runners/train_qmix.py:78-118 one per agent under a mixer. `nets` MLPs in
 * one launch per kernel: every per-net buffer is an array [nets][one net's buffer] and the
 * pointers passed are net 0's (x3 parameters: evx_qmlp_pack3 layout per net; flat parameters,
 * gradients, m, v [nets][evx_qmlp_nparams()]). */
/* DQNAgent.act of net g for rows i*nets + g of obs / q / actions (robot g of env i uses net g),
 * n rows per net (even); dropout rows keyed g*n + i, epsilon draws by the data row. No
 * permutation, no table path (p->stat NULL). */
int evx_qmlp_act_g(const evx_layout *lay, const evx_obs *obs, int32_t n, int32_t nets, const evx_qmlp_params *p,
                   const evx_qmlp_dropout *drop, const evx_qmlp_fwd_out *out, void *stream);
/* evx_qmlp_forward2 for nets blocked problems: net g reads obs rows [g n, (g + 1) n) and writes
 * its [n]-row blocks of h1 (two planes) / x / h2 / q; dropout rows keyed g*n + row. */
int evx_qmlp_forward2_g(const evx_layout *lay, int32_t n, int32_t nets, const evx_obs *obs0,
                        const evx_qmlp_params *p0, const evx_qmlp_dropout *drop0, const evx_qmlp_fwd_out *out0,
                        const evx_obs *obs1, const evx_qmlp_params *p1, const evx_qmlp_dropout *drop1,
                        const evx_qmlp_fwd_out *out1, void *stream);
/* evx_td_loss_zero per net: rows [g B, (g + 1) B) of Q / Qt / act / rew / done / dQ, loss[g]
 * = mean over the net's rows; ws of evx_td_loss_ws_floats(B, nets) floats. */
int evx_td_loss_zero_g(const float *Q, const float *Qt, int32_t A, const int32_t *act, const float *rew,
                       const uint8_t *done, float gamma, int32_t B, int32_t nets, const float *w, float *dQ,
                       float *loss, float *td_abs, float *zero, int64_t nzero, float *ws, int64_t ws_floats,
                       void *stream);
/* evx_qmlp_backward_ss for the blocked forward of evx_qmlp_forward2_g (gradients cleared by the
 * caller); g->part: [nets][evx_qmlp_backward_part_floats(B)], ss [nets][evx_qmlp_norm_parts()]. */
int evx_qmlp_backward_ss_g(const evx_qmlp_params *p, int32_t B, int32_t nets, const float *dq, const uint16_t *x,
                           const uint16_t *h1, const float *h2, float drop_p, uint16_t *dz2, uint16_t *dz1,
                           const evx_qmlp_grads *g, float *ss, void *stream);
/* evx_qmlp_adam_pack3 per net (clip_grad_norm_ per agent, train_qmix.py:107-109); ss
 * [nets][nss], norm_out [nets] or NULL. */
int evx_qmlp_adam_pack3_g(float *p, float *g, float *m, float *v, float max_norm, const evx_adam *h, uint16_t *w1b,
                          uint16_t *w1l, float *b1c, uint16_t *w2b, uint16_t *w2l, uint16_t *w2t, uint16_t *w2tl,
                          uint16_t *w1o, uint16_t *w1ol, const float *ss, int32_t nss, float *norm_out, int32_t nets,
                          void *stream);

/* ---- QMIX mixer (runners/train_qmix.py:39-54 MixingNetwork, loss :78-104) for n <= 16 agents:
 * Q / Qt [n][B][A] (evx_qmlp_forward2_g), act [n][B], rew / done [B]; mix / mix_t the online /
 * target mixer flat in state_dict order (fc1_weight [n][32], fc1_bias [32], fc2_weight [32][1],
 * fc2_bias [1]: evx_qmix_nparams(n)). Writes dQ [n][B][A] (d loss / d Q at the taken actions),
 * the online mixer's gradient and loss[0] = mse; part: evx_qmix_part_floats(B, n) floats of
 * scratch; zero[0..nzero) (the agents' gradients) is cleared in the same launch. */
int32_t evx_qmix_nparams(int32_t n);
int64_t evx_qmix_part_floats(int32_t B, int32_t n);
int evx_qmix_loss(const float *Q, const float *Qt, int32_t A, const int32_t *act, const float *rew,
                  const uint8_t *done, float gamma, int32_t B, int32_t n, const float *mix, const float *mix_t,
                  float *dQ, float *mix_grad, float *loss, float *part, float *zero, int64_t nzero, void *stream);
const char *evx_qmix_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
