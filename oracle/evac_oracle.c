/* TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT (see evac_oracle.h).
 *
 * Literal CPU restatement of the reference hot path. Every function cites the
 * reference file:line it restates (paths relative to
 * /root/reference/Louvre_Evacuation/). Compiled with -ffp-contract=off so the
 * float64 arithmetic is evaluated exactly as CPython/numpy evaluate it.
 */
#include "evac_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* MT19937: CPython Modules/_randommodule.c and numpy mt19937 (same generator) */
/* ------------------------------------------------------------------------ */
#define MT_M 397
#define MT_UPPER 0x80000000u
#define MT_LOWER 0x7fffffffu
#define MT_MATRIX 0x9908b0dfu

static void mt_twist(uint32_t *mt) {
    int kk;
    uint32_t y;
    for (kk = 0; kk < ORC_MT_N - MT_M; kk++) {
        y = (mt[kk] & MT_UPPER) | (mt[kk + 1] & MT_LOWER);
        mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ ((y & 1u) ? MT_MATRIX : 0u);
    }
    for (; kk < ORC_MT_N - 1; kk++) {
        y = (mt[kk] & MT_UPPER) | (mt[kk + 1] & MT_LOWER);
        mt[kk] = mt[kk + (MT_M - ORC_MT_N)] ^ (y >> 1) ^ ((y & 1u) ? MT_MATRIX : 0u);
    }
    y = (mt[ORC_MT_N - 1] & MT_UPPER) | (mt[0] & MT_LOWER);
    mt[ORC_MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ ((y & 1u) ? MT_MATRIX : 0u);
}

uint32_t orc_mt_next(uint32_t *st) {
    uint32_t pos = st[ORC_MT_N];
    if (pos >= ORC_MT_N) {
        mt_twist(st);
        pos = 0;
    }
    uint32_t y = st[pos++];
    st[ORC_MT_N] = pos;
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

/* random.random() == numpy legacy random_sample(): 53-bit double from 2 words */
double orc_mt_random(uint32_t *st) {
    uint32_t a = orc_mt_next(st) >> 5, b = orc_mt_next(st) >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
}

static int bit_length(uint32_t n) {
    int k = 0;
    while (n) {
        k++;
        n >>= 1;
    }
    return k;
}

/* CPython 3.10 Random._randbelow_with_getrandbits (Lib/random.py) */
uint32_t orc_mt_randbelow(uint32_t *st, uint32_t n) {
    if (n == 0) return 0;
    int k = bit_length(n);
    uint32_t r = orc_mt_next(st) >> (32 - k);
    while (r >= n) r = orc_mt_next(st) >> (32 - k);
    return r;
}

static void init_genrand(uint32_t *mt, uint32_t s) {
    mt[0] = s;
    for (int i = 1; i < ORC_MT_N; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    mt[ORC_MT_N] = ORC_MT_N;
}

/* random.seed(int) for 0 <= seed < 2**32: init_by_array([seed]) */
void orc_seed_py(uint32_t seed, uint32_t *mt) {
    uint32_t key[1] = {seed};
    int i = 1, j = 0, k, key_length = 1;
    init_genrand(mt, 19650218u);
    for (k = ORC_MT_N; k; k--) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++;
        j++;
        if (i >= ORC_MT_N) {
            mt[0] = mt[ORC_MT_N - 1];
            i = 1;
        }
        if (j >= key_length) j = 0;
    }
    for (k = ORC_MT_N - 1; k; k--) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= ORC_MT_N) {
            mt[0] = mt[ORC_MT_N - 1];
            i = 1;
        }
    }
    mt[0] = 0x80000000u;
    mt[ORC_MT_N] = ORC_MT_N;
}

/* numpy.random.RandomState(int): mt19937_seed == init_genrand */
void orc_seed_np(uint32_t seed, uint32_t *st) { init_genrand(st, seed); }

void orc_mt_fill_random(uint32_t *st, int n, double *out) {
    for (int i = 0; i < n; i++) out[i] = orc_mt_random(st);
}

void orc_mt_fill_randbelow(uint32_t *st, const int64_t *ns, int n, int64_t *out) {
    for (int i = 0; i < n; i++) out[i] = orc_mt_randbelow(st, (uint32_t)ns[i]);
}

/* ------------------------------------------------------------------------ */
/* numpy pairwise summation (DOUBLE_pairwise_sum, PW_BLOCKSIZE 128)          */
/* ------------------------------------------------------------------------ */
double orc_pairwise_sum(const double *a, long n) {
    if (n < 8) {
        double res = 0.;
        for (long i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8], res;
        long i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        long n2 = n / 2;
        n2 -= n2 % 8;
        return orc_pairwise_sum(a, n2) + orc_pairwise_sum(a + n2, n - n2);
    }
}

/* ------------------------------------------------------------------------ */
/* Environment                                                              */
/* ------------------------------------------------------------------------ */
/* MoveTO (envs/map.py:11-19) */
static const int MOVE_DX[8] = {1, 0, -1, 0, 1, -1, -1, 1};
static const int MOVE_DY[8] = {0, -1, 0, 1, -1, -1, 1, 1};

#define GY(l) ((l)->W + 2)
#define CELL(l, x, y) ((x) * GY(l) + (y))

/* Map.Check_Valid (envs/map.py:85-92) on integer coordinates */
static int check_valid(const orc_layout *l, long x, long y) {
    if (x >= l->L + 1 || x <= 0 || y >= l->W + 1 || y <= 0) return 0;
    return l->valid[CELL(l, x, y)];
}

enum { S_FIRE = 0, S_STEP = 1, S_PEVAC = 2, S_PDEAD = 3 };

/* EvacuationEnv._get_state (envs/evacuation_env.py:84-120) for every robot;
 * robot 0 is centred on Map.robot_position, robot r>0 on robot_positions[r]
 * (EvacuationEnvMulti._get_joint_state, envs/evacuation_env_multi.py:44-53). */
void orc_env_obs(const orc_layout *l, const orc_env *e, double *obs) {
    const int fs = e->scal[S_FIRE];
    const double *dto = l->danger_o + (size_t)fs * l->OX * l->OY;
    for (int r = 0; r < l->R; r++) {
        int cx = r == 0 ? e->view[0] : e->robots[2 * r];
        int cy = r == 0 ? e->view[1] : e->robots[2 * r + 1];
        double *o = obs + (size_t)r * 726;
        for (int i = 0; i < 11; i++)
            for (int j = 0; j < 11; j++) {
                long mx = (long)cx + (i - 5), my = (long)cy + (j - 5);
                double *c = o + (i * 11 + j) * 6;
                int v = check_valid(l, mx, my);
                /* channel 0: space / np.max(space) == finite / inf == 0.0 */
                c[0] = 0.0;
                c[1] = v ? (double)e->rmap[CELL(l, mx, my)] : 0.0;
                long ti = mx - l->ox0, tj = my - l->oy0;
                c[2] = (ti >= 0 && ti < l->OX && tj >= 0 && tj < l->OY) ? dto[ti * l->OY + tj] : 0.0;
                int inb = (mx >= 0 && mx <= l->L + 1 && my >= 0 && my <= l->W + 1);
                c[3] = (!v || (inb && l->barrier[CELL(l, mx, my)])) ? 1.0 : 0.0;
                c[4] = (mx == l->exit_x && my == l->exit_y) ? 1.0 : 0.0;
                c[5] = (i == 5 && j == 5) ? 1.0 : 0.0;
            }
    }
}

/* EvacuationEnv.reset (envs/evacuation_env.py:61-82) + People.__init__
 * placement branch (envs/people.py:183-194) +
 * EvacuationEnvMulti.reset (envs/evacuation_env_multi.py:31-42). */
int orc_env_reset(const orc_layout *l, orc_env *e, double *obs) {
    const int GXY = (l->L + 2) * (l->W + 2);
    e->view[0] = l->reset_view_x;
    e->view[1] = l->reset_view_y;
    memset(e->rmap, 0, (size_t)GXY);
    if (e->thmap) memset(e->thmap, 0, sizeof(int32_t) * GXY);
    const uint32_t nx = (uint32_t)(l->L - 2), ny = (uint32_t)(l->W - 2); /* randint(1, L-2) */
    for (int i = 0; i < l->P; i++) {
        long x = 1 + orc_mt_randbelow(e->py_mt, nx);
        long y = 1 + orc_mt_randbelow(e->py_mt, ny);
        while (!check_valid(l, x, y)) {
            x = 1 + orc_mt_randbelow(e->py_mt, nx);
            y = 1 + orc_mt_randbelow(e->py_mt, ny);
        }
        e->pos[2 * i] = (int32_t)x;
        e->pos[2 * i + 1] = (int32_t)y;
        e->health[i] = 100.0;
        e->acc[i] = 0.0;
        e->flags[i] = 0;
        e->rmap[CELL(l, x, y)] = 1;
        if (e->thmap) e->thmap[CELL(l, x, y)] = 1;
    }
    e->time[0] = 0.0;
    e->scal[S_STEP] = 0;
    e->scal[S_PEVAC] = 0;
    e->scal[S_PDEAD] = 0;
    /* fire models are NOT reset */
    if (l->reset_robots) {
        for (int r = 0; r < l->R; r++) {
            e->robots[2 * r] = l->robot_init[2 * r];
            e->robots[2 * r + 1] = l->robot_init[2 * r + 1];
        }
        e->view[0] = e->robots[0];
        e->view[1] = e->robots[1];
    }
    if (obs) orc_env_obs(l, e, obs);
    return 0;
}

/* Map.move_robot (envs/map.py:160-201) with an integer action */
static void move_robot(const orc_layout *l, orc_env *e, int action, int rid) {
    if (action < 0 || action > 4) return; /* silently ignored, view NOT refreshed */
    long x = e->robots[2 * rid], y = e->robots[2 * rid + 1];
    long nx = x, ny = y;
    if (action == 0) nx = x + 1;
    else if (action == 1) ny = y - 1;
    else if (action == 2) nx = x - 1;
    else if (action == 3) ny = y + 1;
    if (l->rx_lo <= nx && nx <= l->rx_hi && 0 <= ny && ny <= l->W && check_valid(l, nx, ny)) {
        e->robots[2 * rid] = (int32_t)nx;
        e->robots[2 * rid + 1] = (int32_t)ny;
    }
    if (rid == 0) {
        e->view[0] = e->robots[0];
        e->view[1] = e->robots[1];
    }
}

/* Person.update_health (envs/people.py:61-88) */
static void update_health(double *health, uint8_t *flags, double danger, uint32_t *np_mt) {
    if (danger <= 0) return;
    double loss, u;
    if (danger >= 0.8) {
        u = orc_mt_random(np_mt);
        loss = danger * 50.0 + (1.0 + (3.0 - 1.0) * u);
    } else if (danger >= 0.5) {
        u = orc_mt_random(np_mt);
        loss = danger * 40.0 + (0.8 + (2.0 - 0.8) * u);
    } else if (danger >= 0.2) {
        u = orc_mt_random(np_mt);
        loss = danger * 30.0 + (0.5 + (1.5 - 0.5) * u);
    } else {
        u = orc_mt_random(np_mt);
        loss = danger * 20.0 + (0.2 + (1.0 - 0.2) * u);
    }
    if (*health < 50) loss *= 1.2; /* the `elif < 25` branch is unreachable */
    *health -= loss;
    if (*health <= 0) {
        *health = 0;
        *flags |= 2;
    } else if (*health <= 8.0) {
        *flags |= 2;
    }
    if (*health > 100) *health = 100; /* max(0, min(h, 100)) */
    if (*health < 0) *health = 0;
}

/* Person.update_state speed rule (envs/people.py:37-44): a pure function of health */
static double person_speed(double health) {
    if (health < 20) return 0.4;
    double f = 0.3 + 0.7 * (health / 100.0);
    return 1.0 * f;
}

/* People.find_best_direction (envs/people.py:255-297) */
static int find_best_direction(const orc_layout *l, const orc_env *e, long x, long y) {
    int best = -1;
    double max_score = -INFINITY;
    for (int d = 0; d < 8; d++) {
        long nx = x + MOVE_DX[d], ny = y + MOVE_DY[d];
        if (check_valid(l, nx, ny) && e->rmap[CELL(l, nx, ny)] == 0) {
            double delta_p = l->floor[CELL(l, x, y)] - l->floor[CELL(l, nx, ny)];
            double dist = INFINITY;
            for (int r = 0; r < l->R; r++) {
                double dx = (double)(nx - e->robots[2 * r]), dy = (double)(ny - e->robots[2 * r + 1]);
                double dd = sqrt(dx * dx + dy * dy);
                if (dd < dist) dist = dd;
            }
            double effect = 0.0;
            if (dist < l->repel_range) effect = l->repel_k / (dist + 0.1);
            double u = -0.1 + (0.1 - -0.1) * orc_mt_random(e->py_mt);
            double score = delta_p * 5.0 + effect + u;
            if (score > max_score) {
                max_score = score;
                best = d;
            }
        }
    }
    return best;
}

typedef struct {
    int32_t cell;  /* target cell index */
    int n;         /* movers */
    int first;     /* index into mover list */
} target_t;

/* per-thread planner workspace, allocated once per batch (not per step) */
typedef struct {
    int *tgt_of;      /* [GXY] cell -> target slot or -1 */
    int *mover_next;  /* [P] */
    double *scratch;  /* [P] */
    target_t *targets;
    int *mover;
    int *mover_tail;
} orc_work;

static int work_alloc(const orc_layout *l, orc_work *w) {
    const int GXY = (l->L + 2) * (l->W + 2);
    const int P1 = l->P > 0 ? l->P : 1;
    w->tgt_of = (int *)malloc(sizeof(int) * GXY);
    w->mover_next = (int *)malloc(sizeof(int) * P1);
    w->scratch = (double *)malloc(sizeof(double) * P1);
    w->targets = (target_t *)malloc(sizeof(target_t) * P1);
    w->mover = (int *)malloc(sizeof(int) * P1);
    w->mover_tail = (int *)malloc(sizeof(int) * P1);
    if (!w->tgt_of || !w->mover_next || !w->scratch || !w->targets || !w->mover || !w->mover_tail) return -12;
    for (int c = 0; c < GXY; c++) w->tgt_of[c] = -1;
    return 0;
}

static void work_free(orc_work *w) {
    free(w->tgt_of);
    free(w->mover_next);
    free(w->scratch);
    free(w->targets);
    free(w->mover);
    free(w->mover_tail);
}

/* People.run (envs/people.py:196-253) including execute_move (:299-314) */
static void people_run(const orc_layout *l, orc_env *e, orc_work *wk) {
    const int P = l->P;
    const int GXY = (l->L + 2) * (l->W + 2);
    const int fs = e->scal[S_FIRE];
    const double *dp = l->danger_p + (size_t)fs * GXY;
    /* 1. health (map.get_fire_danger at the person's centre) */
    for (int i = 0; i < P; i++) {
        if (!(e->flags[i] & 3)) {
            double danger = dp[CELL(l, e->pos[2 * i], e->pos[2 * i + 1])];
            update_health(&e->health[i], &e->flags[i], danger, e->np_mt);
        }
    }
    /* 2. plan against the rmap snapshot; move_plan keeps dict insertion order */
    int ntargets = 0;
    int *cell_target = wk->tgt_of; /* [GXY] -> target slot or -1 (all -1 between calls) */
    int *mover_next = wk->mover_next;
    target_t *targets = wk->targets;
    int *mover = wk->mover;
    int *mover_tail = wk->mover_tail;
    for (int i = 0; i < P; i++) {
        if (e->flags[i] & 3) continue;
        e->acc[i] += person_speed(e->health[i]) * 0.5;
        if (e->acc[i] >= 1.0) {
            e->acc[i] -= 1.0;
            long x = e->pos[2 * i], y = e->pos[2 * i + 1];
            int d = find_best_direction(l, e, x, y);
            if (d >= 0) {
                int c = CELL(l, x + MOVE_DX[d], y + MOVE_DY[d]);
                int t = cell_target[c];
                if (t < 0) {
                    t = ntargets++;
                    cell_target[c] = t;
                    targets[t].cell = c;
                    targets[t].n = 0;
                    targets[t].first = i;
                    mover_tail[t] = i;
                } else {
                    mover_next[mover_tail[t]] = i;
                    mover_tail[t] = i;
                }
                mover_next[i] = -1;
                targets[t].n++;
            }
        }
    }
    /* 4. execute in insertion order; random.shuffle picks the winner */
    for (int t = 0; t < ntargets; t++) {
        int n = targets[t].n;
        int k = 0;
        for (int m = targets[t].first; m >= 0; m = mover_next[m]) mover[k++] = m;
        for (int i = n - 1; i >= 1; i--) { /* random.shuffle (Lib/random.py, 3.10) */
            int j = (int)orc_mt_randbelow(e->py_mt, (uint32_t)(i + 1));
            int tmp = mover[i];
            mover[i] = mover[j];
            mover[j] = tmp;
        }
        int w = mover[0];
        int c = targets[t].cell;
        int oc = CELL(l, e->pos[2 * w], e->pos[2 * w + 1]);
        e->rmap[oc] = 0;
        e->rmap[c] = 1;
        e->pos[2 * w] = c / GY(l);
        e->pos[2 * w + 1] = c % GY(l);
        if (e->thmap) e->thmap[c] += 1;
        if (l->exitm[c]) {
            e->flags[w] |= 1;
            e->rmap[c] = 0;
        }
        if (e->thmap)
            for (int m = 1; m < n; m++)
                e->thmap[CELL(l, e->pos[2 * mover[m]], e->pos[2 * mover[m] + 1])] += 1;
    }
    for (int t = 0; t < ntargets; t++) cell_target[targets[t].cell] = -1;
}

/* EvacuationEnv._calculate_reward (envs/evacuation_env.py:174-288) */
static double calc_reward(const orc_layout *l, orc_env *e, double *scratch) {
    const int P = l->P;
    double reward = 0;
    const double rx = (double)e->view[0], ry = (double)e->view[1];
    int evac = 0, dead = 0;
    for (int i = 0; i < P; i++) {
        evac += e->flags[i] & 1;
        dead += (e->flags[i] >> 1) & 1;
    }
    int remaining = P - evac - dead;
    int new_evac = evac - e->scal[S_PEVAC];
    reward += new_evac * l->evac_reward;
    double gq = 0;
    for (int i = 0; i < P; i++) {
        if (e->flags[i] & 3) continue;
        double px = e->pos[2 * i] + 0.5, py = e->pos[2 * i + 1] + 0.5;
        double dx = px - rx, dy = py - ry;
        double d = sqrt(dx * dx + dy * dy);
        if (d <= 5) {
            double ex = px - (double)l->exit_x, ey = py - (double)l->exit_y;
            double de = sqrt(ex * ex + ey * ey);
            if (de > 20) gq += 2.0;
            else if (de > 10) gq += 1.5;
            else gq += 1.0;
            if (e->health[i] < 80) gq += 1.0;
        }
    }
    reward += gq;
    if (remaining > 0) {
        long n = 0;
        for (int i = 0; i < P; i++) {
            if (e->flags[i] & 3) continue;
            double dx = rx - (e->pos[2 * i] + 0.5), dy = ry - (e->pos[2 * i + 1] + 0.5);
            scratch[n++] = sqrt(dx * dx + dy * dy);
        }
        double avg = orc_pairwise_sum(scratch, n) / (double)n;
        double dr = 2.0 - fabs(avg - 8.0) * 0.2;
        reward += dr > 0 ? dr : 0; /* max(0, ...) */
    }
    if (remaining > 0) {
        double urgency = (double)remaining / (double)P;
        reward += -0.05 - (urgency * 0.1);
    } else {
        reward -= 0.02;
    }
    if (P - dead > 0) {
        double total = 0.0;
        for (int i = 0; i < P; i++)
            if (!(e->flags[i] & 2)) total += e->health[i];
        double avg_h = total / (double)(P - dead);
        reward += (avg_h - 90) * 0.05;
    }
    if (evac == P) {
        int tb = 300 - e->scal[S_STEP];
        double time_bonus = (tb > 0 ? tb : 0) * 0.2;
        if (P > 0) {
            double s = 0.0;
            for (int i = 0; i < P; i++) s += e->health[i];
            double fah = s / (double)P;
            reward += 100 + time_bonus + (fah - 80) * 1.0;
        } else {
            reward += 100 + time_bonus;
        }
    }
    int new_deaths = dead - e->scal[S_PDEAD];
    reward -= new_deaths * l->death_penalty;
    reward -= dead * l->death_acc_penalty;
    reward += (P - dead) * l->alive_bonus;
    if (e->scal[S_STEP] > 0) {
        double eff = (double)evac / (double)e->scal[S_STEP];
        if (eff > 0.1) reward += eff * 5;
    }
    e->scal[S_PEVAC] = evac;
    e->scal[S_PDEAD] = dead;
    return reward;
}

static int env_step_impl(const orc_layout *l, orc_env *e, const int32_t *actions, double *reward,
                         int32_t *done, double *obs, orc_work *wk) {
    /* EvacuationEnv.step (envs/evacuation_env.py:122-172) /
     * EvacuationEnvMulti.step (envs/evacuation_env_multi.py:55-89) */
    for (int r = 0; r < l->R; r++) move_robot(l, e, actions[r], r);
    people_run(l, e, wk);
    if (e->scal[S_FIRE] < l->t_max) e->scal[S_FIRE] += 1; /* both fire models */
    *reward = calc_reward(l, e, wk->scratch);
    e->time[0] += 0.5;
    e->scal[S_STEP] += 1;
    int evac = 0, dead = 0;
    for (int i = 0; i < l->P; i++) {
        evac += e->flags[i] & 1;
        dead += (e->flags[i] >> 1) & 1;
    }
    *done = (evac + dead == l->P) || (e->time[0] >= 600);
    if (obs) orc_env_obs(l, e, obs);
    return 0;
}

int orc_env_step(const orc_layout *l, orc_env *e, const int32_t *actions, double *reward,
                 int32_t *done, double *obs) {
    orc_work wk;
    if (work_alloc(l, &wk)) {
        work_free(&wk);
        return -12;
    }
    int rc = env_step_impl(l, e, actions, reward, done, obs, &wk);
    work_free(&wk);
    return rc;
}

long orc_run_batch(const orc_layout *l, orc_env *envs, int E, int steps, const int32_t *actions,
                   double *reward_sum, int nthreads) {
    long total = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel reduction(+ : total)
    {
        orc_work wk;
        const int ok = work_alloc(l, &wk) == 0;
#pragma omp for schedule(dynamic, 1)
        for (int ei = 0; ei < E; ei++) {
            double acc_r = 0.0;
            for (int s = 0; s < steps && ok; s++) {
                double r;
                int32_t d;
                env_step_impl(l, &envs[ei], actions + ((size_t)s * E + ei) * l->R, &r, &d, NULL, &wk);
                acc_r += r;
                total++;
                if (d) orc_env_reset(l, &envs[ei], NULL);
            }
            if (reward_sum) reward_sum[ei] = acc_r;
        }
        work_free(&wk);
    }
    return total;
}
