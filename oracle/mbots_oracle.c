/*
 * mbots_oracle.c -- TEST INFRASTRUCTURE ONLY (see mbots_oracle.h).
 *
 * Serial-per-world C restatement of the reference step graph
 * (src/sim/sim.cpp:1061-1220) used as the parity oracle and CPU baseline.
 * Compile with -ffp-contract=off and no fast-math: every float expression is
 * written in the reference's evaluation order and must round identically to
 * the HIP kernels.  Parity of RNG / math / sensor is unpinned (Madrona absent);
 * they follow DESIGN.md section 3.
 */
#include "mbots_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Counter RNG.  Madrona's rand::initKey/split_i/RNG (sim.cpp:1238-1239,     */
/* mgr.cpp:105) is not vendored; the build uses Threefry-2x32-20 (Random123)  */
/* with the same call structure: world key = split(initKey(seed), 0, world),  */
/* one 32-bit draw per counter value.                                         */
/* ------------------------------------------------------------------------ */
static inline uint32_t rotl32(uint32_t x, unsigned r) { return (x << r) | (x >> (32u - r)); }

void orc_threefry2x32(const uint32_t key[2], const uint32_t ctr[2], uint32_t out[2])
{
    static const unsigned R[8] = {13, 15, 26, 6, 17, 29, 16, 24};
    uint32_t ks[3] = {key[0], key[1], 0x1BD11BDAu ^ key[0] ^ key[1]};
    uint32_t x0 = ctr[0] + ks[0];
    uint32_t x1 = ctr[1] + ks[1];
    for (unsigned r = 0; r < 20; ++r) {
        x0 += x1;
        x1 = rotl32(x1, R[r & 7u]);
        x1 ^= x0;
        if ((r & 3u) == 3u) {
            unsigned s = (r + 1u) >> 2;
            x0 += ks[s % 3u];
            x1 += ks[(s + 1u) % 3u] + s;
        }
    }
    out[0] = x0;
    out[1] = x1;
}

float orc_sample_uniform(uint32_t bits) { return (float)(bits >> 8) * (1.0f / 16777216.0f); }

int32_t orc_sample_i32(uint32_t bits, int32_t a, int32_t b)
{
    uint32_t range = (uint32_t)(b - a);
    return a + (int32_t)(((uint64_t)bits * (uint64_t)range) >> 32);
}

uint32_t orc_action_hash(uint32_t seed, uint32_t step, uint32_t gworld, uint32_t slot)
{
    uint32_t k[2] = {seed, step}, c[2] = {gworld, slot}, o[2];
    orc_threefry2x32(k, c, o);
    return o[0];
}

/* ------------------------------------------------------------------------ */
/* State                                                                     */
/* ------------------------------------------------------------------------ */
typedef struct {
    float x, y;          /* base::Position.xy (z is always 1)                  */
    float rw, rz;        /* base::Rotation (rotations are about +z only)       */
    int32_t species;     /* Species (1..4)                                     */
    int32_t health;      /* Health                                             */
    int32_t accum;       /* HealthAccumulator                                  */
    int32_t finder;      /* FinderOutput.hitEntity -> slot, -1 = none          */
    int32_t stats[4];    /* AgentStats                                         */
    float sur[2];        /* SurroundingObservation                             */
    int32_t action[6];   /* Action (copied from obs row in actionSystem)       */
    int32_t obs_row;     /* AgentObservationBridge -> export row, -1 = new     */
    int32_t alive;
} orc_agent;

typedef struct {
    uint32_t key[2];
    uint32_t ctr;
    int32_t cur_food;                       /* Sim::currentNumFood            */
    uint8_t pkg_x[ORC_NUM_CHUNKS][ORC_MAX_PKG];
    uint8_t pkg_y[ORC_NUM_CHUNKS][ORC_MAX_PKG];
    uint32_t pkg_n[ORC_NUM_CHUNKS][ORC_MAX_PKG];
    uint32_t pkg_rot[ORC_NUM_CHUNKS][ORC_MAX_PKG];  /* food entity rotation, 22-bit quarter turn */
    uint32_t num_agents[ORC_NUM_CHUNKS];    /* ChunkInfo::numAgents           */
    uint32_t total_speed[ORC_NUM_CHUNKS];   /* ChunkInfo::totalSpeed          */
    int32_t n;
    orc_agent *ag;                          /* [cap]                          */
    orc_agent *tmp;                         /* [cap]                          */
    float species_reward[ORC_NUM_SPECIES];  /* SpeciesReward                  */
    int32_t species_count[ORC_NUM_SPECIES];
    uint32_t overflow;
} orc_world;

typedef struct {
    int32_t *species;
    float *pos;
    int32_t *health;
    float *sur;
    float *reward;
    int32_t *action;
    int32_t *stats;
    float *hidden;
    int8_t *sem;
    uint8_t *depth;
} orc_cols;

struct orc_sim {
    orc_config cfg;
    orc_world *w;
    orc_cols cur[2], prev[2];   /* double-buffered export table            */
    int tb;                      /* index of the live table                  */
    int32_t *species_count;      /* [W][4] exported                          */
    int32_t *world_off;          /* [W] world-major offsets                  */
    int32_t *row_base;           /* [W][4] first export row per (world,sp)   */
    uint32_t total;
};

static const float kLx = 128.0f, kLy = 96.0f;   /* sim.cpp:161-166 */

static inline uint32_t draw(orc_world *w)
{
    uint32_t c[2] = {w->ctr++, 0u}, o[2];
    orc_threefry2x32(w->key, c, o);
    return o[0];
}
static inline float sample_uniform(orc_world *w) { return orc_sample_uniform(draw(w)); }
static inline int32_t sample_i32(orc_world *w, int32_t a, int32_t b) { return orc_sample_i32(draw(w), a, b); }

/* std::min / std::max as the reference's <algorithm> defines them. */
static inline float fmin_std(float a, float b) { return (b < a) ? b : a; }
static inline float fmax_std(float a, float b) { return (a < b) ? b : a; }

/* Sim::getChunkIndex (sim.inl:49-62) */
static inline int32_t chunk_index(float cx, float cy)
{
    int32_t x = (int32_t)cx, y = (int32_t)cy;
    if (x < 0 || y < 0 || x >= ORC_CHUNKS_X || y >= ORC_CHUNKS_Y) return -1;
    return x + y * ORC_CHUNKS_X;
}

/* Quat::rotateVec({1,0,0}) for a z-only quaternion then normalize()
 * (sim.cpp:466-468): (1 - 2 z^2, 2 w z) / |.|                               */
static inline void heading(float w, float z, float *dx, float *dy)
{
    float vx = 1.0f - 2.0f * (z * z);
    float vy = 2.0f * (z * w);
    float len = sqrtf(vx * vx + vy * vy);
    *dx = vx / len;
    *dy = vy / len;
}

/* Quat::angleAxis(+-0.1, z): (cos 0.05, 0, 0, +-sin 0.05) as correctly rounded
 * floats; host and device cosf/sinf differ, so the literals are fixed.       */
static const float kRotC = 0.99875026039496624f;
static const float kRotS = 0.04997916927067833f;

static void agent_init(orc_agent *a, float x, float y, int32_t species, int32_t health)
{
    memset(a, 0, sizeof(*a));
    a->x = x;
    a->y = y;
    a->rw = 1.0f;   /* Quat::angleAxis(0, z) (sim.cpp:206-207) */
    a->rz = 0.0f;
    a->species = species;
    a->health = health;
    a->accum = health;
    a->finder = -1;
    a->obs_row = -1;
    a->alive = 1;
}

/* ------------------------------------------------------------------------ */
/* Table allocation                                                          */
/* ------------------------------------------------------------------------ */
static int cols_alloc(orc_cols *c, size_t rows)
{
    c->species = calloc(rows, 4);
    c->pos = calloc(rows * 2, 4);
    c->health = calloc(rows, 4);
    c->sur = calloc(rows * 2, 4);
    c->reward = calloc(rows, 4);
    c->action = calloc(rows * 6, 4);
    c->stats = calloc(rows * 4, 4);
    c->hidden = calloc(rows * ORC_HIDDEN, 4);
    c->sem = calloc(rows * ORC_SENSOR, 1);
    c->depth = calloc(rows * ORC_SENSOR, 1);
    return c->species && c->pos && c->health && c->sur && c->reward && c->action &&
           c->stats && c->hidden && c->sem && c->depth;
}
static void cols_free(orc_cols *c)
{
    free(c->species); free(c->pos); free(c->health); free(c->sur); free(c->reward);
    free(c->action); free(c->stats); free(c->hidden); free(c->sem); free(c->depth);
}

/* ------------------------------------------------------------------------ */
/* Parallel world loop                                                       */
/* ------------------------------------------------------------------------ */
typedef void (*world_fn)(orc_sim *, uint32_t);
typedef struct { orc_sim *s; world_fn fn; uint32_t lo, hi; } job_t;
static void *job_run(void *p)
{
    job_t *j = (job_t *)p;
    for (uint32_t w = j->lo; w < j->hi; ++w) j->fn(j->s, w);
    return NULL;
}
static void for_worlds(orc_sim *s, world_fn fn)
{
    uint32_t W = s->cfg.num_worlds, T = s->cfg.num_threads ? s->cfg.num_threads : 1;
    if (T > W) T = W ? W : 1;
    if (T <= 1) {
        for (uint32_t w = 0; w < W; ++w) fn(s, w);
        return;
    }
    pthread_t th[256];
    job_t jobs[256];
    if (T > 256) T = 256;
    for (uint32_t t = 0; t < T; ++t) {
        jobs[t].s = s; jobs[t].fn = fn;
        jobs[t].lo = (uint32_t)((uint64_t)W * t / T);
        jobs[t].hi = (uint32_t)((uint64_t)W * (t + 1) / T);
        pthread_create(&th[t], NULL, job_run, &jobs[t]);
    }
    for (uint32_t t = 0; t < T; ++t) pthread_join(th[t], NULL);
}

/* ------------------------------------------------------------------------ */
/* Step systems (sim.cpp:1061-1181), one world at a time                     */
/* ------------------------------------------------------------------------ */

/* addFoodToChunk (sim.cpp:308-361) */
static int add_food_to_chunk(orc_world *w, int chunk)
{
    (void)sample_i32(w, 0, ORC_CHUNK_W);   /* sim.cpp:311-312: unused draws */
    (void)sample_i32(w, 0, ORC_CHUNK_W);
    for (int i = 0; i < ORC_MAX_PKG; ++i) {
        if (w->pkg_n[chunk][i] == 0) {
            uint32_t rx = (uint32_t)sample_i32(w, 0, ORC_CHUNK_W);
            uint32_t ry = (uint32_t)sample_i32(w, 0, ORC_CHUNK_W);
            w->pkg_x[chunk][i] = (uint8_t)rx;
            w->pkg_y[chunk][i] = (uint8_t)ry;
            w->pkg_n[chunk][i] = 1;
            /* food entity rotation angleAxis(2 pi U, z) (sim.cpp:338-341): the
             * cube is symmetric under quarter turns, so 4U mod 1 -- the low 22
             * bits of U's 24 -- fixes it */
            w->pkg_rot[chunk][i] = (draw(w) >> 8) & 0x3FFFFFu;
            return 1;
        }
        /* numFood < kMaxFoodPerPackage (=1) never holds for a full package */
    }
    return 0;
}

/* addFoodSystem (sim.cpp:363-387) */
static void add_food(orc_world *w)
{
    if (sample_i32(w, 0, 10) == 0) {
        uint32_t n = (uint32_t)sample_i32(w, 1, 3);
        uint32_t diff = (uint32_t)ORC_FOOD_CAP - (uint32_t)w->cur_food;
        if (diff < n) n = diff;
        for (uint32_t i = 0; i < n; ++i) {
            uint32_t cx = (uint32_t)sample_i32(w, 0, ORC_CHUNKS_X);
            uint32_t cy = (uint32_t)sample_i32(w, 0, ORC_CHUNKS_Y);
            if (add_food_to_chunk(w, (int)(cx + cy * ORC_CHUNKS_X))) w->cur_food += 1;
        }
    }
}

/* actionSystem (sim.cpp:419-502) */
static void action_system(orc_sim *s, orc_world *w, orc_agent *a)
{
    const orc_cols *cur = &s->cur[s->tb];
    if (a->obs_row >= 0) memcpy(a->action, cur->action + (size_t)a->obs_row * 6, 24);
    else memset(a->action, 0, 24);

    if (a->action[4] && a->finder >= 0) {                 /* shoot :434-454 */
        orc_agent *t = &w->ag[a->finder];
        t->accum += -50;
        if (t->species == a->species) a->stats[0] = 1;
        else a->stats[1] = 1;
    }
    if (a->action[2]) {                                   /* :456-462 */
        float nw = a->rw * kRotC - a->rz * kRotS;
        float nz = a->rw * kRotS + a->rz * kRotC;
        a->rw = nw; a->rz = nz;
    } else if (a->action[3]) {
        float nw = a->rw * kRotC - a->rz * (-kRotS);
        float nz = a->rw * (-kRotS) + a->rz * kRotC;
        a->rw = nw; a->rz = nz;
    }
    float ox = a->x, oy = a->y, dx, dy;
    heading(a->rw, a->rz, &dx, &dy);
    if (a->action[0]) { a->x = a->x + dx; a->y = a->y + dy; }
    else if (a->action[1]) { a->x = a->x - dx; a->y = a->y - dy; }
    a->x = fmin_std(kLx - 1.0f, fmax_std(0.0f, a->x));    /* :485-486 */
    a->y = fmin_std(kLy - 1.0f, fmax_std(0.0f, a->y));
    float ddx = a->x - ox, ddy = a->y - oy;
    float len = sqrtf(ddx * ddx + ddy * ddy);
    /* getChunkCoord (sim.inl:39-47) + getChunkIndex */
    float ccx = floorf((a->x / 1.0f) / 16.0f), ccy = floorf((a->y / 1.0f) / 16.0f);
    int32_t ci = chunk_index(ccx, ccy);
    w->num_agents[ci] += 1u;
    w->total_speed[ci] += (uint32_t)(len * 2.0f);
}

/* healthSync (sim.cpp:505-581); returns nothing, may append a child */
static void health_sync(orc_world *w, uint32_t cap, int32_t i)
{
    orc_agent *a = &w->ag[i];
    int32_t h = a->accum;
    {
        float chx = (a->x / 1.0f) / 16.0f, chy = (a->y / 1.0f) / 16.0f;
        uint8_t cx = (uint8_t)(16.0f * (chx - floorf(chx)));
        uint8_t cy = (uint8_t)(16.0f * (chy - floorf(chy)));
        int32_t ci = chunk_index(chx, chy);
        for (int k = 0; k < ORC_MAX_PKG; ++k) {
            if (w->pkg_x[ci][k] == cx && w->pkg_y[ci][k] == cy) {
                /* FoodPackage::consume (sim.inl:76-99), serial = lowest slot first */
                if (w->pkg_n[ci][k] != 0) {
                    w->pkg_n[ci][k] -= 1;
                    if (w->pkg_n[ci][k] == 0) w->cur_food -= 1;
                    h = (int32_t)((float)h + 20.0f);
                    a->stats[2] = 1;
                    break;
                }
            }
        }
    }
    if (a->action[5] && h > 10 && a->finder >= 0) {       /* breed :547-569 */
        if (w->ag[a->finder].species == a->species) {
            h -= 40;
            if ((uint32_t)w->n < cap) {
                agent_init(&w->ag[w->n], a->x, a->y, a->species, 50);
                w->n += 1;
            } else {
                w->overflow += 1;
            }
            a->stats[3] = 1;
        }
    }
    if (h <= 0) a->alive = 0;                              /* :574-578 */
    a->health = h;
    a->accum = h;
}

/* updateSurroundingObservation (sim.cpp:583-654) */
static void surrounding(orc_world *w, orc_agent *a)
{
    float cpx = a->x / 1.0f, cpy = a->y / 1.0f;
    cpx = cpx - 16.0f * 0.5f;
    cpy = cpy - 16.0f * 0.5f;
    float chx = cpx / 16.0f, chy = cpy / 16.0f;
    float x0 = floorf(chx), y0 = floorf(chy), x1 = ceilf(chx), y1 = ceilf(chy);
    int32_t i00 = chunk_index(x0, y0), i10 = chunk_index(x1, y0);
    int32_t i01 = chunk_index(x0, y1), i11 = chunk_index(x1, y1);
    float xi = chx - x0, yi = chy - y0;
    float n00 = i00 >= 0 ? (float)w->num_agents[i00] : 0.0f;
    float n10 = i10 >= 0 ? (float)w->num_agents[i10] : 0.0f;
    float n01 = i01 >= 0 ? (float)w->num_agents[i01] : 0.0f;
    float n11 = i11 >= 0 ? (float)w->num_agents[i11] : 0.0f;
    float s00 = i00 >= 0 ? (float)w->total_speed[i00] : 0.0f;
    float s10 = i10 >= 0 ? (float)w->total_speed[i10] : 0.0f;
    float s01 = i01 >= 0 ? (float)w->total_speed[i01] : 0.0f;
    float s11 = i11 >= 0 ? (float)w->total_speed[i11] : 0.0f;
    float nx0 = xi * n10 + (1.0f - xi) * n00;
    float nx1 = xi * n11 + (1.0f - xi) * n01;
    float sx0 = xi * s10 + (1.0f - xi) * s00;
    float sx1 = xi * s11 + (1.0f - xi) * s01;
    a->sur[0] = yi * nx1 + (1.0f - yi) * nx0;
    a->sur[1] = yi * sx1 + (1.0f - yi) * sx0;
}

static void world_phase_a(orc_sim *s, uint32_t wi)
{
    orc_world *w = &s->w[wi];
    const uint32_t A = s->cfg.init_agents, cap = s->cfg.cap;

    memset(w->num_agents, 0, sizeof(w->num_agents));       /* resetChunkInfoSystem :390-397 */
    memset(w->total_speed, 0, sizeof(w->total_speed));
    add_food(w);                                           /* :363-387 */

    const int32_t n0 = w->n;
    for (int32_t i = 0; i < n0; ++i) memset(w->ag[i].stats, 0, 16);
    for (int32_t i = 0; i < n0; ++i) action_system(s, w, &w->ag[i]);
    for (int32_t i = 0; i < n0; ++i) health_sync(w, cap, i);
    for (int32_t i = 0; i < w->n; ++i)                     /* children included */
        if (w->ag[i].alive) surrounding(w, &w->ag[i]);

    /* speciesTrackerUpdate (:719-734) */
    uint32_t cnt[ORC_NUM_SPECIES] = {0}, hsum[ORC_NUM_SPECIES] = {0};
    for (int32_t i = 0; i < w->n; ++i) {
        if (!w->ag[i].alive) continue;
        cnt[w->ag[i].species - 1] += 1u;
        hsum[w->ag[i].species - 1] += (uint32_t)w->ag[i].health;
    }
    /* speciesInfoSync (:791-838) */
    const uint32_t per_species = A / ORC_NUM_SPECIES;
    for (int i = 0; i < ORC_NUM_SPECIES; ++i) {
        uint32_t count = cnt[i];
        float avg = (float)hsum[i] / (float)count;
        if (count == 0) avg = 0.0f;
        w->species_reward[i] = (float)count / (float)A + avg / 100.0f - 2.0f;
        if (count < per_species) {
            for (uint32_t e = count; e < per_species; ++e) {
                float x = sample_uniform(w) * kLx;
                float y = sample_uniform(w) * kLy;
                if ((uint32_t)w->n < cap) {
                    agent_init(&w->ag[w->n], x, y, i + 1, 100);
                    w->n += 1;
                } else {
                    w->overflow += 1;
                }
            }
        }
    }
    /* SortArchetypeNode<Agent, WorldID> (:1129): drop dead rows, keep order */
    int32_t m = 0;
    for (int32_t i = 0; i < w->n; ++i) {
        if (w->ag[i].alive) w->tmp[m++] = w->ag[i];
    }
    /* remap finder slots is unnecessary: the sensor recomputes them below */
    orc_agent *t = w->ag; w->ag = w->tmp; w->tmp = t;
    w->n = m;
    for (int i = 0; i < ORC_NUM_SPECIES; ++i) w->species_count[i] = 0;
    for (int32_t i = 0; i < m; ++i) w->species_count[w->ag[i].species - 1] += 1;
}

/* Global (species, world, slot) row order: SortArchetypeNode<Obs, Species>
 * (:1147-1149) made deterministic. */
static void compute_rows(orc_sim *s)
{
    uint32_t W = s->cfg.num_worlds;
    int32_t base = 0;
    for (int sp = 0; sp < ORC_NUM_SPECIES; ++sp)
        for (uint32_t w = 0; w < W; ++w) {
            s->row_base[w * 4 + sp] = base;
            base += s->w[w].species_count[sp];
            s->species_count[w * 4 + sp] = s->w[w].species_count[sp];
        }
    s->total = (uint32_t)base;
    int32_t off = 0;
    for (uint32_t w = 0; w < W; ++w) { s->world_off[w] = off; off += s->w[w].n; }
}

/* updateObservations (:687-717) + updateSensorOutputIdx (:736-789) +
 * rewardSystem (:840-983, setting 8) into the other table. */
static void world_phase_c(orc_sim *s, uint32_t wi)
{
    orc_world *w = &s->w[wi];
    const orc_cols *oc = &s->cur[s->tb], *op = &s->prev[s->tb];
    orc_cols *nc = &s->cur[s->tb ^ 1], *np = &s->prev[s->tb ^ 1];
    int32_t rank[ORC_NUM_SPECIES] = {0};
    /* SpeciesReward row of the next world (B.3 faithful off-by-one) */
    const uint32_t W = s->cfg.num_worlds;
    float next_r0 = 0.0f;
    if (wi + 1 < W) {
        /* reward of the next world is final after phase A of every world */
        next_r0 = s->w[wi + 1].species_reward[0];
    }
    for (int32_t i = 0; i < w->n; ++i) {
        orc_agent *a = &w->ag[i];
        int sp = a->species - 1;
        size_t r = (size_t)(s->row_base[wi * 4 + sp] + rank[sp]++);
        nc->species[r] = a->species;
        nc->pos[r * 2] = a->x;
        nc->pos[r * 2 + 1] = a->y;
        nc->health[r] = a->health;
        nc->sur[r * 2] = a->sur[0];
        nc->sur[r * 2 + 1] = a->sur[1];
        memcpy(nc->stats + r * 4, a->stats, 16);
        if (a->obs_row >= 0) {
            size_t o = (size_t)a->obs_row;
            memcpy(nc->action + r * 6, oc->action + o * 6, 24);
            memcpy(nc->hidden + r * ORC_HIDDEN, oc->hidden + o * ORC_HIDDEN, 4 * ORC_HIDDEN);
            np->species[r] = op->species[o];
            memcpy(np->pos + r * 2, op->pos + o * 2, 8);
            np->health[r] = op->health[o];
            memcpy(np->sur + r * 2, op->sur + o * 2, 8);
            np->reward[r] = op->reward[o];
            memcpy(np->action + r * 6, op->action + o * 6, 24);
            memcpy(np->stats + r * 4, op->stats + o * 4, 16);
            memcpy(np->hidden + r * ORC_HIDDEN, op->hidden + o * ORC_HIDDEN, 4 * ORC_HIDDEN);
            memcpy(np->sem + r * ORC_SENSOR, oc->sem + o * ORC_SENSOR, ORC_SENSOR);
            memcpy(np->depth + r * ORC_SENSOR, oc->depth + o * ORC_SENSOR, ORC_SENSOR);
        } else {
            memset(nc->action + r * 6, 0, 24);
            memset(nc->hidden + r * ORC_HIDDEN, 0, 4 * ORC_HIDDEN);
            np->species[r] = 0;
            memset(np->pos + r * 2, 0, 8);
            np->health[r] = 0;
            memset(np->sur + r * 2, 0, 8);
            np->reward[r] = 0.0f;
            memset(np->action + r * 6, 0, 24);
            memset(np->stats + r * 4, 0, 16);
            memset(np->hidden + r * ORC_HIDDEN, 0, 4 * ORC_HIDDEN);
            memset(np->sem + r * ORC_SENSOR, 0, ORC_SENSOR);
            memset(np->depth + r * ORC_SENSOR, 0, ORC_SENSOR);
        }
        /* rewardSystem, setting 8 (:942-956) */
        float sr;
        if (s->cfg.reward_fixed) sr = w->species_reward[sp];
        else sr = (a->species < ORC_NUM_SPECIES) ? w->species_reward[a->species] : next_r0;
        float rew = sr + (float)a->health / 100.0f - 0.5f;
        if (a->stats[2]) rew += 10.0f;
        if (a->stats[3]) rew += 10.0f;
        if (a->stats[1]) rew += 15.0f;
        nc->reward[r] = rew;
        memset(a->stats, 0, 16);
        a->obs_row = (int32_t)r;
    }
}

/* ------------------------------------------------------------------------ */
/* Sensor (Madrona RenderingSystem raycast; build-defined spec)*/
/*                                                                           */
/* 32 pinhole pixels per agent (24 forward over the 90-degree FOV, 8 backward,*/
/* gfx.cpp:252-253) plus the forward centre "finder" ray, cast horizontally   */
/* from the agent's centre (attachEntityToView offset {0,0,0}, sim.cpp:221)   */
/* and seeing only what lies beyond nearSphere = 1.1 from it (mgr.cpp:133):   */
/* a ray hits an object iff it leaves the object at distance >= 1.1.  Other   */
/* agents are circles of radius 0.92 (agent_render.obj's cross-section in the */
/* rays' plane, z = 0 of the mesh: radii 0.910-0.921); food packages are the  */
/* +-1 cube_render.obj boxes rotated about z (raster_box).  In the agent's    */
/* frame (f along the heading h, l along r = (hy, -hx)) ray k runs along      */
/* (1, u) forward / -(1, u) backward; its near point P0 = 1.1 (1, u)/|(1, u)| */
/* (the ray parameter s0 = 1.1 / |(1, u)| along it).  Depth is view-space z   */
/* (one per object): f - 0.92 for circles, the nearest corner's for squares   */
/* (clamped at 0, 14-bit mantissa: zq); walls: the ray's exit from the inner  */
/* arena rectangle when P0 lies in it, s0 when P0 lies inside a wall box, no  */
/* wall (a miss: semantic -1, depth 255) when P0 lies beyond the walls.  Each */
/* pixel takes the lexicographic minimum of (z, order): walls 0, food 1 + k,  */
/* agents 64 + slot.                                                         */
/* ------------------------------------------------------------------------ */
static const float kInLo = 0.0f + 0.2f;     /* walls: makeWalls (sim.cpp:157-194), */
static const float kInHiX = 128.0f - 0.2f;  /* 0.2-thick boxes on the boundary    */
static const float kInHiY = 96.0f - 0.2f;
static const float kOutLo = 0.0f - 0.2f;    /* the boxes' outer faces             */
static const float kOutHiX = 128.0f + 0.2f;
static const float kOutHiY = 96.0f + 0.2f;
static const float kNearSphere = 1.1f;      /* mgr.cpp:133                        */
static const float kAgentR = 0.92f;         /* agent disc radius in the ray plane */
static const float kAgentR2 = 0.8464f;      /* kAgentR^2                          */

/* pixel k's offset u = (2k + 1) / 24 - 1 (forward, k < 24) or
 * (2(k - 24) + 1) / 8 - 1 (backward), as one rounding: (2k - 23) * (1/24),
 * (2(k - 24) - 7) / 8 (exact); the finder ray (k = 32) has u = 0 */
static float ray_u(int k)
{
    if (k < 24) return (float)(2 * k - 23) * (1.0f / 24.0f);
    if (k < ORC_SENSOR) return (float)(2 * (k - 24) - 7) * 0.125f;
    return 0.0f;
}

/* ray k's near point in the agent frame, (c, s) = 1.1 (1, u) / sqrt(1 + u^2)
 * (c is also the ray parameter s0 of that point), and e = 1.1 sqrt(1 + u^2) */
static void near_pt(int k, float *c, float *s, float *e)
{
    float u = ray_u(k);
    float n = sqrtf(1.0f + u * u);
    *c = kNearSphere / n;
    *s = u * *c;
    *e = kNearSphere * n;
}

/* ray direction k of heading (hx, hy) */
static void ray_dir(int k, float hx, float hy, float *dx, float *dy)
{
    if (k < 24) {
        float u = ray_u(k);
        *dx = hx + u * hy;
        *dy = hy + u * (-hx);
    } else if (k < ORC_SENSOR) {
        float u = ray_u(k);
        *dx = -(hx + u * hy);
        *dy = -(hy + u * (-hx));
    } else {
        *dx = hx;
        *dy = hy;
    }
}

static int in_inner(float x, float y)
{
    return x >= kInLo && x <= kInHiX && y >= kInLo && y <= kInHiY;
}

/* inside one of the four wall boxes (sim.cpp:168-180: centres (64, 0),
 * (0, 48), (64, 96), (128, 48); half extents (64, 0.2), (0.2, 48), ...) */
static int in_wall_box(float x, float y)
{
    int xs = x >= 0.0f && x <= 128.0f, ys = y >= 0.0f && y <= 96.0f;
    int bx = (x >= kOutLo && x <= kInLo) || (x >= kInHiX && x <= kOutHiX);
    int by = (y >= kOutLo && y <= kInLo) || (y >= kInHiY && y <= kOutHiY);
    return (bx && ys) || (by && xs);
}

/* wall depth of a ray whose near point lies in the inner rectangle: its exit
 * from the rectangle along (dx, dy) from the origin */
static float wall_z(float ox, float oy, float dx, float dy)
{
    float tx = INFINITY, ty = INFINITY;
    if (dx > 0.0f) tx = (kInHiX - ox) / dx;
    else if (dx < 0.0f) tx = (kInLo - ox) / dx;
    if (dy > 0.0f) ty = (kInHiY - oy) / dy;
    else if (dy < 0.0f) ty = (kInLo - oy) / dy;
    float t = fmin_std(tx, ty);
    return t == 0.0f ? 0.0f : t;
}

static inline float max0(float x) { return x > 0.0f ? x : 0.0f; }

/* object depths keep 14 mantissa bits (the low 9 carry the object order in
 * the HIP kernel's 32-bit z-buffer key: food 1 + k, agents 64 + slot < 320);
 * floor(z) is unchanged for z < 2^14 */
static inline float zq(float z)
{
    uint32_t b;
    memcpy(&b, &z, 4);
    b &= ~0x1FFu;
    memcpy(&z, &b, 4);
    return z;
}

/* An object at view depth z hides the wall on ray (dx, dy) (near point in the
 * inner rectangle) iff the ray meets it strictly before leaving the
 * rectangle, tested as z * d < (X - o) per axis (no division). */
static int beats_wall(float ox, float oy, float dx, float dy, float z)
{
    if (dx > 0.0f) { if (!(z * dx < kInHiX - ox)) return 0; }
    else if (dx < 0.0f) { if (!(z * dx > kInLo - ox)) return 0; }
    if (dy > 0.0f) { if (!(z * dy < kInHiY - oy)) return 0; }
    else if (dy < 0.0f) { if (!(z * dy > kInLo - oy)) return 0; }
    return 1;
}

typedef struct { float z; uint32_t order; } orc_hit;

static inline void consider(orc_hit *h, float z, uint32_t order)
{
    if (z < h->z || (z == h->z && order < h->order)) { h->z = z; h->order = order; }
}

/* one object (a radius-0.92 circle at (cx, cy)) against all 33 rays of an
 * agent.  Ray (1, u) meets the circle's line iff
 * q(u) = (A u - 2 l f) u + C <= 0 (A = f^2 - R^2, C = l^2 - R^2); it leaves
 * the circle beyond the near sphere iff its near point P0 lies inside the
 * circle, or the chord's midpoint lies beyond P0: p >= e with p = f + u l
 * (backward: -p).  Depth f - R (backward -f - R). */
static void raster(orc_hit *hits, float ax, float ay, float hx, float hy, float cx, float cy,
                   uint32_t order)
{
    float vx = cx - ax, vy = cy - ay;
    float f = vx * hx + vy * hy;
    float l = vx * hy - vy * hx;
    float A = f * f - kAgentR2, B2 = 2.0f * (l * f), C = l * l - kAgentR2;
    float zf = zq(max0(f - kAgentR)), zb = zq(max0(-f - kAgentR));
    for (int k = 0; k <= ORC_SENSOR; ++k) {
        int fwd = k < 24 || k == ORC_SENSOR;
        float u = ray_u(k), c, s, e;
        near_pt(k, &c, &s, &e);
        float q = (A * u - B2) * u + C;
        float p = f + u * l;
        float nx = fwd ? c - f : -c - f, ny = fwd ? s - l : -s - l;
        int in0 = nx * nx + ny * ny <= kAgentR2;
        int hit = in0 || (q <= 0.0f && (fwd ? p : -p) >= e);
        if (hit) consider(&hits[k], fwd ? zf : zb, order);
    }
}

/* Food is the cube_render.obj +-1 box rotated about z by the package's draw
 * (sim.cpp:332-341); a horizontal ray at the agent's height meets its square
 * cross-section.  Rotation: quarter-turn fraction q (22 bits) -> angle
 * w = q (pi/2) 2^-22, cos / sin by fixed Taylor polynomials (host and device
 * libm differ; these are plain float operations, identical on both).       */
static const float kQuarterTurnUnit = 1.57079632679489662f / 4194304.0f;   /* (pi/2) 2^-22 */

static void food_cs(uint32_t q22, float *c, float *s)
{
    float w = (float)q22 * kQuarterTurnUnit;
    float w2 = w * w;
    *s = w * (1.0f - w2 * (1.0f / 6.0f) *
                  (1.0f - w2 * (1.0f / 20.0f) *
                       (1.0f - w2 * (1.0f / 42.0f) *
                            (1.0f - w2 * (1.0f / 72.0f) * (1.0f - w2 * (1.0f / 110.0f))))));
    *c = 1.0f - w2 * 0.5f *
                    (1.0f - w2 * (1.0f / 12.0f) *
                         (1.0f - w2 * (1.0f / 30.0f) *
                              (1.0f - w2 * (1.0f / 56.0f) *
                                   (1.0f - w2 * (1.0f / 90.0f) * (1.0f - w2 * (1.0f / 132.0f))))));
}

/* In the agent frame (f along h, l along r) the square has centre (f, l) and
 * unit axes (p, q), (-q, p).  Ray u is the line Y = u X; with
 * S(v) = v.Y - u v.X the corners' S are S(centre) +- S(axis 1) +- S(axis 2),
 * so the line meets the square iff |l - u f| <= |q - u p| + |p + u q|.  Along
 * the ray s (1, u) the square's slabs give the parameter interval [lo, hi]
 * (box coordinates s b_i - m_i, m1 = f p + l q, m2 = l p - f q, b1 = p + u q,
 * b2 = u p - q); a forward ray leaves it beyond the near sphere iff
 * hi >= s0, a backward one iff lo <= -s0 (s0 = 1.1 / |(1, u)|; box_hit).  Depth (one
 * per object, like the circles' f - R): the nearest corner's view depth,
 * max(0, f - (|p| + |q|)) forward, max(0, -(f + ...)) backward. */
static int box_line_hit(float f, float l, float p, float q, float u)
{
    return fabsf(l - u * f) <= fabsf(q - u * p) + fabsf(p + u * q);
}

/* A slab (box coordinate s b - m) ends past t iff m + 1 >= t b (b > 0) /
 * m - 1 <= t b (b < 0); it starts before t iff m - 1 <= t b / m + 1 >= t b
 * (always for b == 0, which the line test covers) -- the slab ends
 * (m -+ 1) / b multiplied out. */
static int slab_reaches(float m, float b, float t)
{
    float tb = t * b;
    if (b > 0.0f) return m + 1.0f >= tb;
    if (b < 0.0f) return m - 1.0f <= tb;
    return 1;
}

static int slab_starts_before(float m, float b, float t)
{
    float tb = t * b;
    if (b > 0.0f) return m - 1.0f <= tb;
    if (b < 0.0f) return m + 1.0f >= tb;
    return 1;
}

/* the line test, then the exit beyond the near point (ray parameter s0):
 * the square's X span [f - ext, f + ext] along the ray bounds its slab
 * interval -- wholly past s0 a hit, wholly before a miss -- else forward
 * every slab must end past s0, backward every slab must start before -s0 */
static int box_hit(float f, float l, float p, float q, float ext, float u, int fwd, float s0)
{
    if (!box_line_hit(f, l, p, q, u)) return 0;
    float zf = fwd ? f : -f;
    if (zf - ext >= s0) return 1;
    if (zf + ext < s0) return 0;
    float m1 = f * p + l * q, m2 = l * p - f * q;
    float b1 = p + u * q, b2 = u * p - q;
    if (fwd) return slab_reaches(m1, b1, s0) && slab_reaches(m2, b2, s0);
    return slab_starts_before(m1, b1, -s0) && slab_starts_before(m2, b2, -s0);
}

static void raster_box(orc_hit *hits, float ax, float ay, float hx, float hy, float cx, float cy,
                       uint32_t rot, uint32_t order)
{
    float vx = cx - ax, vy = cy - ay;
    float f = vx * hx + vy * hy;
    float l = vx * hy - vy * hx;
    float c, s;
    food_cs(rot, &c, &s);
    float p = c * hx + s * hy;
    float q = c * hy - s * hx;
    float ext = fabsf(p) + fabsf(q);
    float zf = zq(max0(f - ext)), zb = zq(max0(-(f + ext)));
    for (int k = 0; k <= ORC_SENSOR; ++k) {
        int fwd = k < 24 || k == ORC_SENSOR;
        float nc, ns, ne;
        near_pt(k, &nc, &ns, &ne);
        if (box_hit(f, l, p, q, ext, ray_u(k), fwd, nc)) consider(&hits[k], fwd ? zf : zb, order);
    }
}

static inline uint8_t depth_u8(float t)
{
    if (!(t < 255.0f)) return 255;
    return (uint8_t)(int32_t)t;
}

/* what ray k of an agent at (ox, oy) with heading (hx, hy) sees, given its
 * nearest object hit h (order 0xFFFFFFFF: none): h itself, the wall (order
 * 0) or nothing (order ORC_MISS) */
#define ORC_MISS 0xFFFFFFFEu
static orc_hit resolve(orc_hit h, int k, float ox, float oy, float hx, float hy)
{
    int fwd = k < 24 || k == ORC_SENSOR;
    float dx, dy, c, s, e;
    ray_dir(k, hx, hy, &dx, &dy);
    near_pt(k, &c, &s, &e);
    float ex = c * hx + s * hy, ey = c * hy + s * (-hx);
    float px = fwd ? ox + ex : ox - ex, py = fwd ? oy + ey : oy - ey;
    int obj = h.order != 0xFFFFFFFFu;
    orc_hit out = h;
    if (in_inner(px, py)) {
        if (!obj || !beats_wall(ox, oy, dx, dy, h.z)) { out.z = wall_z(ox, oy, dx, dy); out.order = 0; }
    } else if (in_wall_box(px, py)) {
        out.z = c;
        out.order = 0;
    } else if (!obj) {
        out.z = INFINITY;
        out.order = ORC_MISS;
    }
    return out;
}

/* the sensor of agents [lo, hi) of world wi: each agent writes only its own
 * rows and finder, so agent ranges of one world run in parallel */
static void world_phase_d_range(orc_sim *s, uint32_t wi, int32_t lo, int32_t hi)
{
    orc_world *w = &s->w[wi];
    orc_cols *nc = &s->cur[s->tb ^ 1];
    orc_hit hits[ORC_SENSOR + 1];
    for (int32_t i = lo; i < hi; ++i) {
        orc_agent *a = &w->ag[i];
        float hx, hy;
        heading(a->rw, a->rz, &hx, &hy);
        for (int k = 0; k <= ORC_SENSOR; ++k) {
            hits[k].z = INFINITY;
            hits[k].order = 0xFFFFFFFFu;   /* no object */
        }
        uint32_t nf = 0;
        for (int c = 0; c < ORC_NUM_CHUNKS; ++c) {
            float bx = (float)((c % ORC_CHUNKS_X) * ORC_CHUNK_W);
            float by = (float)((c / ORC_CHUNKS_X) * ORC_CHUNK_W);
            for (int k = 0; k < ORC_MAX_PKG; ++k) {
                if (w->pkg_n[c][k] == 0) continue;
                float fx = (float)w->pkg_x[c][k] + bx, fy = (float)w->pkg_y[c][k] + by;
                raster_box(hits, a->x, a->y, hx, hy, fx, fy, w->pkg_rot[c][k], 1u + nf);
                nf += 1;
            }
        }
        for (int32_t j = 0; j < w->n; ++j) {
            if (j == i) continue;
            raster(hits, a->x, a->y, hx, hy, w->ag[j].x, w->ag[j].y, 64u + (uint32_t)j);
        }
        /* resolve each ray against the walls */
        for (int k = 0; k <= ORC_SENSOR; ++k) hits[k] = resolve(hits[k], k, a->x, a->y, hx, hy);
        int8_t *sem = nc->sem + (size_t)a->obs_row * ORC_SENSOR;
        uint8_t *dep = nc->depth + (size_t)a->obs_row * ORC_SENSOR;
        for (int k = 0; k < ORC_SENSOR; ++k) {
            uint32_t o = hits[k].order;
            sem[k] = (int8_t)(o == ORC_MISS ? -1 : o == 0 ? 5 : (o < 64 ? 6 : w->ag[o - 64].species));
            dep[k] = depth_u8(hits[k].z);
        }
        uint32_t fo = hits[ORC_SENSOR].order;
        a->finder = (fo >= 64 && fo != ORC_MISS) ? (int32_t)(fo - 64) : -1;
    }
}

/* the sensor over every world's agents, split evenly by agent count (a few
 * worlds of thousands of agents still use every thread) */
typedef struct { orc_sim *s; uint64_t lo, hi; } sensor_job_t;
static void *sensor_job_run(void *p)
{
    sensor_job_t *j = (sensor_job_t *)p;
    uint64_t g = 0;
    for (uint32_t wi = 0; wi < j->s->cfg.num_worlds && g < j->hi; ++wi) {
        uint64_t n = (uint64_t)j->s->w[wi].n, a = j->lo > g ? j->lo - g : 0, b = j->hi - g < n ? j->hi - g : n;
        if (a < b) world_phase_d_range(j->s, wi, (int32_t)a, (int32_t)b);
        g += n;
    }
    return NULL;
}
static void sensor_all(orc_sim *s)
{
    uint64_t G = 0;
    for (uint32_t wi = 0; wi < s->cfg.num_worlds; ++wi) G += (uint64_t)s->w[wi].n;
    uint32_t T = s->cfg.num_threads ? s->cfg.num_threads : 1;
    if (T > 256) T = 256;
    if ((uint64_t)T > G) T = G ? (uint32_t)G : 1;
    pthread_t th[256];
    sensor_job_t jobs[256];
    for (uint32_t t = 0; t < T; ++t) {
        jobs[t].s = s;
        jobs[t].lo = G * t / T;
        jobs[t].hi = G * (t + 1) / T;
        if (T > 1) pthread_create(&th[t], NULL, sensor_job_run, &jobs[t]);
    }
    if (T <= 1) sensor_job_run(&jobs[0]);
    else
        for (uint32_t t = 0; t < T; ++t) pthread_join(th[t], NULL);
}

/* ------------------------------------------------------------------------ */
/* Public API                                                                */
/* ------------------------------------------------------------------------ */
static void finish_step(orc_sim *s)
{
    compute_rows(s);
    for_worlds(s, world_phase_c);
    sensor_all(s);
    s->tb ^= 1;
}

orc_sim *orc_create(const orc_config *cfg)
{
    orc_sim *s = calloc(1, sizeof(*s));
    if (!s) return NULL;
    s->cfg = *cfg;
    uint32_t W = cfg->num_worlds, cap = cfg->cap;
    size_t rows = (size_t)W * cap;
    s->w = calloc(W, sizeof(orc_world));
    s->species_count = calloc((size_t)W * 4, 4);
    s->world_off = calloc(W, 4);
    s->row_base = calloc((size_t)W * 4, 4);
    int ok = s->w && s->species_count && s->world_off && s->row_base;
    for (int b = 0; b < 2 && ok; ++b) ok = cols_alloc(&s->cur[b], rows) && cols_alloc(&s->prev[b], rows);
    if (!ok) { orc_destroy(s); return NULL; }
    for (uint32_t wi = 0; wi < W; ++wi) {
        orc_world *w = &s->w[wi];
        w->ag = calloc(cap, sizeof(orc_agent));
        w->tmp = calloc(cap, sizeof(orc_agent));
        if (!w->ag || !w->tmp) { orc_destroy(s); return NULL; }
        /* Sim::Sim (sim.cpp:1232-1256): rng = split_i(initKey(seed), 0, world) */
        uint32_t k0[2] = {cfg->rand_seed, 0u}, c[2] = {0u, cfg->world_offset + wi};
        orc_threefry2x32(k0, c, w->key);
        w->ctr = 0;
        /* initWorld (sim.cpp:233-275) */
        for (uint32_t i = 0; i < cfg->init_agents && i < cap; ++i) {
            int32_t sp = (int32_t)(i % ORC_NUM_SPECIES) + 1;
            float x = sample_uniform(w) * kLx;
            float y = sample_uniform(w) * kLy;
            agent_init(&w->ag[i], x, y, sp, 100);
            w->n += 1;
        }
        for (int i = 0; i < ORC_NUM_SPECIES; ++i) w->species_count[i] = 0;
        for (int32_t i = 0; i < w->n; ++i) w->species_count[w->ag[i].species - 1] += 1;
    }
    /* Initial export: rows in species-major order; Prev and sensor columns zero. */
    compute_rows(s);
    orc_cols *c0 = &s->cur[0];
    for (uint32_t wi = 0; wi < W; ++wi) {
        orc_world *w = &s->w[wi];
        int32_t rank[4] = {0};
        for (int32_t i = 0; i < w->n; ++i) {
            orc_agent *a = &w->ag[i];
            int sp = a->species - 1;
            int32_t r = s->row_base[wi * 4 + sp] + rank[sp]++;
            c0->species[r] = a->species;
            c0->pos[r * 2] = a->x;
            c0->pos[r * 2 + 1] = a->y;
            c0->health[r] = a->health;
            a->obs_row = r;
        }
    }
    s->tb = 0;
    return s;
}

void orc_destroy(orc_sim *s)
{
    if (!s) return;
    if (s->w) {
        for (uint32_t i = 0; i < s->cfg.num_worlds; ++i) { free(s->w[i].ag); free(s->w[i].tmp); }
        free(s->w);
    }
    for (int b = 0; b < 2; ++b) { cols_free(&s->cur[b]); cols_free(&s->prev[b]); }
    free(s->species_count); free(s->world_off); free(s->row_base);
    free(s);
}

void orc_step(orc_sim *s)
{
    for_worlds(s, world_phase_a);
    finish_step(s);
}

/* shiftObservationsSystem + shiftHiddenState (sim.cpp:1002-1048) */
void orc_shift_observations(orc_sim *s)
{
    orc_cols *c = &s->cur[s->tb], *p = &s->prev[s->tb];
    size_t n = s->total;
    memcpy(p->species, c->species, n * 4);
    memcpy(p->pos, c->pos, n * 8);
    memcpy(p->health, c->health, n * 4);
    memcpy(p->sur, c->sur, n * 8);
    memcpy(p->reward, c->reward, n * 4);
    memcpy(p->action, c->action, n * 24);
    for (size_t r = 0; r < n; ++r) {
        p->stats[r * 4 + 0] = c->stats[r * 4 + 0];
        p->stats[r * 4 + 1] = c->stats[r * 4 + 0];   /* :1034 hitEnemy <- hitFriendly */
        p->stats[r * 4 + 2] = c->stats[r * 4 + 2];
        p->stats[r * 4 + 3] = c->stats[r * 4 + 3];
    }
    memcpy(p->hidden, c->hidden, n * 4 * ORC_HIDDEN);
}

uint32_t orc_num_agents(const orc_sim *s) { return s->total; }

void *orc_column(orc_sim *s, int col, int is_prev)
{
    orc_cols *c = is_prev ? &s->prev[s->tb] : &s->cur[s->tb];
    switch (col) {
    case ORC_COL_SPECIES: return c->species;
    case ORC_COL_POS: return c->pos;
    case ORC_COL_HEALTH: return c->health;
    case ORC_COL_SURROUND: return c->sur;
    case ORC_COL_REWARD: return c->reward;
    case ORC_COL_ACTION: return c->action;
    case ORC_COL_STATS: return c->stats;
    case ORC_COL_HIDDEN: return c->hidden;
    case ORC_COL_SEMANTIC: return c->sem;
    case ORC_COL_DEPTH: return c->depth;
    default: return NULL;
    }
}

int32_t *orc_species_count(orc_sim *s) { return s->species_count; }

void orc_world_counts(const orc_sim *s, int32_t *counts, int32_t *offsets)
{
    for (uint32_t w = 0; w < s->cfg.num_worlds; ++w) {
        if (counts) counts[w] = s->w[w].n;
        if (offsets) offsets[w] = s->world_off[w];
    }
}

void orc_write_synthetic_actions(orc_sim *s, uint32_t seed, uint32_t step, int write_hidden)
{
    orc_cols *c = &s->cur[s->tb];
    for (uint32_t wi = 0; wi < s->cfg.num_worlds; ++wi) {
        orc_world *w = &s->w[wi];
        uint32_t gw = s->cfg.world_offset + wi;
        for (int32_t i = 0; i < w->n; ++i) {
            size_t r = (size_t)w->ag[i].obs_row;
            uint32_t h = orc_action_hash(seed, step, gw, (uint32_t)i);
            uint32_t k = h % 6u;
            for (uint32_t j = 0; j < 6; ++j) c->action[r * 6 + j] = (j == k) ? 1 : 0;
            if (write_hidden) {   /* both words of draw k: hidden[2k], hidden[2k + 1] */
                for (uint32_t q = 0; q < ORC_HIDDEN / 2; ++q) {
                    uint32_t kk[2] = {seed ^ 0x9E3779B9u, step};
                    uint32_t cc[2] = {gw, (uint32_t)i * (ORC_HIDDEN / 2) + q}, hb[2];
                    orc_threefry2x32(kk, cc, hb);
                    c->hidden[r * ORC_HIDDEN + 2 * q] = orc_sample_uniform(hb[0]) - 0.5f;
                    c->hidden[r * ORC_HIDDEN + 2 * q + 1] = orc_sample_uniform(hb[1]) - 0.5f;
                }
            }
        }
    }
}

void orc_sensor_index(const orc_sim *s, int32_t *out)
{
    for (uint32_t wi = 0; wi < s->cfg.num_worlds; ++wi)
        for (int32_t i = 0; i < s->w[wi].n; ++i) out[s->world_off[wi] + i] = s->w[wi].ag[i].obs_row;
}

uint32_t orc_overflow(const orc_sim *s)
{
    uint32_t o = 0;
    for (uint32_t w = 0; w < s->cfg.num_worlds; ++w) o += s->w[w].overflow;
    return o;
}

void orc_world_state(const orc_sim *s, uint32_t wi, float *xy, float *rot, int32_t *species,
                     int32_t *health, int32_t *finder, int32_t *n)
{
    const orc_world *w = &s->w[wi];
    *n = w->n;
    for (int32_t i = 0; i < w->n; ++i) {
        const orc_agent *a = &w->ag[i];
        if (xy) { xy[2 * i] = a->x; xy[2 * i + 1] = a->y; }
        if (rot) { rot[2 * i] = a->rw; rot[2 * i + 1] = a->rz; }
        if (species) species[i] = a->species;
        if (health) health[i] = a->health;
        if (finder) finder[i] = a->finder;
    }
}

int32_t orc_world_food(const orc_sim *s, uint32_t wi, int32_t *out)
{
    const orc_world *w = &s->w[wi];
    int32_t k = 0;
    for (int ch = 0; ch < ORC_NUM_CHUNKS; ++ch)
        for (int p = 0; p < ORC_MAX_PKG; ++p) {
            if (w->pkg_n[ch][p] == 0) continue;
            out[4 * k + 0] = ch;
            out[4 * k + 1] = (ch % ORC_CHUNKS_X) * ORC_CHUNK_W + w->pkg_x[ch][p];
            out[4 * k + 2] = (ch / ORC_CHUNKS_X) * ORC_CHUNK_W + w->pkg_y[ch][p];
            out[4 * k + 3] = (int32_t)w->pkg_rot[ch][p];
            ++k;
        }
    return k;
}

void orc_probe_agent(float ax, float ay, float hx, float hy, float cx, float cy, uint8_t *hit, float *z)
{
    orc_hit hits[ORC_SENSOR + 1];
    for (int k = 0; k <= ORC_SENSOR; ++k) { hits[k].z = INFINITY; hits[k].order = 0xFFFFFFFFu; }
    raster(hits, ax, ay, hx, hy, cx, cy, 64u);
    for (int k = 0; k <= ORC_SENSOR; ++k) {
        hit[k] = hits[k].order == 64u;
        z[k] = hits[k].z;
    }
}

void orc_probe_walls(float ax, float ay, float hx, float hy, int8_t *sem, uint8_t *depth)
{
    for (int k = 0; k <= ORC_SENSOR; ++k) {
        orc_hit none = {INFINITY, 0xFFFFFFFFu};
        orc_hit h = resolve(none, k, ax, ay, hx, hy);
        sem[k] = (int8_t)(h.order == ORC_MISS ? -1 : 5);
        depth[k] = depth_u8(h.z);
    }
}

void orc_probe_box(float ax, float ay, float hx, float hy, float cx, float cy, uint32_t rot,
                   uint8_t *hit, float *z)
{
    orc_hit hits[ORC_SENSOR + 1];
    for (int k = 0; k <= ORC_SENSOR; ++k) { hits[k].z = INFINITY; hits[k].order = 0xFFFFFFFFu; }
    raster_box(hits, ax, ay, hx, hy, cx, cy, rot, 1u);
    for (int k = 0; k <= ORC_SENSOR; ++k) {
        hit[k] = hits[k].order == 1u;
        z[k] = hits[k].z;
    }
}
