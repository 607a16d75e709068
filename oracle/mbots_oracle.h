/*
 * mbots_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C11) of the llGuy/madrona-bots per-step simulation
 * (src/sim/sim.cpp, src/sim/sim.inl, src/sim/types.hpp, src/entry/mgr.cpp).
 * It is the parity checker for the HIP product path and the CPU baseline of
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  The product (madrona-bots_amd/) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned" for the arithmetic that lives in the
 * un-vendored Madrona submodule (RNG, quaternion math, raycast sensor, ECS
 * creation/sort order) -- the reference cannot be built or imported in this
 * container and ships no golden vectors.  Those
 * pieces follow the build's written spec.  Everything
 * else restates the cited reference lines; boundary shapes are pinned by the
 * reference checkpoints (obs width 69, action width 6: tests/golden/).
 */
#ifndef MBOTS_ORACLE_H
#define MBOTS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* src/sim/types.hpp:13-14, :78-80; src/entry/mgr.cpp:104-113 */
#define ORC_NUM_SPECIES   4
#define ORC_HIDDEN        16
#define ORC_SENSOR        32
#define ORC_CHUNKS_X      8
#define ORC_CHUNKS_Y      6
#define ORC_NUM_CHUNKS    48
#define ORC_CHUNK_W       16
#define ORC_MAX_PKG       5
#define ORC_FOOD_CAP      30

typedef struct orc_sim orc_sim;

typedef struct {
    uint32_t num_worlds;        /* worlds held by this instance            */
    uint32_t world_offset;      /* global index of world 0 (sharding)     */
    uint32_t rand_seed;
    uint32_t init_agents;       /* initNumAgentsPerWorld                   */
    uint32_t cap;               /* per-world agent slot capacity           */
    uint32_t reward_fixed;      /* 0: faithful rewards[speciesID]; 1: [id-1] */
    uint32_t num_threads;       /* host threads for the world loops        */
} orc_config;

/* Column identifiers of the exported observation table (mgr.cpp:199-422). */
enum {
    ORC_COL_SPECIES = 0,  /* int32 [N]      */
    ORC_COL_POS,          /* f32   [N][2]   */
    ORC_COL_HEALTH,       /* int32 [N]      */
    ORC_COL_SURROUND,     /* f32   [N][2]   */
    ORC_COL_REWARD,       /* f32   [N]      */
    ORC_COL_ACTION,       /* int32 [N][6]   */
    ORC_COL_STATS,        /* int32 [N][4]   */
    ORC_COL_HIDDEN,       /* f32   [N][16]  */
    ORC_COL_SEMANTIC,     /* int8  [N][32]  */
    ORC_COL_DEPTH,        /* uint8 [N][32]  */
    ORC_NUM_COLS
};

orc_sim *orc_create(const orc_config *cfg);
void     orc_destroy(orc_sim *s);
void     orc_step(orc_sim *s);
void     orc_shift_observations(orc_sim *s);
uint32_t orc_num_agents(const orc_sim *s);
/* pointer to the current (is_prev=0) or Prev* (is_prev=1) column */
void    *orc_column(orc_sim *s, int col, int is_prev);
int32_t *orc_species_count(orc_sim *s);           /* [W][4]          */
/* per-world agent counts / world-major offsets (agentOffsetForWorld) */
void     orc_world_counts(const orc_sim *s, int32_t *counts, int32_t *offsets);
/* identity-keyed synthetic action stream: one-hot(hash(seed,step,gw,slot)%6);
 * hidden[k] = hash-derived float when write_hidden != 0 */
void     orc_write_synthetic_actions(orc_sim *s, uint32_t seed, uint32_t step,
                                     int write_hidden);
/* per-world agent slot -> export row (sensorIndexTensor in world-major order) */
void     orc_sensor_index(const orc_sim *s, int32_t *out);
uint32_t orc_overflow(const orc_sim *s);
/* debug views of the per-world slot state (tests) */
void     orc_world_state(const orc_sim *s, uint32_t w, float *xy, float *rot,
                         int32_t *species, int32_t *health, int32_t *finder,
                         int32_t *n);
/* live food packages of world w in (chunk, package) order: out[k] = (chunk,
 * x, y, 22-bit rotation); returns their count (<= 240 entries of 4) */
int32_t  orc_world_food(const orc_sim *s, uint32_t w, int32_t *out);

/* exposed primitives for known-answer tests */
/* one food box (centre (cx, cy), 22-bit rotation) seen from an agent at
 * (ax, ay) with heading (hx, hy): hit[k] / depth z[k] per ray (32 pixels,
 * the finder ray last) */
void     orc_probe_box(float ax, float ay, float hx, float hy, float cx, float cy,
                       uint32_t rot, uint8_t *hit, float *z);
/* the same for another agent's disc centred at (cx, cy) */
void     orc_probe_agent(float ax, float ay, float hx, float hy, float cx, float cy,
                         uint8_t *hit, float *z);
/* what each ray of a lone agent sees of the walls: sem[k] (5 wall, -1 miss)
 * and depth[k] bytes (the finder ray last: 5 / -1) */
void     orc_probe_walls(float ax, float ay, float hx, float hy, int8_t *sem, uint8_t *depth);
void     orc_threefry2x32(const uint32_t key[2], const uint32_t ctr[2],
                          uint32_t out[2]);
float    orc_sample_uniform(uint32_t bits);
int32_t  orc_sample_i32(uint32_t bits, int32_t a, int32_t b);
uint32_t orc_action_hash(uint32_t seed, uint32_t step, uint32_t gworld,
                         uint32_t slot);

#ifdef __cplusplus
}
#endif
#endif
