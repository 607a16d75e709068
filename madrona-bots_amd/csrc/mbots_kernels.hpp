// mbots_kernels.hpp -- device state descriptors and kernel launchers.
#pragma once

#include "mbots_device.hpp"
#include "../../include/mbots.h"

namespace mbots {

constexpr uint32_t kFlagRewardFixed = 0x1u;   // MBOTS_FLAG_REWARD_FIXED
constexpr uint32_t kFlagFixDepth = 0x2u;      // MBOTS_FLAG_FIX_DEPTH_ALIAS
constexpr uint32_t kFlagShardGhost = 0x4u;    // MBOTS_FLAG_SHARD_GHOST

// Agent / world state in HBM (SoA).  Agent columns are [W][cap].
struct SimState {
    float *x, *y, *rw, *rz;         // base::Position.xy, base::Rotation (w, z)
    int32_t *species;               // Species
    int32_t *health;                // Health (== HealthAccumulator between steps)
    int32_t *finder;                // FinderOutput hit -> slot in the same world, -1 none
    int32_t *obsrow;                // AgentObservationBridge -> export row (K3a writes it, the
                                    // next K1 reads it)
    float *sur0, *sur1;             // SurroundingObservation (step-local)
    uint32_t *stats;                // AgentStats bits (step-local)
    int32_t *n;                     // [W] live agents per world
    uint32_t *ctr;                  // [W] RNG counter
    uint2 *key;                     // [W] RNG key
    uint64_t *food;                 // [W][48] per chunk: 5 x (x | y << 4) bytes, live mask << 40
    uint32_t *food_rot;             // [W][5][48] food box rotation (22-bit quarter turn) per package
    int32_t *cur_food;              // [W] Sim::currentNumFood
    float *sreward;                 // [W][4] SpeciesReward
    int32_t *scount;                // [W][4] SpeciesCount (exported)
    int32_t *row_base;              // [W][4] first export row of (world, species)
    int32_t *world_off;             // [W] world-major agent offsets
    int32_t *src_of;                // [W*cap] new export row -> old row (-1: new agent)
    uint32_t *overflow;             // [W] dropped births/respawns
    uint32_t *totals;               // [0] = N, [1..4] = per-species rows, [kTotRows] = table rows
                                    // incl. the shard ghost's (after row N), [kTotOverflow]
    uint32_t *totals_host;          // mapped pinned mirror of totals (written by K2)
    int32_t *tiles;                 // [2][5][ntiles][kTileBuckets] per-tile species/agent counts (K1 -> K2)
    unsigned long long *agent_steps;
    float4 *raytab;                 // [36] per ray (32 pixels, the finder): u, NearPt c, s, e
    int32_t *sorder;                // [W] the sensor's world order (K2: each tile by descending
                                    // population), or null: world order (W not a multiple of
                                    // the 1024-world tile)
    // K1's output half of the double-buffered columns the sensor reads (the
    // sensor of step t runs beside step t+1's K1; swap_state after each K1)
    float *x_out, *y_out, *rw_out, *rz_out;
    int32_t *species_out, *n_out;
    int32_t *obsrow_out;            // K1 -> K3a / the sensor: each slot's old export row (not
                                    // swapped with obsrow -- K1 reads obsrow, K3a rewrites it --
                                    // but one of two buffers by step parity, set by the host:
                                    // in K1-finder mode the sensor of step t reads it beside
                                    // step t+1's K1)
    uint64_t *food_out;
    // the fork as a value wait (small world counts, mbots_step): K2's last
    // block stores `epoch` into sig_fork (signal memory); epoch 0: no flag
    uint32_t *fork_ctr;             // K2 blocks done (reset by the last)
    uint32_t *sig_fork;
    uint32_t epoch;
    uint32_t W, cap, A, world_offset, flags, seed, ntiles;
    // K1 computes the finder slots its actions read itself (world_finders;
    // small world counts) instead of reading the last sensor's S.finder, so it
    // does not wait for that sensor
    uint32_t k1_finder;
    // ... except on the first step after init (no sensor has run: the finder
    // slots are the init's "none", S.finder), set by the host for that launch
    uint32_t finder_from_state;
    // (K1-finder mode) the last table's sensor rows: the sensor itself moves
    // them into its rows' prev-sensor columns (null: the shift / moves do)
    const int8_t *psem_src;
    const uint8_t *pdepth_src;
    uint32_t Wx;                    // exported worlds: W, or W - 1 with the shard ghost (the
                                    // last world, its rows placed after every exported row)
    // mixed capacity classes (agent_capacity > 128 outside K1-finder mode): the
    // 128-slot kernels take every world that fits them and the class kernels
    // only the worlds K2 listed -- big_k1: 2 n + A > 128 (the next K1 could
    // overflow 128 slots), big_s: n > 128 (this step's sensor) -- each [2][W]
    // by step parity, with their counts in big_cnt[parity][2]
    uint32_t mixed;
    uint32_t track_maxpop;          // K2 publishes each tile's largest world (kTotMaxPop; set by
                                    // the first mbots_max_population)
    uint32_t list_par;              // the parity whose lists this launch reads (host-set)
    int32_t *big_k1, *big_s;
    uint32_t *big_cnt;
};

// the small kernel class of mixed-class dispatch
constexpr int kSmallCap = 128;
// a world whose next K1 needs the class kernel: it may end with 2 n + A agents
__host__ __device__ inline bool k1_needs_class(int n, uint32_t A) { return 2 * n + (int)A > kSmallCap; }

inline void swap_state(SimState &S)
{
    auto sw = [](auto &a, auto &b) { auto t = a; a = b; b = t; };
    sw(S.x, S.x_out); sw(S.y, S.y_out); sw(S.rw, S.rw_out); sw(S.rz, S.rz_out);
    sw(S.species, S.species_out); sw(S.n, S.n_out);
    sw(S.food, S.food_out);
}

// One half of the double-buffered species-major observation table
// (AgentObservationArchetype, types.hpp:228-252, + raycast output columns).
struct ObsTable {
    int32_t *species;  float *pos;  int32_t *health;  float *sur;  float *reward;
    int32_t *action;   int32_t *stats;  float *hidden;  int8_t *sem;  uint8_t *depth;
    int32_t *pspecies; float *ppos; int32_t *phealth; float *psur; float *preward;
    int32_t *paction;  int32_t *pstats; float *phidden; int8_t *psem; uint8_t *pdepth;
};

constexpr int kTotRows = 5;   // totals[kTotRows]: rows the moves / shift / checkpoints cover
constexpr int kTotMaxPop = 8;     // totals_host[kTotMaxPop + tile]: the tile's largest world
                                  // population after the last K2 (the pinned mirror only)
constexpr int kTotOverflow = 6;   // totals[kTotOverflow]: births / respawns dropped at the
                                  // capacity cap so far (exported worlds; K1 adds, K2 mirrors)
uint32_t scan_tiles(uint32_t W);
// whether the sensor renders worlds in K2's population order (every scan tile
// full)
bool sensor_order_used(uint32_t W);
// K1 blocks add their counts into one of kTileBuckets copies of their tile's
// counters (block index mod 8): fewer same-address atomics at K1's end
constexpr int kTileBuckets = 8;
hipError_t launch_init(const SimState &S, hipStream_t st);
// the sensor's ray table (host-computed with the kernels' own u_of / near_pt)
hipError_t upload_ray_table(const SimState &S, hipStream_t st);
hipError_t launch_tile_sum(const SimState &S, int parity, hipStream_t st);
hipError_t launch_raise_flag(uint32_t *flag, uint32_t v, hipStream_t st);
hipError_t launch_world_step(const SimState &S, const ObsTable &cur, int parity, hipStream_t st,
                             hipEvent_t done = nullptr);
// plain_events: record `done` with hipEventRecord (stream capture) instead of on the dispatch
hipError_t launch_scan(const SimState &S, int parity, hipStream_t st, hipEvent_t done = nullptr,
                       bool plain_events = false);
// mixed classes: the K1 class list of slot `slot` rebuilt from S.n (after a
// checkpoint load; K2 builds it every step)
hipError_t launch_build_lists(const SimState &S, int slot, hipStream_t st);
hipError_t launch_export_rows(const SimState &S, const ObsTable &nxt, int init, hipStream_t st);
// K4 parts (DESIGN.md "Deferred Prev moves"): Action + HiddenState; the same
// also into PrevAction / PrevHiddenState (the fused shift); the prev sensor;
// PrevAction / PrevHiddenState; the six other Prev* columns
constexpr int kMoveAH = 1, kMoveAHShift = 2, kMoveSensor = 4, kMovePrevAH = 8, kMovePrev6 = 16;
constexpr int kMoveAll = kMoveAH | kMoveSensor | kMovePrevAH | kMovePrev6;
hipError_t launch_move(const SimState &S, const ObsTable &cur, const ObsTable &nxt, int prev_lazy,
                       int parts, hipStream_t st);
hipError_t launch_sensor(const SimState &S, const ObsTable &nxt, hipStream_t st,
                         hipEvent_t done = nullptr, bool plain_events = false);
// shift modes: every Prev* column / Action + HiddenState only (lazy) / the six
// columns a lazy shift left (materialise)
constexpr int kShiftAll = 0, kShiftEager = 1, kShiftRest = 2;
hipError_t launch_shift(const SimState &S, const ObsTable &t, int mode, hipStream_t st);
hipError_t launch_synthetic_actions(const SimState &S, const ObsTable &t, uint32_t seed,
                                    uint32_t step, int write_hidden, hipStream_t st);
hipError_t launch_sensor_index(const SimState &S, int32_t *out, hipStream_t st);
// six_src: the other half, when the current half's six Prev* columns are
// still the step's deferred move (prev rows gather their three columns along
// src_of, as the move would; six_lazy: that move's source is its current ones)
hipError_t launch_construct_obs(const SimState &S, const ObsTable &t, int prev, int prev_lazy,
                                float *out, uint32_t out_rows, hipStream_t st,
                                const ObsTable *six_src = nullptr, int six_lazy = 0);
// rollout records of the config-5 gather (MBOTS_ROLLOUT_BYTES[_DEPTH])
constexpr uint32_t kRolloutBytes = 64, kRolloutBytesDepth = 96;
hipError_t launch_pack_rollout(const SimState &S, const ObsTable &t, void *out, uint32_t out_rows,
                               hipStream_t st);
hipError_t launch_unpack_rollout(const void *recs, uint32_t n, int fixd, float *obs, float *reward,
                                 int32_t *stats, hipStream_t st);
// learner records of the config-5 round trip (MBOTS_LEARNER_BYTES[_DEPTH])
constexpr uint32_t kLearnerBytes = 272, kLearnerBytesDepth = 336;
// `t` holds every logical column's storage (the manager materialised the
// step's deferred moves); prev_lazy: the six Prev* columns are the current ones
hipError_t launch_pack_learner(const SimState &S, const ObsTable &t, int prev_lazy, void *out, uint32_t out_rows,
                               hipStream_t st);
hipError_t launch_unpack_learner(const void *recs, uint32_t n, int fixd, const mbots_learner_out &o,
                                 hipStream_t st);
// slim learner records (MBOTS_LEARNER_SLIM_BYTES[_DEPTH]): `t` the current half
// (prev_lazy: its six Prev* columns are the current ones); the previous
// observation columns the step still owes are gathered along S.src_of inside
// the launch -- the six from `six_src` (six_lazy: from its current columns),
// the prev sensor from `sem_src`'s sensor rows -- when those are non-null
constexpr uint32_t kLearnerSlimBytes = 128, kLearnerSlimBytesDepth = 192;
hipError_t launch_pack_learner_slim(const SimState &S, const ObsTable &t, int prev_lazy, const ObsTable *six_src,
                                    int six_lazy, const ObsTable *sem_src, void *out, uint32_t out_rows,
                                    hipStream_t st);
hipError_t launch_unpack_learner_slim(const void *recs, uint32_t n, int fixd, const mbots_learner_out &o,
                                      int32_t *src, hipStream_t st);
// the learner rank's rebuild of Action / HiddenState / PrevHiddenState from
// slim records' provenance (mbots_rebuild_learner): per (rank, species) the
// first global row of the gathered table, and of the last table with the
// owning rank's local first row
struct RebuildPlan {
    int32_t ranks;
    int32_t sp_end[4];                                  // gathered table: species segment ends
    int32_t cur_g[MBOTS_MAX_LEARNER_RANKS][4];          // gathered: first global row of (rank, species)
    int32_t last_l[MBOTS_MAX_LEARNER_RANKS][4];         // last table: first local row of (rank, species)
    int32_t last_g[MBOTS_MAX_LEARNER_RANKS][4];         // last table: its first global row
};
RebuildPlan rebuild_plan(const int64_t *cur_counts, const int64_t *last_counts, uint32_t ranks);
// global row of the last table for gathered row r with provenance o (-1: none)
__host__ __device__ inline int32_t rebuild_row(const RebuildPlan &p, int32_t r, int32_t o)
{
    if (o < 0) return -1;
    int s = 0;
    while (s < 3 && r >= p.sp_end[s]) ++s;
    int k = 0;
    while (k + 1 < p.ranks && r >= p.cur_g[k + 1][s]) ++k;
    int t = 3;
    while (t > 0 && o < p.last_l[k][t]) --t;
    return p.last_g[k][t] + (o - p.last_l[k][t]);
}
hipError_t launch_rebuild_learner(const RebuildPlan &p, const int32_t *src, uint32_t rows, uint32_t last_rows,
                                  const int32_t *last_action, const float *last_memory, const float *last_hidden,
                                  int32_t *action, float *hidden, float *prev_hidden, hipStream_t st);

}  // namespace mbots
