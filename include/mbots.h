/*
 * mbots.h -- C ABI of the MI355X-native madrona-bots simulator (libmbots.so).
 *
 * This is the drop-in boundary for the reference's host surface:
 *   class Manager            src/entry/mgr.hpp:10-68
 *   Manager::Impl::make      src/entry/mgr.cpp:98-172
 *   nanobind SimManager      src/entry/entry.cpp:16-45
 * Plain pointers, sizes and status codes only (no torch / HIP C++ types).
 * Every function returns MBOTS_OK (0) or a negative MBOTS_E* code; the text of
 * the last error on the calling thread is available from mbots_last_error().
 * The one positive status is mbots_step's MBOTS_W_CAPACITY (a warning: the
 * step ran).
 * Streams are passed as `void *` holding a hipStream_t (NULL = default stream;
 * ignored in MBOTS_EXEC_CPU mode, where every call completes before returning).
 *
 * Ownership (mgr.cpp:70-76): the handle owns every device buffer; tensors
 * returned by mbots_export are non-owning views that stay valid until the next
 * mbots_step (the export tables are double-buffered and swap on every step;
 * the reference's views are likewise shape-stale after step()).
 */
#ifndef MBOTS_H
#define MBOTS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MBOTS_OK             0
#define MBOTS_E_INVALID    (-1)   /* bad argument / config             */
#define MBOTS_E_HIP        (-2)   /* HIP runtime error                  */
#define MBOTS_E_NOMEM      (-3)   /* device / host allocation failed    */
#define MBOTS_E_RANGE      (-4)   /* index out of range                 */
#define MBOTS_E_CAPACITY   (-5)   /* mbots_step with MBOTS_FLAG_STRICT_CAPACITY:
                                     agents were dropped at agent_capacity (the
                                     step ran; see MBOTS_W_CAPACITY) */
/* mbots_step warning (the step ran): since the last report, births or
 * respawns were dropped because a world had reached agent_capacity.  The
 * reference's tables have no cap (makeAgent in healthSync and in the respawn,
 * sim.cpp:561-564, :830-834), so from that step on the run diverges from the
 * reference's.  Reported from the row counts the device last published, so
 * it can come a few steps after the drop (once per rise of mbots_overflow). */
#define MBOTS_W_CAPACITY     1

/* Manager::Config flags (build extensions; default 0 = reference-faithful) */
#define MBOTS_FLAG_REWARD_FIXED     0x1u  /* rewards[speciesID-1] (fixes sim.cpp:943) */
#define MBOTS_FLAG_FIX_DEPTH_ALIAS  0x2u  /* depth_tensor exports real depth (sim.cpp:102-112) */
/* shard ghost: also step world world_offset + num_worlds (the next shard's
 * first world), never exported, so the faithful rewards[speciesID] of the
 * shard's last world reads the same SpeciesInfo row as on one device
 * (sim.cpp:943).  The ghost's agents act on what
 * mbots_write_synthetic_actions writes (the identity-keyed stream is keyed by
 * global world, so with it N shards == one device exactly); its rows lie past
 * row N, outside every exported view, so a learner writing actions through
 * the views leaves them to replay their last actions (carried through the row
 * moves and the shift like every row's).  Every shard but the last sets it. */
#define MBOTS_FLAG_SHARD_GHOST      0x4u
/* a capacity drop (MBOTS_W_CAPACITY) is an error: mbots_step returns
 * MBOTS_E_CAPACITY instead */
#define MBOTS_FLAG_STRICT_CAPACITY  0x8u

/* agent_capacity: 4..4096 slots per world (MBOTS_MAX_CAPACITY); the kernel
 * classes are 128 (default), 256, 512, 1024, 2048 and 4096 slots.  Up to 256 the
 * sensor's per-pixel depth key carries the object order (64 + slot for
 * agents) in the low 9 bits of a 32-bit word; the larger classes keep the same
 * quantised depth and the order in a 64-bit key, so a world renders the same
 * bytes in every class.  The K1 finder mode (<= 2048 worlds) is a <= 256-slot
 * mode. */
#define MBOTS_MAX_CAPACITY          4096u

/* execution modes (madrona::ExecMode; the reference's callers pick CPU when
 * no GPU is present, learn/env.py:12-15) */
#define MBOTS_EXEC_HIP  0   /* gfx950 kernels on device gpu_id (default)     */
#define MBOTS_EXEC_CPU  1   /* host threads; bit-identical results, host views */

/* Manager::Config (src/entry/mgr.hpp:12-23) plus sharding / capacity knobs. */
typedef struct mbots_config {
    int32_t  gpu_id;                    /* gpuID                              */
    uint32_t num_worlds;                /* numWorlds held by this instance    */
    uint32_t rand_seed;                 /* randSeed                           */
    uint32_t init_num_agents_per_world; /* initNumAgentsPerWorld              */
    uint32_t sensor_size;               /* sensorSize; must be 32             */
    uint32_t world_offset;              /* global index of world 0 (shards)   */
    uint32_t agent_capacity;            /* per-world slot cap (0 -> 128)      */
    uint32_t flags;                     /* MBOTS_FLAG_*                       */
    int32_t  exec_mode;                 /* MBOTS_EXEC_* (ExecMode)            */
} mbots_config;

/* Export slots; numbering mirrors enum class ExportID (src/sim/sim.hpp:18-55). */
enum mbots_export_id {
    MBOTS_EXPORT_RESET = 0,
    MBOTS_EXPORT_ACTION = 1,
    MBOTS_EXPORT_PREV_ACTION = 2,
    MBOTS_EXPORT_HIDDEN_STATE = 3,
    MBOTS_EXPORT_PREV_HIDDEN_STATE = 4,
    MBOTS_EXPORT_REWARD = 5,
    MBOTS_EXPORT_PREV_REWARD = 6,
    MBOTS_EXPORT_DONE = 7,
    MBOTS_EXPORT_POSITION = 8,
    MBOTS_EXPORT_PREV_POSITION = 9,
    MBOTS_EXPORT_HEALTH = 10,
    MBOTS_EXPORT_PREV_HEALTH = 11,
    MBOTS_EXPORT_SURROUNDING = 12,
    MBOTS_EXPORT_PREV_SURROUNDING = 13,
    MBOTS_EXPORT_SENSOR_SEMANTIC = 14,
    MBOTS_EXPORT_SENSOR_DEPTH = 15,
    MBOTS_EXPORT_PREV_SENSOR_SEMANTIC = 16,
    MBOTS_EXPORT_PREV_SENSOR_DEPTH = 17,
    MBOTS_EXPORT_STATS = 18,
    MBOTS_EXPORT_PREV_STATS = 19,
    MBOTS_EXPORT_SENSOR_INDEX = 20,
    MBOTS_EXPORT_SPECIES_COUNT = 21,
    MBOTS_EXPORT_NUM_REFERENCE = 22,
    /* build extensions (not exported by the reference) */
    MBOTS_EXPORT_SPECIES = 32,           /* SpeciesObservation column     */
    MBOTS_EXPORT_PREV_SPECIES = 33       /* PrevSpeciesObservation column */
};

/* element types (madrona::py::TensorElementType subset) */
enum mbots_dtype {
    MBOTS_DTYPE_UINT8 = 0,
    MBOTS_DTYPE_INT8 = 1,
    MBOTS_DTYPE_INT32 = 2,
    MBOTS_DTYPE_FLOAT32 = 3
};

/* A non-owning 2-D tensor view (madrona::py::Tensor, mgr.cpp:70-76). */
typedef struct mbots_tensor {
    void   *data;        /* device pointer                                  */
    int32_t dtype;       /* enum mbots_dtype                                */
    int32_t device;      /* HIP device ordinal (gpuID); -1: host memory (CPU mode) */
    int64_t dims[2];     /* rows, columns                                   */
} mbots_tensor;

typedef struct mbots_handle mbots_handle;

/* Manager::Manager / Impl::make (mgr.cpp:98-172, :180-183).  Runs world init
 * (Sim::Sim, sim.cpp:1232-1256) and the Init graph (sim.cpp:1050-1059). */
int mbots_create(const mbots_config *cfg, mbots_handle **out);
/* Manager::~Manager (mgr.cpp:185-187) */
int mbots_destroy(mbots_handle *h);

/* Manager::step (mgr.cpp:51-63, :189-192): Step + Sensor graphs, enqueued on
 * `stream`.  Unlike the reference it does not block; mbots_num_agents and the
 * host-side offsets synchronise with the last step on demand. */
int mbots_step(mbots_handle *h, void *stream);
/* Manager::shiftObservations (mgr.cpp:65-68, :194-197) */
int mbots_shift_observations(mbots_handle *h, void *stream);

/* SimBridge::totalNumAgents (sim.hpp:74-78, sim.cpp:992-993).  Waits for the
 * last step's counters. */
int mbots_num_agents(mbots_handle *h, uint32_t *out);
/* Manager::exportTensor / the 11 tensor accessors (mgr.cpp:70-76, :199-422).
 * The reference's step() is synchronous (mgr.cpp:51-63), so its views are
 * valid on any stream; mbots_export keeps that contract: it returns after the
 * view's data is final (host-synchronising with the manager's last stream). */
int mbots_export(mbots_handle *h, int32_t export_id, mbots_tensor *out);
/* Stream-ordered form (what the Python surface uses): any deferred copy or
 * join the view needs is enqueued on `stream`, after everything the manager
 * enqueued on the stream of its previous call, so the view's data is final in
 * stream order on `stream`.  The view's row count (dims[0] = N) is host
 * state: the first call after a step waits once on the host for that step's
 * row counts (mbots_num_agents); the data copies and joins themselves do not
 * synchronise the host.  MBOTS_EXPORT_SENSOR_INDEX is computed on `stream`
 * and synchronised before returning. */
int mbots_export_on(mbots_handle *h, int32_t export_id, void *stream, mbots_tensor *out);
/* Manager::setAction (mgr.cpp:251-272): row = export row (species-major). */
int mbots_set_action(mbots_handle *h, uint32_t row, const int32_t action[6]);
/* Manager::agentOffsetForWorld (mgr.cpp:274-277) */
int mbots_agent_offset_for_world(mbots_handle *h, uint32_t world, uint32_t *out);

/* Learner observation rows (learn/util.py:14-29 construct_obs over every
 * species at once): out (device, >= out_rows x 69 f32, row-major) receives rows
 * [0, min(N, out_rows)) of [depth 32 | health 1 | position 2 | semantic 32 |
 * surrounding 2], exactly torch.cat's promotion of the exported views
 * (prev != 0: the Prev* views).  Launched on `stream` after the sensor rows. */
int mbots_construct_obs(mbots_handle *h, int32_t prev, float *out, uint64_t out_rows,
                        void *stream);

/* Rollout records for the learner-rank gather (BASELINE config 5):
 * the raw columns the reference's training loop reads after step()
 * (learn/training_loop.py:43-57, :87; learn/util.py:14-29), one fixed-size
 * record per export row, so a rank ships ~64 B per agent instead of the 276-B
 * f32 learner row:
 *   bytes  0..31  semantic (int8 x 32)        32..35  health (int32 bits)
 *         36..43  position (f32 x 2)          44..51  surrounding (f32 x 2)
 *         52..55  reward (f32)                56..59  stats (4 x uint8 flags)
 *         60..63  zero
 *         64..95  depth (uint8 x 32), only with MBOTS_FLAG_FIX_DEPTH_ALIAS
 * mbots_pack_rollout writes rows [0, min(N, out_rows)) into `out` (device
 * memory of the manager's GPU, 16-byte aligned; host memory in CPU mode). */
#define MBOTS_ROLLOUT_BYTES        64u
#define MBOTS_ROLLOUT_BYTES_DEPTH  96u
int mbots_rollout_record_bytes(mbots_handle *h, uint32_t *out);
int mbots_pack_rollout(mbots_handle *h, void *out, uint64_t out_rows, void *stream);
/* Learner side, no manager needed: `rows` gathered records (with_depth: the
 * 96-B form) -> obs [rows, 69] f32 exactly as mbots_construct_obs builds them,
 * reward [rows] f32 and stats [rows, 4] int32 (either may be NULL; records
 * and stats 16-B aligned on the device).  device >= 0: pointers are device memory of that GPU and the
 * kernel runs on `stream`; device == -1: host memory, done before returning. */
int mbots_unpack_rollout(const void *records, uint64_t rows, int32_t with_depth, int32_t device,
                         float *obs, float *reward, int32_t *stats, void *stream);

/* Learner records: the config-5 round trip (BASELINE config 5, SURVEY 8e
 * steps 1-3).  Everything learn/training_loop.py reads between step() and its
 * writes -- the rollout record above (current observation columns, reward,
 * stats: :49-50, :58), the previous observation columns (:87), Action (:47,
 * :93), HiddenState (:48, :58) and PrevHiddenState (:89) -- one record per
 * export row:
 *   bytes   0..63   the rollout record (bytes 60..63 zero)
 *          64..95   prev semantic        96..99   prev health (int32 bits)
 *         100..107  prev position       108..115  prev surrounding
 *         116..139  Action (int32 x 6)  140..143  zero
 *         144..207  HiddenState (f32 x 16)
 *         208..271  PrevHiddenState (f32 x 16)
 *         272..335  depth, prev depth (uint8 x 32 each), only with
 *                   MBOTS_FLAG_FIX_DEPTH_ALIAS
 * mbots_pack_learner writes rows [0, min(N, out_rows)) into `out` (16-byte
 * aligned device memory; host memory in CPU mode). */
#define MBOTS_LEARNER_BYTES        272u
#define MBOTS_LEARNER_BYTES_DEPTH  336u
int mbots_learner_record_bytes(mbots_handle *h, uint32_t *out);
int mbots_pack_learner(mbots_handle *h, void *out, uint64_t out_rows, void *stream);
/* Learner side (no manager): records -> any of these (NULL: skipped); obs and
 * prev_obs are construct_obs rows of the current / previous columns
 * (learn/util.py:14-29, bit-identical). */
typedef struct mbots_learner_out {
    float   *obs;          /* [rows, 69] */
    float   *prev_obs;     /* [rows, 69] */
    float   *reward;       /* [rows]     */
    int32_t *stats;        /* [rows, 4]  */
    int32_t *action;       /* [rows, 6]  */
    float   *hidden;       /* [rows, 16] */
    float   *prev_hidden;  /* [rows, 16] */
} mbots_learner_out;
int mbots_unpack_learner(const void *records, uint64_t rows, int32_t with_depth, int32_t device,
                         const mbots_learner_out *out, void *stream);
/* Slim learner records (config 5 with row provenance): the
 * learner record without Action, HiddenState and PrevHiddenState -- 152 B of
 * the 272 that only echo what the learner rank itself wrote (training_loop.py
 * :136-137) one and two steps back, reordered by the species sort.  In their
 * place the record carries each row's provenance: src, the row's index in the
 * table before this step (-1: born or respawned this step), from which the
 * learner rank rebuilds the three columns (harness/gather.py LearnerState):
 *   bytes   0..59   as the learner record       60..63   src (int32)
 *          64..115  as the learner record (the previous observation columns)
 *         116..127  zero
 *         128..191  depth, prev depth (uint8 x 32 each), only with
 *                   MBOTS_FLAG_FIX_DEPTH_ALIAS
 * The rebuilt columns equal the manager's as long as every row's Action and
 * HiddenState were written after the last step, after its shift(s) (the
 * learner's loop: step, gather, shift, write).  mbots_pack_learner_slim
 * moves none of the step's deferred columns: the previous observation rows
 * the step still owes are gathered inside its launch. */
#define MBOTS_LEARNER_SLIM_BYTES        128u
#define MBOTS_LEARNER_SLIM_BYTES_DEPTH  192u
int mbots_pack_learner_slim(mbots_handle *h, void *out, uint64_t out_rows, void *stream);
/* records -> obs, prev_obs, reward, stats of `out` (its action / hidden /
 * prev_hidden must be NULL) and src [rows] int32 (may be NULL) */
int mbots_unpack_learner_slim(const void *records, uint64_t rows, int32_t with_depth, int32_t device,
                              const mbots_learner_out *out, int32_t *src, void *stream);
/* The learner rank's rebuild from slim records (no manager): for every row r
 * of the gathered global table (species-major, per species rank-major: the
 * reassembly of harness/gather.py) with provenance src[r] (the owning rank's
 * row before the step, -1 new), its row g in the last global table, then
 *   action[r] = last_action[g], hidden[r] = last_memory[g],
 *   prev_hidden[r] = last_hidden[g]            (zeros for src = -1)
 * -- the learner's own writes after the last step and that step's
 * HiddenState, moved as the species sort moved the rows.  cur_counts /
 * last_counts: [ranks][4] species rows per rank of the gathered / the last
 * table (host memory, ranks <= MBOTS_MAX_LEARNER_RANKS).  device >= 0:
 * every array is device memory of that GPU (16-B aligned), on `stream`;
 * device == -1: host memory. */
#define MBOTS_MAX_LEARNER_RANKS 32u
int mbots_rebuild_learner(const int32_t *src, uint64_t rows, const int64_t *cur_counts,
                          const int64_t *last_counts, uint32_t ranks, const int32_t *last_action,
                          const float *last_memory, const float *last_hidden, uint64_t last_rows,
                          int32_t *action, float *hidden, float *prev_hidden, int32_t device,
                          void *stream);
/* The learner's writes (training_loop.py:136-137: action_tensor[...] = one_hot,
 * memory_tensor[...] = new_memory) for every row at once: `rows` rows of
 * Action [rows, 6] int32 and/or HiddenState [rows, 16] f32 (either may be
 * NULL) from memory of the manager's device (host memory in CPU mode) into
 * the current export table, rows [0, rows).  rows is N, or mbots_num_rows()
 * to also write the shard ghost's rows (the next shard's first world, which
 * then acts exactly as on the next rank). */
int mbots_write_actions(mbots_handle *h, const int32_t *action, const float *hidden, uint64_t rows,
                        void *stream);
/* every table row: N plus the shard ghost's (which follow row N) */
int mbots_num_rows(mbots_handle *h, uint32_t *out);
/* the largest world population after the last step (the shard ghost
 * included): waits for that step's row counts only (K2), not for its sensor
 * or the caller's chain -- what SimManager(agent_capacity="auto") checks
 * before each step (a step adds at most n births and A respawns) */
int mbots_max_population(mbots_handle *h, uint32_t *out);

/* Checkpoint / restore (the reference has none): the live state
 * after the last step (agent SoA, RNG keys/counters, food, the current export
 * table's N rows) as a host blob.  A manager created with the same
 * configuration continues bit-exactly after mbots_load_checkpoint -- also
 * one of another agent_capacity, when every world of the blob fits it (the
 * per-slot columns are re-laid out; a world that does not fit is refused
 * before anything is overwritten).  The Python SimManager's
 * agent_capacity="auto" grows a run through the capacity classes this way. */
int mbots_checkpoint_size(mbots_handle *h, uint64_t *bytes);
int mbots_save_checkpoint(mbots_handle *h, void *host_dst, uint64_t bytes);
int mbots_load_checkpoint(mbots_handle *h, const void *host_src, uint64_t bytes);
/* Debug dump of one world (viewer replacement): host arrays of agent_capacity
 * rows -- (x, y, rot.w, rot.z) f32, (species, health, finder) i32 -- the 48
 * packed food records, the food boxes' rotations ([5][48] 22-bit quarter-turn
 * fractions; may be NULL) and the live agent count. */
int mbots_world_state(mbots_handle *h, uint32_t world, float *xy_rwrz, int32_t *sp_hp_finder,
                      uint64_t *food, uint32_t *food_rot, int32_t *n_out);

/* Stream ordering: every call that takes a stream enqueues on it after all
 * work this manager enqueued on the stream of its previous call (an event
 * hop when the two differ; not across a graph capture's boundary).  That
 * previous stream must still exist when a call on another stream is made
 * (torch's pooled streams always do). */
/* Build utilities (benchmark / test harness, not reference API):
 * identity-keyed synthetic action stream: one-hot(threefry(seed,step |
 * global_world, slot) % 6) written into the Action column of every live agent;
 * hidden state gets hash-derived floats when write_hidden != 0. */
int mbots_write_synthetic_actions(mbots_handle *h, uint32_t seed, uint32_t step,
                                  int32_t write_hidden, void *stream);
/* Make `stream` wait for this manager's outstanding work on its internal
 * stream (the last step's sensor).  Every accessor that needs the sensor rows
 * does this itself; a caller recording steps into a HIP graph (stream capture)
 * ends the captured sequence with it, so the capture has no unjoined work. */
int mbots_join(mbots_handle *h, void *stream);
/* Record `event` (a hipEvent_t, timing-enabled) on the internal stream after
 * the last step's sensor: a timing point for benchmarks that adds no wait to
 * any stream (bench.py's device span: the later of this and an event on the
 * caller's stream).  No step yet, or CPU mode: MBOTS_E_INVALID. */
int mbots_record_sensor_done(mbots_handle *h, void *event);
/* running total of agent-steps (sum over steps of live agents after the step) */
int mbots_agent_steps(mbots_handle *h, uint64_t *out);
/* births/respawns dropped because a world reached agent_capacity */
int mbots_overflow(mbots_handle *h, uint64_t *out);
/* Per-kernel device timing (bench.py roofline): when enabled, HIP events are
 * recorded on the launch stream around every kernel; mbots_kernel_times
 * synchronises and returns the summed milliseconds per kernel class
 * (index = enum mbots_timed_kernel) and the number of launches of each. */
enum mbots_timed_kernel {
    MBOTS_TK_WORLD_STEP = 0, MBOTS_TK_SCAN = 1, MBOTS_TK_EXPORT = 2,
    MBOTS_TK_SENSOR = 3, MBOTS_TK_SHIFT = 4, MBOTS_TK_ACTIONS = 5, MBOTS_TK_MOVE = 6,
    MBOTS_TK_OBS = 7, MBOTS_TK_COUNT = 8
};
int mbots_enable_kernel_timing(mbots_handle *h, int32_t enable);
int mbots_kernel_times(mbots_handle *h, double ms[MBOTS_TK_COUNT],
                       uint64_t launches[MBOTS_TK_COUNT]);
/* The step schedule the manager chose (diagnostics, no device call):
 * out[0] flags -- 1 K1-finder mode (the next K1 does not wait for the last
 * sensor), 2 fork by value, 4 join by value, 8 MBOTS_SWAP, 16 mixed capacity
 * classes (MBOTS_MIXED); out[1] the last
 * value-wait epoch raised; out[2] how often the epochs restarted from 0;
 * out[3] steps run.  CPU mode: all 0 but out[3]. */
int mbots_schedule_info(mbots_handle *h, uint32_t out[4]);

const char *mbots_last_error(void);

/* Environment.
 * MBOTS_VALUE_FORK=0: the step's cross-stream hops (K1 -> the sensor's
 *   internal stream, and the sensor back to the next step) are event waits.
 *   Otherwise, from 2049 to 8192 worlds and while the host runs ahead of the
 *   device (up to 2048 the next step's K1 computes the finder slots itself and
 *   does not wait for the sensor; the fork is then an event wait),
 *   they are hipStreamWaitValue32 waits on signal words a kernel stores (about
 *   3 us instead of 7 per hop).  The runtime carries such a wait as a polling
 *   kernel on the waiting stream; a tool or mode that runs the device's
 *   kernels one at a time can dispatch that poller before its producer and
 *   never finish it, so the value waits are also off whenever one of
 *   MBOTS_SERIALISING_ENV is set (non-empty, not "0") when the manager is
 *   created: rocprofv3 counter collection, an HSA tools library, a legacy
 *   rocprof input file, or serialised kernel dispatch.
 * MBOTS_SWAP (read at mbots_create; above 8192 worlds): by default ("1") K1
 *   and K2 run on the internal stream before the sensor, with no cross-stream
 *   hop between them, and the caller's stream joins after K2 for the export
 *   rows (the sensor's chain sets the step's pace: -2 % against the forked
 *   schedule); MBOTS_SWAP=0 keeps K1 and K2 on the caller's stream and forks
 *   the sensor off after K2.
 * MBOTS_MIXED (read at mbots_create; agent_capacity above 128, outside the
 *   K1 finder mode): by default ("1") the 128-slot K1 and sensor run every
 *   world that fits them and the capacity class's kernels only the worlds K2
 *   lists (a world whose step could outgrow 128 slots, one with more than 128
 *   agents); MBOTS_MIXED=0 runs every world in the class's kernels (the same
 *   bits, slower).
 * MBOTS_CPU_THREADS: host threads of MBOTS_EXEC_CPU (default: the machine's
 *   hardware threads, at most 16).
 * MBOTS_EPOCH_START=<n> (read at mbots_create; a test hook): the value waits
 *   count their epochs on from n (at most 0x7FFFFFF0, where they restart
 *   from 0 after draining the device), so a short run crosses the restart. */
#define MBOTS_SERIALISING_ENV \
    { "ROCPROF_COUNTER_COLLECTION", "HSA_TOOLS_LIB", "ROCP_INPUT", "AMD_SERIALIZE_KERNEL", \
      "AMD_SERIALIZE_COPY" }

#ifdef __cplusplus
}
#endif
#endif
