// mbots_manager.cpp -- host orchestration (the reference's Manager,
// src/entry/mgr.cpp) behind the C ABI declared in include/mbots.h.
//
// MI355X-first differences from the reference Manager:
//  * no runtime compilation: kernels are ahead-of-time gfx950 code objects;
//  * every launch goes on the caller's HIP stream (torch's current stream), and
//    step() does not block -- the host-side agent count is fetched lazily by an
//    async D2H copy into pinned memory plus an event (mgr.cpp:57-62 did two
//    blocking cudaMemcpy per step);
//  * all device memory is one arena sized for `num_worlds * agent_capacity`
//    rows (288 GB HBM per GPU leaves ample headroom);
//  * the species-major export table is double-buffered: a step writes the new
//    table while reading the old one (no in-place radix sort of 264-B rows).
#if defined(MB_PROBE_NO_JOIN) && !defined(MB_PROBE_BUILD)
#error "MB_PROBE_NO_JOIN gives wrong finder slots: a probe build (scripts/build_var.sh -DMB_PROBE_BUILD) only"
#endif
#include <hip/hip_ext.h>
#include "../../include/mbots.h"
#include "mbots_kernels.hpp"
#include "mbots_cpu.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess)                                                              \
            return fail(MBOTS_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

struct Arena {
    char *base = nullptr;
    size_t used = 0, size = 0;
    template <typename T>
    T *take(size_t count)
    {
        size_t bytes = (count * sizeof(T) + 255) & ~size_t(255);
        T *p = reinterpret_cast<T *>(base + used);
        used += bytes;
        return p;
    }
};

struct TimedPair {
    hipEvent_t a, b;
    int kind;
};

}  // namespace

struct mbots_handle {
    mbots_config cfg{};
    std::unique_ptr<mbots::cpu::Sim> cpu;   // MBOTS_EXEC_CPU: the host world step
    int device = 0;
    mbots::SimState S{};
    mbots::ObsTable T[2]{};
    int tb = 0;
    int parity = 0;                   // K1 -> K2 tile-count buffer of this step
    Arena arena;
    int32_t *done_zeros = nullptr;    // Done column (never written, sim.cpp:74-75, B.7)
    int32_t *reset_zeros = nullptr;   // WorldReset singleton per world
    int32_t *sensor_index = nullptr;  // scratch for sensorIndexTensor
    uint32_t *h_totals = nullptr;     // pinned mirror of S.totals
    hipEvent_t ev_totals = nullptr;
    hipStream_t aux = nullptr;        // internal stream of the K3b sensor (forked after K2)
    hipEvent_t ev_join[2] = {nullptr, nullptr};   // K3b of alternate steps done (aux)
    int last_join = -1;               // ev_join of the latest K3b, -1: none pending
    unsigned long long join_capture = 0;   // stream-capture id it was recorded in (0: none)
    int prev_join = -1;               // ev_join of the K3b before it (its rows are the other
                                      // table half's), -1: none
    unsigned long long prev_capture = 0;
    uint64_t join_serial[2] = {0, 0}; // the sensor launch (1, 2, ...) each ev_join marks
    uint64_t sensor_serial = 0;       // sensors launched
    uint64_t waited_serial = 0;       // the newest sensor the manager's stream order has waited
                                      // for (outside graph capture; every call follows the last)
    bool k1_finder = false;           // K1 computes the finder slots (small world counts):
                                      // the next K1 does not wait for the sensor
    bool sensed = false;              // a sensor has run since init (the finder slots are then
                                      // the centre ray's, before it the init's "none")
    int32_t *row_base2[2] = {nullptr, nullptr};   // row bases / sensor order of alternate
    int32_t *sorder2[2] = {nullptr, nullptr};     // steps (a sensor may still read the last
                                                  // step's while the next K2 writes)
    int32_t *obsrow_out2[2] = {nullptr, nullptr}; // K1's old-row column of alternate steps (in
                                                  // K1-finder mode the sensor reads the last
                                                  // step's while the next K1 writes)
    unsigned long long cap_seen = 0;  // the stream capture the last captured step belonged to
    hipStream_t cap_stream = nullptr; // the stream it was recorded on (live while capturing)
    uint64_t cap_steps = 0;           // steps recorded into it (mbots_join wants an even count)
    bool poisoned = false;            // a graph of an odd number of steps was captured: the
                                      // host's table bookkeeping no longer follows the device
    uint32_t ovf_reported = 0;        // capacity drops reported so far (MBOTS_W_CAPACITY)
    // deferred K4 parts of a table half (moved from the other half along the
    // last src_of when needed): PrevAction / PrevHiddenState, the six other
    // Prev* columns (from the other half's current ones when six_lazy)
    bool cur_ah_pending[2] = {false, false};   // Action / HiddenState themselves
    bool psem_pending[2] = {false, false};     // the prev sensor (moved only when read: dead at
                                               // the next step)
    bool ah_pending[2] = {false, false};
    bool six_pending[2] = {false, false};
    bool six_lazy[2] = {false, false};
    // the half's current Action / HiddenState column is its Prev column: a
    // fused shift gathered the moved rows into PrevAction / PrevHiddenState only
    // (the learner overwrites the current ones next); readers go through
    // src_view, accessors copy first (materialize_cur_ah)
    bool a_alias[2] = {false, false};
    bool h_alias[2] = {false, false};
    bool prev_lazy[2] = {false, false};   // table half's six shift-owned Prev* columns are
                                          // still its current ones (lazy shift, K5)
    hipEvent_t ev_hop = nullptr;      // orders a call's stream after the last one used
    // the swapped schedule (above 8192 worlds unless MBOTS_SWAP=0): K1 and K2 on
    // the sensor's stream, the caller's stream joining after K2 (DESIGN.md 4
    // "Which chain sets the pace")
    bool swap = false;
    hipEvent_t ev_caller = nullptr;   // the caller's stream at a step's start
    uint32_t *sig_fork = nullptr;     // the fork's signal word (small world counts)
    uint32_t *sig_join = nullptr;     // the join's (raised after the sensor)
    uint32_t epoch = 0;               // the last epoch K2 raised (never 0)
    uint32_t epoch_wraps = 0;         // times the epochs restarted from 0 (kEpochWrap)
    uint32_t join_epoch = 0;          // the epoch raised after the last sensor (0: none;
                                      // the join is then the sensor's event)
    bool totals_ok = false;           // h_totals holds the last step's counts (synchronised)
    bool maxpop_stale = false;        // no K2 since a checkpoint load: the tile maxima are old
    int forced = 0;                   // deferred parts the caller's reads needed since the
                                      // last step (kMove*): the next step prefetches them
    int prefetched = 0;               // parts this step prefetched and no shift superseded
    uint64_t steps = 0;               // steps run
    hipStream_t last_stream = nullptr;
    bool timing = false;
    std::vector<TimedPair> pending;
    std::vector<hipEvent_t> pool;
    double acc_ms[MBOTS_TK_COUNT] = {};
    uint64_t acc_n[MBOTS_TK_COUNT] = {};
};

namespace {

// The fork (K2 -> the sensor's queue) as a hipStreamWaitValue32 on a flag K2's
// last block stores, instead of a wait on K2's completion signal: the hop is
// ~3 us instead of ~7 (scripts/ubench/hop_latency.hip).  At small world
// counts the step is a latency chain and that is -1 to -4 % at 4096 worlds;
// from 16384 on the chip is throughput-bound from K1's end on and the flag's
// fences cost about what the hop saves (±0 at 16384, +0.2-0.6 % at 65536), so
// events there (profiles/r04_value_fork_small_ab.jsonl,
// profiles/r04_value_waits_ab.jsonl, DESIGN_EXPERIMENTS.md round 4).
#ifndef MB_VALUE_FORK_MAX
#define MB_VALUE_FORK_MAX 8192
#endif
#ifndef MB_VALUE_JOIN
#define MB_VALUE_JOIN 1   // the join too: a one-wave kernel after the sensor raises it
#endif
#ifndef MB_VALUE_JOIN_MAX
#define MB_VALUE_JOIN_MAX 8192
#endif
#ifndef MB_FINDER_PSEM_BY_SENSOR
#define MB_FINDER_PSEM_BY_SENSOR 1   // K1-finder mode: the sensor moves the prev-sensor rows itself
#endif
#ifndef MB_SWAP_DEFAULT
#define MB_SWAP_DEFAULT 1   // MBOTS_SWAP's default (large world counts)
#endif
#ifndef MB_VALUE_ADAPT
#define MB_VALUE_ADAPT 1   // value waits only while the host runs ahead of the device
#endif
// Up to this many worlds K1 computes the next step's finder slots itself
// (world_finders), so the next K1 waits only for the caller's stream, not for
// this step's sensor: the sensor chain and the caller chain of consecutive
// steps overlap ("Small world counts")
#ifndef MB_FINDER_AUX_LOW
#define MB_FINDER_AUX_LOW 0
#endif
#ifndef MB_K1_FINDER_MAX
#define MB_K1_FINDER_MAX 2048
#endif
// The runtime carries the wait as a polling kernel on the sensor's queue, which
// spins until K2 (on the caller's queue) raises the flag: under a tool that runs
// the device's kernels one at a time (rocprofv3 counter collection,
// AMD_SERIALIZE_KERNEL) the poller can be dispatched first and never end, so
// those keep the event wait (as does MBOTS_VALUE_FORK=0).
// the value waits' epochs restart from 0 once they reach this (mbots_step)
constexpr uint32_t kEpochWrap = 0x7FFFFFF0u;
bool env_set(const char *name)
{
    const char *v = std::getenv(name);
    return v && *v && std::strcmp(v, "0") != 0;
}
// (the list and the switch are documented in include/mbots.h, "Environment")
bool value_waits_safe()
{
    const char *o = std::getenv("MBOTS_VALUE_FORK");
    if (o && std::strcmp(o, "0") == 0) return false;
    static const char *const kSerialising[] = MBOTS_SERIALISING_ENV;
    for (const char *name : kSerialising)
        if (env_set(name)) return false;
    return true;
}
// (K1-finder mode: the caller's chain no longer waits for the sensor, and the
// value fork's 5.5 us enqueue lands on that chain's host time; an event fork
// measured -5 % at 2048 worlds)
bool fork_by_value(uint32_t W) { return W <= MB_VALUE_FORK_MAX && W > MB_K1_FINDER_MAX && value_waits_safe(); }
bool join_by_value(uint32_t W)
{
    return MB_VALUE_JOIN && W <= MB_VALUE_JOIN_MAX && W > MB_K1_FINDER_MAX && value_waits_safe();
}

hipEvent_t get_event(mbots_handle *h)
{
    if (!h->pool.empty()) {
        hipEvent_t e = h->pool.back();
        h->pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

template <typename F>
int timed(mbots_handle *h, int kind, hipStream_t st, F &&launch)
{
    TimedPair tp{nullptr, nullptr, kind};
    if (h->timing) {
        tp.a = get_event(h);
        tp.b = get_event(h);
        HIP_TRY(hipEventRecord(tp.a, st));
    }
    HIP_TRY(launch());
    if (h->timing) {
        HIP_TRY(hipEventRecord(tp.b, st));
        h->pending.push_back(tp);
    }
    return MBOTS_OK;
}

void fill_table(mbots::ObsTable &t, Arena &a, size_t rows)
{
    using namespace mbots;
    t.species = a.take<int32_t>(rows);
    t.pos = a.take<float>(rows * 2);
    t.health = a.take<int32_t>(rows);
    t.sur = a.take<float>(rows * 2);
    t.reward = a.take<float>(rows);
    t.action = a.take<int32_t>(rows * 6);
    t.stats = a.take<int32_t>(rows * 4);
    t.hidden = a.take<float>(rows * kHidden);
    t.sem = a.take<int8_t>(rows * kSensor);
    t.depth = a.take<uint8_t>(rows * kSensor);
    t.pspecies = a.take<int32_t>(rows);
    t.ppos = a.take<float>(rows * 2);
    t.phealth = a.take<int32_t>(rows);
    t.psur = a.take<float>(rows * 2);
    t.preward = a.take<float>(rows);
    t.paction = a.take<int32_t>(rows * 6);
    t.pstats = a.take<int32_t>(rows * 4);
    t.phidden = a.take<float>(rows * kHidden);
    t.psem = a.take<int8_t>(rows * kSensor);
    t.pdepth = a.take<uint8_t>(rows * kSensor);
}

size_t layout(mbots_handle *h, Arena &a)
{
    using namespace mbots;
    const size_t W = h->S.W, cap = h->cfg.agent_capacity, rows = W * cap;
    SimState &S = h->S;
    S.x = a.take<float>(rows);
    S.y = a.take<float>(rows);
    S.rw = a.take<float>(rows);
    S.rz = a.take<float>(rows);
    S.species = a.take<int32_t>(rows);
    S.health = a.take<int32_t>(rows);
    S.finder = a.take<int32_t>(rows);
    S.obsrow = a.take<int32_t>(rows);
    S.sur0 = a.take<float>(rows);
    S.sur1 = a.take<float>(rows);
    S.stats = a.take<uint32_t>(rows);
    S.n = a.take<int32_t>(W);
    S.ctr = a.take<uint32_t>(W);
    S.key = a.take<uint2>(W);
    S.food = a.take<uint64_t>(W * kNumChunks);
    S.food_rot = a.take<uint32_t>(W * kNumPkg);
    S.cur_food = a.take<int32_t>(W);
    S.sreward = a.take<float>(W * kNumSpecies);
    S.scount = a.take<int32_t>(W * kNumSpecies);
    h->row_base2[0] = a.take<int32_t>(W * kNumSpecies);
    h->row_base2[1] = a.take<int32_t>(W * kNumSpecies);
    S.row_base = h->row_base2[0];
    S.world_off = a.take<int32_t>(W);
    S.src_of = a.take<int32_t>(rows);
    S.overflow = a.take<uint32_t>(W);
    S.fork_ctr = a.take<uint32_t>(1);
    S.totals = a.take<uint32_t>(8);
    S.ntiles = scan_tiles((uint32_t)W);
    S.tiles = a.take<int32_t>((size_t)2 * S.ntiles * kTileBuckets * 5);
    S.agent_steps = a.take<unsigned long long>(1);
    S.raytab = a.take<float4>(36);
    S.big_k1 = a.take<int32_t>(2 * W);   // mixed capacity classes (K2's lists)
    S.big_s = a.take<int32_t>(2 * W);
    S.big_cnt = a.take<uint32_t>(4);
    h->sorder2[0] = h->sorder2[1] = nullptr;
    if (sensor_order_used((uint32_t)W)) {
        h->sorder2[0] = a.take<int32_t>(W);
        h->sorder2[1] = a.take<int32_t>(W);
    }
    S.sorder = h->sorder2[0];
    S.x_out = a.take<float>(rows);
    S.y_out = a.take<float>(rows);
    S.rw_out = a.take<float>(rows);
    S.rz_out = a.take<float>(rows);
    S.species_out = a.take<int32_t>(rows);
    h->obsrow_out2[0] = a.take<int32_t>(rows);
    h->obsrow_out2[1] = a.take<int32_t>(rows);
    S.obsrow_out = h->obsrow_out2[0];
    S.n_out = a.take<int32_t>(W);
    S.food_out = a.take<uint64_t>(W * kNumChunks);
    fill_table(h->T[0], a, rows);
    fill_table(h->T[1], a, rows);
    h->done_zeros = a.take<int32_t>(rows);
    h->reset_zeros = a.take<int32_t>(W);
    h->sensor_index = a.take<int32_t>(rows);
    return a.used;
}

hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// table half `half` as its readers see it: an aliased current Action /
// HiddenState column read from its Prev column
mbots::ObsTable src_view(const mbots_handle *h, int half)
{
    mbots::ObsTable t = h->T[half];
    if (h->a_alias[half]) t.action = t.paction;
    if (h->h_alias[half]) t.hidden = t.phidden;
    return t;
}

bool capturing(hipStream_t st);
// make `st` wait for the last step's sensor (its rows, and the moves it did)
int wait_sensor(mbots_handle *h, hipStream_t st)
{
    if (h->last_join >= 0) {
        HIP_TRY(hipStreamWaitEvent(st, h->ev_join[h->last_join], 0));
        if (!capturing(st)) h->waited_serial = std::max(h->waited_serial, h->join_serial[h->last_join]);
    }
    return MBOTS_OK;
}

// make `st` wait for the sensor before the last one, whose rows are the other
// table half's (the prev-sensor moves read them).  Only needed when K1 does
// not wait for the sensors (k1_finder): otherwise the last step's K1 did.
// (Under stream capture, only an event recorded in the same capture.)
int wait_prev_sensor(mbots_handle *h, hipStream_t st)
{
    if (!h->k1_finder || h->prev_join < 0) return MBOTS_OK;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    unsigned long long cid = 0;
    HIP_TRY(hipStreamGetCaptureInfo(st, &cs, &cid));
    const bool cap = cs == hipStreamCaptureStatusActive;
    if (cap && h->prev_capture != cid) return MBOTS_OK;
    // (one cross-queue wait per step: the shift's for its prev-sensor rows
    // covers the next K1's)
    if (!cap && h->waited_serial >= h->join_serial[h->prev_join]) return MBOTS_OK;
    HIP_TRY(hipStreamWaitEvent(st, h->ev_join[h->prev_join], 0));
    if (!cap) h->waited_serial = std::max(h->waited_serial, h->join_serial[h->prev_join]);
    return MBOTS_OK;
}

bool capturing(hipStream_t st)
{
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive;
}

// A graph captured with an odd number of steps leaves the table halves and the
// host's deferred-move bookkeeping out of step with the device after a replay
// (ADVICE r3/r4): every device entry point refuses to run from then on --
// checked here (use_stream, sync_totals and the entry points that use neither)
// and by mbots_step when the next capture starts.
// (only a capture that has ENDED with an odd count poisons; a call
// on another stream while the capture is still recording is refused alone)
bool capture_open(const mbots_handle *h)
{
    if (!h->cap_stream || !h->cap_seen) return false;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    unsigned long long cid = 0;
    if (hipStreamGetCaptureInfo(h->cap_stream, &cs, &cid) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return cs == hipStreamCaptureStatusActive && cid == h->cap_seen;
}

int capture_guard(mbots_handle *h, hipStream_t st)
{
    static const char *kMsg = "the last graph capture recorded an odd number of steps, so the manager's "
                              "table halves no longer follow the device; capture an even number of steps "
                              "(ending with join()) and create a new manager";
    if (h->poisoned) return fail(MBOTS_E_INVALID, kMsg);
    if ((h->cap_steps & 1) && !capturing(st)) {
        if (capture_open(h))
            return fail(MBOTS_E_INVALID, "a graph capture of this manager's steps is still recording on another "
                                         "stream: call the manager on the capturing stream, or after the "
                                         "capture has ended");
        h->poisoned = true;
        return fail(MBOTS_E_INVALID, kMsg);
    }
    return MBOTS_OK;
}

// Every call enqueues on the caller's stream (torch's current stream); a call
// on another stream than the previous one is ordered after everything the
// manager enqueued there (an event hop), so steps, deferred copies and the
// views they produce form one stream-ordered sequence whatever streams the
// caller switches between.  (Not across a graph capture's boundary: a capture
// cannot wait for work outside it.)
int use_stream(mbots_handle *h, hipStream_t st)
{
    if (int rc = capture_guard(h, st)) return rc;
    if (st != h->last_stream && !capturing(st) && !capturing(h->last_stream)) {
        HIP_TRY(hipEventRecord(h->ev_hop, h->last_stream));
        HIP_TRY(hipStreamWaitEvent(st, h->ev_hop, 0));
    }
    h->last_stream = st;
    return MBOTS_OK;
}

// copy the six Prev* columns a lazy shift left as views of the current ones
// (on the stream the caller uses next)
int materialize_prev(mbots_handle *h, hipStream_t st)
{
    if (h->six_pending[h->tb]) {   // a step's deferred move (no shift since)
        HIP_TRY(hipSetDevice(h->device));
        const int rc = timed(h, MBOTS_TK_MOVE, st, [&] {
            return mbots::launch_move(h->S, h->T[h->tb ^ 1], h->T[h->tb], h->six_lazy[h->tb] ? 1 : 0,
                                      mbots::kMovePrev6, st);
        });
        if (rc) return rc;
        h->six_pending[h->tb] = false;
        return MBOTS_OK;
    }
    if (!h->prev_lazy[h->tb]) return MBOTS_OK;
    HIP_TRY(hipSetDevice(h->device));
    const int rc = timed(h, MBOTS_TK_MOVE, st,
                         [&] { return mbots::launch_shift(h->S, h->T[h->tb], mbots::kShiftRest, st); });
    if (rc) return rc;
    h->prev_lazy[h->tb] = false;
    return MBOTS_OK;
}

// the deferred K4 part: PrevAction / PrevHiddenState of the current half from
// the other half, along the last step's src_of (both intact until the next
// step's K3a / K4)
int materialize_cur_ah(mbots_handle *h, hipStream_t st, int alias_cols);
int materialize_prev_ah(mbots_handle *h, hipStream_t st)
{
    if (!h->ah_pending[h->tb]) return MBOTS_OK;
    // the Prev storage holds the current columns (aliased): copied out before
    // the Prev move overwrites it
    const int cols = (h->a_alias[h->tb] ? 1 : 0) | (h->h_alias[h->tb] ? 2 : 0);
    if (cols) {
        const int rc = materialize_cur_ah(h, st, cols);
        if (rc) return rc;
    }
    HIP_TRY(hipSetDevice(h->device));
    const int rc = timed(h, MBOTS_TK_MOVE, st, [&] {
        return mbots::launch_move(h->S, h->T[h->tb ^ 1], h->T[h->tb], 0, mbots::kMovePrevAH, st);
    });
    if (rc) return rc;
    h->ah_pending[h->tb] = false;
    return MBOTS_OK;
}

// the deferred Action / HiddenState move of the current half (K1, the learner
// and every accessor of the two columns need it; a shift fuses it); then the
// columns of `alias_cols` (1 Action, 2 HiddenState) a fused shift left as
// views of their Prev columns are copied out
int sync_totals(mbots_handle *h);
int materialize_cur_ah(mbots_handle *h, hipStream_t st, int alias_cols)
{
    const int tb = h->tb;
    if (h->cur_ah_pending[tb]) {
        HIP_TRY(hipSetDevice(h->device));
        const mbots::ObsTable src = src_view(h, tb ^ 1);
        const int rc = timed(h, MBOTS_TK_MOVE, st, [&] {
            return mbots::launch_move(h->S, src, h->T[tb], 0, mbots::kMoveAH, st);
        });
        if (rc) return rc;
        h->cur_ah_pending[tb] = false;
    }
    const bool ca = (alias_cols & 1) && h->a_alias[tb], ch = (alias_cols & 2) && h->h_alias[tb];
    if (!ca && !ch) return MBOTS_OK;
    HIP_TRY(hipSetDevice(h->device));
    int rc = sync_totals(h);
    if (rc) return rc;
    const size_t N = h->h_totals[mbots::kTotRows];   // the shard ghost's rows included
    const mbots::ObsTable &t = h->T[tb];
    rc = timed(h, MBOTS_TK_MOVE, st, [&] {
        hipError_t e = hipSuccess;
        if (ca && N) e = hipMemcpyAsync(t.action, t.paction, N * 6 * sizeof(int32_t), hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess && ch && N)
            e = hipMemcpyAsync(t.hidden, t.phidden, N * mbots::kHidden * sizeof(float), hipMemcpyDeviceToDevice, st);
        return e;
    });
    if (rc) return rc;
    if (ca) h->a_alias[tb] = false;
    if (ch) h->h_alias[tb] = false;
    return MBOTS_OK;
}

// the deferred prev-sensor move of the current half (accessors of the prev
// sensor, construct_obs(prev), checkpoints, the next step; a shift fuses it)
int materialize_psem(mbots_handle *h, hipStream_t st)
{
    if (!h->psem_pending[h->tb]) return MBOTS_OK;
    HIP_TRY(hipSetDevice(h->device));
    if (int rc = wait_prev_sensor(h, st)) return rc;   // its source rows are that sensor's
    const int rc = timed(h, MBOTS_TK_MOVE, st, [&] {
        return mbots::launch_move(h->S, h->T[h->tb ^ 1], h->T[h->tb], 0, mbots::kMoveSensor, st);
    });
    if (rc) return rc;
    h->psem_pending[h->tb] = false;
    return MBOTS_OK;
}

// deferred parts still owed by the current half (kMove* bits)
int pending_mask(const mbots_handle *h)
{
    const int tb = h->tb;
    return (h->cur_ah_pending[tb] ? mbots::kMoveAH : 0) | (h->psem_pending[tb] ? mbots::kMoveSensor : 0) |
           (h->ah_pending[tb] ? mbots::kMovePrevAH : 0) | (h->six_pending[tb] ? mbots::kMovePrev6 : 0);
}

// a caller's read that needs the parts `need`: the ones the step deferred
// (owed when the read came) or prefetched are remembered for the next step
void note_use(mbots_handle *h, int need, int owed)
{
    h->forced |= need & (owed | h->prefetched);
}

// the stream the manager last launched on is being captured into a graph
bool capturing_now(const mbots_handle *h)
{
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(h->last_stream, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive;
}

int sync_totals(mbots_handle *h)
{
    // the step's row counts are final once synchronised: later accessors of the
    // same step skip the runtime calls (the reference loop reads ~10 views per
    // step and is host-bound at small world counts, scripts/refhost.py) -- not
    // once graphs exist, whose replays change the counts behind the host's back
    if (int rc = capture_guard(h, h->last_stream)) return rc;
    if (h->totals_ok && h->cap_seen == 0) return MBOTS_OK;
    HIP_TRY(hipSetDevice(h->device));
    // a host-side row count during stream capture would be the capture-time
    // count baked into every replay (and the event wait is not capturable)
    if (capturing_now(h))
        return fail(MBOTS_E_INVALID,
                    "needs the host-side agent count, which is not available while the stream is "
                    "captured into a graph: capture only step / shift_observations / "
                    "write_synthetic_actions / join (device-side writers), read accessors after replay");
    HIP_TRY(hipEventSynchronize(h->ev_totals));
    h->totals_ok = true;
    return MBOTS_OK;
}

int record_totals(mbots_handle *h, hipStream_t st)
{
    HIP_TRY(hipMemcpyAsync(h->h_totals, h->S.totals, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           st));
    HIP_TRY(hipEventRecord(h->ev_totals, st));
    return MBOTS_OK;
}

}  // namespace

// checkpoint segments (mbots_save_checkpoint / mbots_load_checkpoint)
namespace {
struct CkptHeader {
    char magic[8];
    uint32_t version, num_worlds, cap, A, world_offset, flags, seed, n_rows;
    uint64_t bytes;
    uint32_t sensed, pad;   // 4: whether a sensor had run (the finder slots are its)
};
// 3: totals[kTotRows] (every table row, the shard ghost's included) is part
// of the state and must equal the header's n_rows; 4: `sensed`
constexpr uint32_t kCkptVersion = 4;

struct Seg {
    void *p;
    size_t bytes;
};

// the first kSlotSegs segments are per-slot columns ([world][cap]); `cap`:
// the capacity the segments are sized for (0: the manager's)
constexpr size_t kSlotSegs = 11;
std::vector<Seg> ckpt_segments(mbots_handle *h, mbots::ObsTable &t, uint32_t n_rows, uint32_t cap = 0)
{
    using namespace mbots;
    SimState &S = h->S;
    const size_t W = S.W, rows = W * (cap ? cap : h->cfg.agent_capacity), N = n_rows;
    std::vector<Seg> v = {
        {S.x, rows * 4}, {S.y, rows * 4}, {S.rw, rows * 4}, {S.rz, rows * 4},
        {S.species, rows * 4}, {S.health, rows * 4}, {S.finder, rows * 4}, {S.obsrow, rows * 4},
        {S.sur0, rows * 4}, {S.sur1, rows * 4}, {S.stats, rows * 4},
        {S.n, W * 4}, {S.ctr, W * 4}, {S.key, W * 8}, {S.food, W * kNumChunks * 8},
        {S.food_rot, W * kNumPkg * 4},
        {S.cur_food, W * 4}, {S.sreward, W * kNumSpecies * 4}, {S.scount, W * kNumSpecies * 4},
        {S.row_base, W * kNumSpecies * 4}, {S.world_off, W * 4}, {S.overflow, W * 4},
        {S.totals, 8 * 4}, {S.agent_steps, 8},
        {t.species, N * 4}, {t.pos, N * 8}, {t.health, N * 4}, {t.sur, N * 8}, {t.reward, N * 4},
        {t.action, N * 24}, {t.stats, N * 16}, {t.hidden, N * kHidden * 4},
        {t.sem, N * kSensor}, {t.depth, N * kSensor},
        {t.pspecies, N * 4}, {t.ppos, N * 8}, {t.phealth, N * 4}, {t.psur, N * 8},
        {t.preward, N * 4}, {t.paction, N * 24}, {t.pstats, N * 16}, {t.phidden, N * kHidden * 4},
        {t.psem, N * kSensor}, {t.pdepth, N * kSensor},
    };
    return v;
}

size_t ckpt_bytes(const std::vector<Seg> &v)
{
    size_t b = sizeof(CkptHeader);
    for (const Seg &s : v) b += s.bytes;
    return b;
}
// rollout records on the host (CPU mode, and the learner side of a gather
// that landed in host memory): the layout of include/mbots.h, the values of
// pack_rollout_kernel / unpack_rollout_kernel (plain bit copies and the
// uint8 / int8 -> f32 conversions of construct_obs)
void pack_rollout_host(const int8_t *sem, const uint8_t *depth, const int32_t *health, const float *pos,
                       const float *sur, const float *reward, const int32_t *stats, uint64_t n, uint8_t *out)
{
    const size_t rec = depth ? MBOTS_ROLLOUT_BYTES_DEPTH : MBOTS_ROLLOUT_BYTES;
    for (uint64_t r = 0; r < n; ++r) {
        uint8_t *o = out + r * rec;
        memcpy(o, sem + r * mbots::kSensor, 32);
        memcpy(o + 32, health + r, 4);
        memcpy(o + 36, pos + 2 * r, 8);
        memcpy(o + 44, sur + 2 * r, 8);
        memcpy(o + 52, reward + r, 4);
        for (int k = 0; k < 4; ++k) o[56 + k] = (uint8_t)stats[4 * r + k];
        memset(o + 60, 0, 4);
        if (depth) memcpy(o + 64, depth + r * mbots::kSensor, 32);
    }
}

void unpack_rollout_host(const uint8_t *recs, uint64_t n, bool with_depth, float *obs, float *reward,
                         int32_t *stats)
{
    const size_t rec = with_depth ? MBOTS_ROLLOUT_BYTES_DEPTH : MBOTS_ROLLOUT_BYTES;
    for (uint64_t r = 0; r < n; ++r) {
        const uint8_t *q = recs + r * rec;
        float *o = obs + r * 69;
        const uint8_t *d = with_depth ? q + 64 : q;
        for (int c = 0; c < 32; ++c) o[c] = (float)d[c];
        memcpy(o + 32, q + 32, 12);   // health bits, position
        for (int c = 0; c < 32; ++c) o[35 + c] = (float)(int8_t)q[c];
        memcpy(o + 67, q + 44, 8);    // surroundings
        if (reward) memcpy(reward + r, q + 52, 4);
        if (stats)
            for (int k = 0; k < 4; ++k) stats[4 * r + k] = q[56 + k];
    }
}

// learner records on the host (CPU mode, and a gather that landed in host
// memory): the layout of include/mbots.h, the values of pack_learner_kernel /
// unpack_learner_kernel
void pack_learner_host(const mbots::cpu::Table &t, bool fixd, uint64_t n, uint8_t *out)
{
    const size_t rec = fixd ? MBOTS_LEARNER_BYTES_DEPTH : MBOTS_LEARNER_BYTES;
    for (uint64_t r = 0; r < n; ++r) {
        uint8_t *o = out + r * rec;
        pack_rollout_host(t.sem.data() + r * mbots::kSensor, nullptr, t.health.data() + r, t.pos.data() + 2 * r,
                          t.sur.data() + 2 * r, t.reward.data() + r, t.stats.data() + 4 * r, 1, o);
        memcpy(o + 64, t.psem.data() + r * mbots::kSensor, 32);
        memcpy(o + 96, t.phealth.data() + r, 4);
        memcpy(o + 100, t.ppos.data() + 2 * r, 8);
        memcpy(o + 108, t.psur.data() + 2 * r, 8);
        memcpy(o + 116, t.action.data() + 6 * r, 24);
        memset(o + 140, 0, 4);
        memcpy(o + 144, t.hidden.data() + mbots::kHidden * r, 64);
        memcpy(o + 208, t.phidden.data() + mbots::kHidden * r, 64);
        if (fixd) {
            memcpy(o + 272, t.depth.data() + r * mbots::kSensor, 32);
            memcpy(o + 304, t.pdepth.data() + r * mbots::kSensor, 32);
        }
    }
}

// slim learner records on the host (CPU mode: every column materialised)
void pack_learner_slim_host(const mbots::cpu::Table &t, const int32_t *src_of, bool fixd, uint64_t n,
                            uint8_t *out)
{
    const size_t rec = fixd ? MBOTS_LEARNER_SLIM_BYTES_DEPTH : MBOTS_LEARNER_SLIM_BYTES;
    for (uint64_t r = 0; r < n; ++r) {
        uint8_t *o = out + r * rec;
        pack_rollout_host(t.sem.data() + r * mbots::kSensor, nullptr, t.health.data() + r, t.pos.data() + 2 * r,
                          t.sur.data() + 2 * r, t.reward.data() + r, t.stats.data() + 4 * r, 1, o);
        memcpy(o + 60, src_of + r, 4);
        memcpy(o + 64, t.psem.data() + r * mbots::kSensor, 32);
        memcpy(o + 96, t.phealth.data() + r, 4);
        memcpy(o + 100, t.ppos.data() + 2 * r, 8);
        memcpy(o + 108, t.psur.data() + 2 * r, 8);
        memset(o + 116, 0, 12);
        if (fixd) {
            memcpy(o + 128, t.depth.data() + r * mbots::kSensor, 32);
            memcpy(o + 160, t.pdepth.data() + r * mbots::kSensor, 32);
        }
    }
}

void unpack_learner_host(const uint8_t *recs, uint64_t n, bool fixd, const mbots_learner_out &o, bool slim = false,
                         int32_t *src = nullptr)
{
    const size_t rec = slim ? (fixd ? MBOTS_LEARNER_SLIM_BYTES_DEPTH : MBOTS_LEARNER_SLIM_BYTES)
                            : (fixd ? MBOTS_LEARNER_BYTES_DEPTH : MBOTS_LEARNER_BYTES);
    const size_t dc = slim ? 128 : 272, dp = slim ? 160 : 304;
    for (uint64_t r = 0; r < n; ++r) {
        const uint8_t *q = recs + r * rec;
        if (src) memcpy(src + r, q + 60, 4);
        for (int prev = 0; prev < 2; ++prev) {
            float *ob = prev ? o.prev_obs : o.obs;
            if (!ob) continue;
            ob += r * 69;
            const uint8_t *b = q + (prev ? 64 : 0);
            const uint8_t *d = fixd ? q + (prev ? dp : dc) : b;
            for (int c = 0; c < 32; ++c) ob[c] = (float)d[c];
            memcpy(ob + 32, b + 32, 12);   // health bits, position
            for (int c = 0; c < 32; ++c) ob[35 + c] = (float)(int8_t)b[c];
            memcpy(ob + 67, b + 44, 8);    // surroundings
        }
        if (o.reward) memcpy(o.reward + r, q + 52, 4);
        if (o.stats)
            for (int k = 0; k < 4; ++k) o.stats[4 * r + k] = q[56 + k];
        if (slim) continue;
        if (o.action) memcpy(o.action + 6 * r, q + 116, 24);
        if (o.hidden) memcpy(o.hidden + mbots::kHidden * r, q + 144, 64);
        if (o.prev_hidden) memcpy(o.prev_hidden + mbots::kHidden * r, q + 208, 64);
    }
}

}  // namespace

extern "C" {

const char *mbots_last_error(void) { return g_err.c_str(); }

int mbots_create(const mbots_config *cfg_in, mbots_handle **out)
{
    if (!cfg_in || !out) return fail(MBOTS_E_INVALID, "null argument");
    *out = nullptr;
    mbots_config cfg = *cfg_in;
    if (cfg.agent_capacity == 0) cfg.agent_capacity = 128;
    if (cfg.sensor_size == 0) cfg.sensor_size = 32;
    if (cfg.num_worlds == 0) return fail(MBOTS_E_INVALID, "num_worlds must be > 0");
    if (cfg.sensor_size != (uint32_t)mbots::kSensor)
        return fail(MBOTS_E_INVALID, "sensor_size must be 32 (mgr.hpp:19, entry.cpp:27)");
    static_assert(mbots::kMaxCap == (int)MBOTS_MAX_CAPACITY, "include/mbots.h");
    if (cfg.agent_capacity > (uint32_t)mbots::kMaxCap || cfg.agent_capacity < 4)
        return fail(MBOTS_E_INVALID, "agent_capacity must be in [4, " + std::to_string(mbots::kMaxCap) + "]");
    if (cfg.init_num_agents_per_world > cfg.agent_capacity)
        return fail(MBOTS_E_INVALID, "init_num_agents_per_world exceeds agent_capacity");
    if (cfg.init_num_agents_per_world < (uint32_t)mbots::kNumSpecies)
        return fail(MBOTS_E_INVALID, "init_num_agents_per_world must be >= 4");
    const uint64_t rows = (uint64_t)cfg.num_worlds * cfg.agent_capacity;
    if (rows >= (1ull << 31)) return fail(MBOTS_E_INVALID, "num_worlds * agent_capacity >= 2^31");
    if (cfg.exec_mode != MBOTS_EXEC_HIP && cfg.exec_mode != MBOTS_EXEC_CPU)
        return fail(MBOTS_E_INVALID, "exec_mode must be MBOTS_EXEC_HIP or MBOTS_EXEC_CPU");
    if (cfg.exec_mode == MBOTS_EXEC_CPU) {   // no HIP call on this path: runs without a GPU
        mbots_handle *h = new (std::nothrow) mbots_handle();
        if (!h) return fail(MBOTS_E_NOMEM, "host allocation failed");
        h->cfg = cfg;
        h->device = -1;
        try {
            h->cpu = std::make_unique<mbots::cpu::Sim>(cfg);
        } catch (const std::bad_alloc &) {
            delete h;
            return fail(MBOTS_E_NOMEM, "host allocation of the CPU-mode state failed");
        }
        *out = h;
        return MBOTS_OK;
    }

    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (cfg.gpu_id < 0 || cfg.gpu_id >= ndev)
        return fail(MBOTS_E_INVALID, "gpu_id out of range (" + std::to_string(ndev) + " devices)");
    HIP_TRY(hipSetDevice(cfg.gpu_id));

    mbots_handle *h = new mbots_handle();
    h->cfg = cfg;
    h->device = cfg.gpu_id;
    // the shard ghost is one more simulated world (the last), never exported
    h->S.W = cfg.num_worlds + ((cfg.flags & MBOTS_FLAG_SHARD_GHOST) ? 1u : 0u);
    h->S.Wx = cfg.num_worlds;
    Arena probe;
    const size_t bytes = layout(h, probe);
    if (hipMalloc(&h->arena.base, bytes) != hipSuccess) {
        delete h;
        return fail(MBOTS_E_NOMEM, "hipMalloc of " + std::to_string(bytes) + " bytes failed");
    }
    h->arena.size = bytes;
    h->arena.used = 0;
    layout(h, h->arena);
    mbots::SimState &S = h->S;
    S.cap = cfg.agent_capacity;
    S.A = cfg.init_num_agents_per_world;
    S.world_offset = cfg.world_offset;
    S.flags = cfg.flags;
    S.seed = cfg.rand_seed;
    // (the K1 finder pass keeps camera slots in bytes: a <= 256-slot mode)
    h->k1_finder = S.W <= MB_K1_FINDER_MAX && S.cap <= 256;
    S.k1_finder = h->k1_finder ? 1u : 0u;
    {
        // mixed capacity classes (round 6): above 128 slots the 128-slot K1
        // and sensor take every world that fits them and the class kernels
        // only the worlds K2 lists (DESIGN.md "Capacity"); MBOTS_MIXED=0 runs
        // every world in the class kernels
        const char *e = std::getenv("MBOTS_MIXED");
        const bool want = !(e && *e == '0');
        S.mixed = (want && S.cap > (uint32_t)mbots::kSmallCap && !h->k1_finder) ? 1u : 0u;
    }

    int rc = MBOTS_OK;
    auto check = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && rc == MBOTS_OK)
            rc = fail(MBOTS_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
    };
    // (8 totals, then each scan tile's largest world: mbots_max_population)
    check(hipHostMalloc((void **)&h->h_totals, ((size_t)mbots::kTotMaxPop + S.ntiles) * sizeof(uint32_t),
                        hipHostMallocMapped),
          "hipHostMalloc");
    if (rc == MBOTS_OK)
        check(hipHostGetDevicePointer((void **)&S.totals_host, h->h_totals, 0),
              "hipHostGetDevicePointer");
    // (these ride on kernel dispatches as their stop events; synchronisation
    // only: no timestamps, and a device-scope release -- the host reads only the
    // pinned row counts, which K2 writes system-coherent and fences itself)
    constexpr unsigned kSyncEvent = hipEventDisableTiming | hipEventReleaseToDevice;
    check(hipEventCreateWithFlags(&h->ev_totals, kSyncEvent), "hipEventCreateWithFlags");
    check(hipEventCreateWithFlags(&h->ev_hop, kSyncEvent), "hipEventCreateWithFlags");
    {
        // the words hipStreamWaitValue32 polls (the runtime's wait kernel reads
        // them); without signal memory the waits stay event waits
        auto signal_word = [&](uint32_t *&p) {
            if (rc != MBOTS_OK) return;
            if (hipExtMallocWithFlags((void **)&p, 8, hipMallocSignalMemory) != hipSuccess) {
                (void)hipGetLastError();
                p = nullptr;
                return;
            }
            check(hipMemset(p, 0, 8), "hipMemset");
        };
        if (fork_by_value((uint32_t)S.W)) signal_word(h->sig_fork);
        if (join_by_value((uint32_t)S.W)) signal_word(h->sig_join);
        S.sig_fork = h->sig_fork;
        // test hook: the epoch to count on from (near kEpochWrap, so a short
        // run crosses the wrap; include/mbots.h "Environment")
        if (const char *e = std::getenv("MBOTS_EPOCH_START"))
            h->epoch = std::min<uint32_t>((uint32_t)std::strtoul(e, nullptr, 0), kEpochWrap);
    }
    {
        // (the default above 8192 worlds since round 6: with the prev-sensor
        // move lazy the caller's chain is the shorter one from the first steps
        // on, and the swap takes both hops off the sensor's chain: -1.9 % in
        // the driver's window, -2.1 % at steady state, interleaved on one box;
        // MBOTS_SWAP=0 restores the forked schedule)
        const char *e = std::getenv("MBOTS_SWAP");
        const bool want = e && *e ? e[0] == '1' : MB_SWAP_DEFAULT != 0;
        h->swap = want && S.W > MB_VALUE_FORK_MAX && !h->k1_finder && !h->sig_fork && !h->sig_join;
    }
    if (h->swap) check(hipEventCreateWithFlags(&h->ev_caller, kSyncEvent), "hipEventCreateWithFlags");
    check(hipEventCreateWithFlags(&h->ev_join[0], kSyncEvent), "hipEventCreateWithFlags");
    check(hipEventCreateWithFlags(&h->ev_join[1], kSyncEvent), "hipEventCreateWithFlags");
    {
        // the sensor is the step's longer chain once the deferred Prev moves
        // left the caller's stream lighter: its stream gets the higher priority
        // (step -1.9 %, same box; DESIGN.md "Schedule")
        int least = 0, greatest = 0;
        check(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
        // (K1-finder mode: the caller's chain is the longer one, the sensor's the
        // filler)
        const int prio = h->k1_finder && MB_FINDER_AUX_LOW ? least : greatest;
        check(hipStreamCreateWithPriority(&h->aux, hipStreamNonBlocking, prio),
              "hipStreamCreateWithPriority");
    }
    hipStream_t st = nullptr;
    check(hipMemsetAsync(h->arena.base, 0, bytes, st), "hipMemsetAsync");
    // Sim::Sim / initWorld (sim.cpp:1232-1256) + initial export of the rows
    check(mbots::upload_ray_table(S, st), "upload_ray_table");
    check(mbots::launch_init(S, st), "init_kernel");
    check(mbots::launch_tile_sum(S, 0, st), "tile_sum_kernel");
    check(mbots::launch_scan(S, 0, st), "scan_kernel");
    check(mbots::launch_export_rows(S, h->T[0], 1, st), "export_rows_kernel(init)");
    check(mbots::launch_move(S, h->T[1], h->T[0], 0, mbots::kMoveAll, st), "move_kernel(init)");
    if (rc == MBOTS_OK) rc = record_totals(h, st);
    check(hipStreamSynchronize(st), "hipStreamSynchronize");
    if (rc != MBOTS_OK) {
        mbots_destroy(h);
        return rc;
    }
    // the init scan counted the initial population as agent-steps; reset
    unsigned long long zero = 0;
    check(hipMemcpy(S.agent_steps, &zero, sizeof(zero), hipMemcpyHostToDevice), "hipMemcpy");
    h->tb = 0;
    h->parity = 1;   // the init scan consumed buffer 0 and cleared buffer 1
    *out = h;
    return rc;
}

int mbots_destroy(mbots_handle *h)
{
    if (!h) return MBOTS_OK;
    if (h->cpu) {
        delete h;
        return MBOTS_OK;
    }
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();
    for (auto &p : h->pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (auto e : h->pool) (void)hipEventDestroy(e);
    if (h->ev_totals) (void)hipEventDestroy(h->ev_totals);
    if (h->ev_hop) (void)hipEventDestroy(h->ev_hop);
    if (h->ev_caller) (void)hipEventDestroy(h->ev_caller);
    if (h->sig_fork) (void)hipFree(h->sig_fork);
    if (h->sig_join) (void)hipFree(h->sig_join);
    for (auto e : h->ev_join) if (e) (void)hipEventDestroy(e);
    if (h->aux) (void)hipStreamDestroy(h->aux);
    if (h->h_totals) (void)hipHostFree(h->h_totals);
    if (h->arena.base) (void)hipFree(h->arena.base);
    delete h;
    return MBOTS_OK;
}

// MBOTS_W_CAPACITY / MBOTS_E_CAPACITY once per rise of the dropped-agent total
static int capacity_report(mbots_handle *h, uint32_t dropped)
{
    if (dropped <= h->ovf_reported) return MBOTS_OK;
    const uint32_t was = h->ovf_reported;
    h->ovf_reported = dropped;
    g_err = std::to_string(dropped - was) + " births / respawns dropped at agent_capacity " +
            std::to_string(h->cfg.agent_capacity) + " (" + std::to_string(dropped) +
            " in total): the reference's worlds have no cap (sim.cpp:561-564, :830-834), so the run now "
            "differs from the reference's" +
            (h->cfg.agent_capacity < MBOTS_MAX_CAPACITY
                 ? "; raise agent_capacity (at most " + std::to_string(MBOTS_MAX_CAPACITY) + ")"
                 : " (" + std::to_string(MBOTS_MAX_CAPACITY) + " is the largest agent_capacity)");
    return (h->cfg.flags & MBOTS_FLAG_STRICT_CAPACITY) ? MBOTS_E_CAPACITY : MBOTS_W_CAPACITY;
}

int mbots_step(mbots_handle *h, void *stream)
{
    if (!h) return fail(MBOTS_E_INVALID, "null handle");
    if (h->cpu) {
        h->cpu->step();
        ++h->steps;
        return capacity_report(h, (uint32_t)std::min<uint64_t>(h->cpu->overflow(), 0xFFFFFFFFu));
    }
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = as_stream(stream);
    int rc;
    hipStreamCaptureStatus cap_status = hipStreamCaptureStatusNone;
    unsigned long long cap_id = 0;
    HIP_TRY(hipStreamGetCaptureInfo(st, &cap_status, &cap_id));
    const bool capturing = cap_status == hipStreamCaptureStatusActive;
    if (capturing && cap_id != h->cap_seen) {
        // a new capture: the previous one must have held an even number of steps
        if ((rc = capture_guard(h, nullptr))) return rc;
        h->cap_seen = cap_id;
        h->cap_stream = st;
        h->cap_steps = 0;
    }
    if ((rc = use_stream(h, st))) return rc;
    if (capturing) ++h->cap_steps;
    const mbots::ObsTable &nxt = h->T[h->tb ^ 1];
    const int par = h->parity;
    const int lazy = h->prev_lazy[h->tb] ? 1 : 0;
    // the parts the caller's reads forced last step (a learner that reads the
    // observation and PrevHiddenState between step and shift, as
    // training_loop.py:47-88 does): moved right after this step's K3a, beside
    // the sensor, instead of behind the wait for it (DESIGN.md "Prefetch")
    int prefetch = h->forced;
    h->forced = 0;
    h->prefetched = prefetch;
    // no shift since the last step: its deferred Prev moves first
    if (h->six_pending[h->tb] && (rc = materialize_prev(h, st))) return rc;
    if ((rc = materialize_prev_ah(h, st))) return rc;
    if ((rc = materialize_cur_ah(h, st, 0))) return rc;
    // (a prev sensor still owed is dead from here on: the new table's prev
    // sensor is the last table's sensor rows, updateSensorOutputIdx
    // sim.cpp:736-789, not its prev sensor -- so it is never moved)
    // K1 reads the learner's actions through the half's view (an aliased
    // Action column is its PrevAction), and so do this step's moves
    const mbots::ObsTable cur = src_view(h, h->tb);
    // K1 reads the finder slots the previous step's sensor wrote, and writes the
    // state half that sensor read; the halves swap after K1.
    // (under stream capture only a join recorded in the same capture is waited
    // for: a replay starts after the previous launch of the graph completed)
    // (small world counts, eagerly, while the device still runs the previous
    // step: the flag a wave after the sensor raised.  A host that arrives after
    // the sensor has finished -- a host-bound loop, where the value waits'
    // extra enqueues would only add host time -- takes the event wait, and this
    // step raises no flags.)
    bool ahead = false;
    if (!capturing && (h->sig_fork || h->sig_join) && MB_VALUE_ADAPT) {
        ahead = h->last_join < 0 || hipEventQuery(h->ev_join[h->last_join]) == hipErrorNotReady;
        (void)hipGetLastError();   // (hipEventQuery reports "not ready" as an error)
    } else if (!capturing && (h->sig_fork || h->sig_join)) {
        ahead = true;
    }
    const int before = h->last_join;                  // the last step's sensor (its rows are
    const unsigned long long before_cap = h->join_capture;   // the current half's)
    // MBOTS_SWAP=1: K1, K2 and the sensor on the internal stream with no hop
    // between them; K1 after the last sensor (the same stream) and after what
    // the caller enqueued so far (the learner's writes)
    const bool swap = h->swap && !capturing;
    const hipStream_t kst = swap ? h->aux : st;
    if (swap) {
        HIP_TRY(hipEventRecord(h->ev_caller, st));
        HIP_TRY(hipStreamWaitEvent(h->aux, h->ev_caller, 0));
    } else if (h->k1_finder) {
        // K1 computed the finder slots this K1 reads; it must only not overwrite
        // the state half the sensor before the last one may still read
        if ((rc = wait_prev_sensor(h, st))) return rc;
    } else if (!capturing && h->join_epoch != 0 && ahead) {
        // ">=" (VERDICT r5 item 5): the flag only grows -- one writer, raised in
        // step order on the sensor's queue -- so this wait passes whenever it is
        // reached, even after a later step has raised the flag again; an
        // equality wait would hang there (the round-5 probe's fork did)
        HIP_TRY(hipStreamWaitValue32(st, h->sig_join, h->join_epoch, hipStreamWaitValueGte, 0xFFFFFFFFu));
    } else if (h->last_join >= 0 && (!capturing || h->join_capture == cap_id)) {
        HIP_TRY(hipStreamWaitEvent(st, h->ev_join[h->last_join], 0));
        if (!capturing) h->waited_serial = std::max(h->waited_serial, h->join_serial[h->last_join]);
    }
    h->S.finder_from_state = h->sensed ? 0u : 1u;
    // K1 writes this step's old rows into the half the step before last used:
    // the sensor that read it (K1-finder mode: the sensor before the last one)
    // has been waited for above
    h->S.obsrow_out = h->obsrow_out2[par];
    if ((rc = timed(h, MBOTS_TK_WORLD_STEP, kst,
                    [&] { return mbots::launch_world_step(h->S, cur, par, kst); })))
        return rc;
    mbots::swap_state(h->S);
    // K2 writes the row counts into the pinned mirror; accessors and the
    // sensor's stream wait on ev_totals, carried by K2's own dispatch
    // (under stream capture -- a caller recording steps into a HIP graph -- the
    // fork / join events are recorded by hipEventRecord, the capturable form)
    // the fork by value (small world counts, eagerly): K2's last block raises
    // this step's epoch (under capture replays would repeat it: the event then)
    uint32_t epoch = 0;
    if ((h->sig_fork || h->sig_join) && !capturing && ahead) {
        if (h->epoch >= kEpochWrap) {
            // both waits are "flag >= epoch": before the counter wraps, drain
            // the device and restart both from 0 -- the resets complete before
            // any later wait is enqueued (exercised by
            // tests/test_robustness.py::test_value_wait_epoch_wrap through
            // MBOTS_EPOCH_START)
            HIP_TRY(hipDeviceSynchronize());
            if (h->sig_fork) HIP_TRY(hipMemset(h->sig_fork, 0, 8));
            if (h->sig_join) HIP_TRY(hipMemset(h->sig_join, 0, 8));
            HIP_TRY(hipDeviceSynchronize());
            h->epoch = 0;
            h->join_epoch = 0;
            ++h->epoch_wraps;
        }
        epoch = ++h->epoch;
    }
    h->S.epoch = h->sig_fork ? epoch : 0u;
    // this step's row bases and sensor order go to the buffer the step before
    // last used (its sensor has been waited for: above, or by the event join)
    h->S.row_base = h->row_base2[par];
    h->S.sorder = h->sorder2[par];
    // this step's row counts are K2's: no host read of them before it (ADVICE r4:
    // cleared here, after every materialisation above that may sync the last ones)
    h->totals_ok = false;
    rc = timed(h, MBOTS_TK_SCAN, kst, [&] { return mbots::launch_scan(h->S, par, kst, h->ev_totals, capturing); });
    h->maxpop_stale = false;
    h->S.epoch = 0;
    if (rc) return rc;
    // fork after K2: the K3b sensor (VALU-bound; it derives the export rows from
    // K2's row_base itself) runs on the aux stream while this stream goes on
    // with K3a export, shift_observations and the learner's action writes --
    // none of which reads the sensor rows or the finder slots.  The next step's
    // K1 and the semantic/depth accessors wait for ev_join.
    const int jcur = h->last_join == 0 ? 1 : 0;
    // (">=": the fork flag only grows -- K2's last block raises each step's
    // epoch in step order -- so the wait passes whenever the sensor's queue
    // reaches it, also after a later K2 raised the flag again; equality would
    // hang there)
    if (swap) HIP_TRY(hipStreamWaitEvent(st, h->ev_totals, 0));   // K3a after K2 (the caller's join)
    else if (epoch && h->sig_fork) HIP_TRY(hipStreamWaitValue32(h->aux, h->sig_fork, epoch, hipStreamWaitValueGte, 0xFFFFFFFFu));
    else HIP_TRY(hipStreamWaitEvent(h->aux, h->ev_totals, 0));
    // (K1-finder mode: the sensor also moves the last table's sensor rows into
    // its rows' prev-sensor columns, so no caller-stream wait is needed for them)
    const bool psem_by_sensor = h->k1_finder && MB_FINDER_PSEM_BY_SENSOR;
    if (psem_by_sensor) {
        h->S.psem_src = h->T[h->tb].sem;
        h->S.pdepth_src = (h->cfg.flags & MBOTS_FLAG_FIX_DEPTH_ALIAS) ? h->T[h->tb].depth : nullptr;
    }
    h->S.list_par = (uint32_t)par;   // (mixed classes: this step's K2 lists)
    rc = timed(h, MBOTS_TK_SENSOR, h->aux, [&] {
        return mbots::launch_sensor(h->S, nxt, h->aux, h->ev_join[jcur], capturing);
    });
    h->S.psem_src = nullptr;
    h->S.pdepth_src = nullptr;
    if (rc) return rc;
    h->sensed = true;
    h->join_serial[jcur] = ++h->sensor_serial;
    h->prev_join = before;
    h->prev_capture = before_cap;
    h->last_join = jcur;
    h->join_capture = capturing ? cap_id : 0;
    h->join_epoch = 0;
    if (epoch && h->sig_join) {
        HIP_TRY(mbots::launch_raise_flag(h->sig_join, epoch, h->aux));
        h->join_epoch = epoch;
    }
    if ((rc = timed(h, MBOTS_TK_EXPORT, st,
                    [&] { return mbots::launch_export_rows(h->S, nxt, 0, st); })))
        return rc;
    // (the prev sensor is the sensor's own part in K1-finder mode; moved here
    // instead, its source rows are the last sensor's, which this step's K1 did
    // not wait for in that mode)
    if (psem_by_sensor) prefetch &= ~mbots::kMoveSensor;
    if ((prefetch & mbots::kMoveSensor) && (rc = wait_prev_sensor(h, st))) return rc;
    if (prefetch && (rc = timed(h, MBOTS_TK_MOVE, st, [&] {
                         return mbots::launch_move(h->S, cur, nxt, lazy, prefetch, st);
                     })))
        return rc;
    ++h->steps;
    h->parity ^= 1;
    h->tb ^= 1;
    const int nt = h->tb;
    // the new half's Prev* columns: eight moves deferred (a shift overwrites them)
    h->prev_lazy[nt] = false;
    h->a_alias[nt] = h->h_alias[nt] = false;
    h->cur_ah_pending[nt] = true;
    h->psem_pending[nt] = !psem_by_sensor;
    h->ah_pending[nt] = true;
    h->six_pending[nt] = true;
    h->six_lazy[nt] = lazy != 0;
    if (prefetch & mbots::kMoveAH) h->cur_ah_pending[nt] = false;
    if (prefetch & mbots::kMoveSensor) h->psem_pending[nt] = false;
    if (prefetch & mbots::kMovePrevAH) h->ah_pending[nt] = false;
    if (prefetch & mbots::kMovePrev6) h->six_pending[nt] = false;
    // capacity drops the device has published so far (K2's pinned mirror of a
    // recent step: no synchronisation)
    return capacity_report(h, __atomic_load_n(&h->h_totals[mbots::kTotOverflow], __ATOMIC_RELAXED));
}

int mbots_shift_observations(mbots_handle *h, void *stream)
{
    if (!h) return fail(MBOTS_E_INVALID, "null handle");
    if (h->cpu) {
        h->cpu->shift_observations();
        return MBOTS_OK;
    }
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = as_stream(stream);
    int rc = use_stream(h, st);
    if (rc) return rc;
    // Action / HiddenState now; the other six Prev* columns stay views of the
    // current ones until the next step or an accessor needs them (K5, lazy
    // shift).  Action / HiddenState still in the other half: one gather writes their
    // Prev copies, and the current columns become views of those (the learner
    // overwrites them next; DESIGN.md "Aliased current Action / HiddenState")
    // -- the fused shift.  The step's prev-sensor move is not the shift's
    // (shiftObservationsSystem, sim.cpp:1001-1035, leaves the sensor alone):
    // it stays owed until a reader needs it and dies at the next step
    // (DESIGN.md "Lazy prev sensor").
    const int tb = h->tb;
    const bool fused = h->cur_ah_pending[tb];
    if (fused) {
        const mbots::ObsTable src = src_view(h, tb ^ 1);
        rc = timed(h, MBOTS_TK_SHIFT, st, [&] {
            return mbots::launch_move(h->S, src, h->T[tb], 0, mbots::kMoveAHShift, st);
        });
    } else if (!(h->a_alias[tb] && h->h_alias[tb])) {   // both aliased: already equal
        if ((rc = materialize_cur_ah(h, st, 3))) return rc;
        rc = timed(h, MBOTS_TK_SHIFT, st,
                   [&] { return mbots::launch_shift(h->S, h->T[tb], mbots::kShiftEager, st); });
    }
    if (rc == MBOTS_OK) {
        // Action / HiddenState and every Prev* column but the sensor's are the
        // shift's now: a later read of them is not the step's deferred move
        h->prefetched &= mbots::kMoveSensor;
        if (fused) h->a_alias[tb] = h->h_alias[tb] = true;
        h->cur_ah_pending[tb] = false;
        h->prev_lazy[tb] = true;
        h->ah_pending[tb] = false;   // the shift wrote PrevAction / PrevHiddenState
        h->six_pending[tb] = false;  // ... and made the six the current columns
    }
    return rc;
}

int mbots_num_agents(mbots_handle *h, uint32_t *out)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (h->cpu) {
        *out = h->cpu->num_agents();
        return MBOTS_OK;
    }
    int rc = sync_totals(h);
    if (rc) return rc;
    *out = h->h_totals[0];
    return MBOTS_OK;
}

int mbots_export_on(mbots_handle *h, int32_t id, void *stream, mbots_tensor *out)
{
    using namespace mbots;
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (h->cpu) {
        const int r = h->cpu->export_tensor(id, out);
        return r ? fail(r, "unknown export id " + std::to_string(id)) : MBOTS_OK;
    }
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = as_stream(stream);
    uint32_t N = 0;
    int rc = mbots_num_agents(h, &N);
    if (rc) return rc;
    // the view's deferred copies and joins go on the reader's stream, after
    // everything the manager enqueued (the step may have run on another)
    if ((rc = use_stream(h, st))) return rc;
    const int owed = pending_mask(h);
    int need = 0;
    switch (id) {
    case MBOTS_EXPORT_PREV_SPECIES: case MBOTS_EXPORT_PREV_POSITION: case MBOTS_EXPORT_PREV_HEALTH:
    case MBOTS_EXPORT_PREV_SURROUNDING: case MBOTS_EXPORT_PREV_REWARD: case MBOTS_EXPORT_PREV_STATS:
        need = mbots::kMovePrev6;
        if ((rc = materialize_prev(h, st))) return rc;
        break;
    case MBOTS_EXPORT_PREV_ACTION: case MBOTS_EXPORT_PREV_HIDDEN_STATE:
        need = mbots::kMovePrevAH;
        if ((rc = materialize_prev_ah(h, st))) return rc;
        break;
    case MBOTS_EXPORT_ACTION: case MBOTS_EXPORT_HIDDEN_STATE:
        need = mbots::kMoveAH;
        if ((rc = materialize_cur_ah(h, st, id == MBOTS_EXPORT_ACTION ? 1 : 2))) return rc;
        break;
    case MBOTS_EXPORT_PREV_SENSOR_SEMANTIC: case MBOTS_EXPORT_PREV_SENSOR_DEPTH:
        need = mbots::kMoveSensor;
        if ((rc = materialize_psem(h, st))) return rc;
        if (h->k1_finder && (rc = wait_sensor(h, st))) return rc;   // the sensor moved them
        break;
    default: break;
    }
    note_use(h, need, owed);
    const ObsTable &t = h->T[h->tb];
    const bool fixd = (h->cfg.flags & MBOTS_FLAG_FIX_DEPTH_ALIAS) != 0;
    void *p = nullptr;
    int dt = MBOTS_DTYPE_INT32;
    int64_t rows = N, cols = 1;
    switch (id) {
    case MBOTS_EXPORT_RESET: p = h->reset_zeros; rows = h->cfg.num_worlds; break;
    case MBOTS_EXPORT_ACTION: p = t.action; cols = 6; break;
    case MBOTS_EXPORT_PREV_ACTION: p = t.paction; cols = 6; break;
    case MBOTS_EXPORT_HIDDEN_STATE: p = t.hidden; dt = MBOTS_DTYPE_FLOAT32; cols = kHidden; break;
    case MBOTS_EXPORT_PREV_HIDDEN_STATE: p = t.phidden; dt = MBOTS_DTYPE_FLOAT32; cols = kHidden; break;
    case MBOTS_EXPORT_REWARD: p = t.reward; dt = MBOTS_DTYPE_FLOAT32; break;
    case MBOTS_EXPORT_PREV_REWARD: p = t.preward; dt = MBOTS_DTYPE_FLOAT32; break;
    case MBOTS_EXPORT_DONE: p = h->done_zeros; break;
    case MBOTS_EXPORT_POSITION: p = t.pos; dt = MBOTS_DTYPE_FLOAT32; cols = 2; break;
    case MBOTS_EXPORT_PREV_POSITION: p = t.ppos; dt = MBOTS_DTYPE_FLOAT32; cols = 2; break;
    // int32 health bits exported as a float32 view (types.hpp:119-124, mgr.cpp:329-346; B.2)
    case MBOTS_EXPORT_HEALTH: p = t.health; dt = MBOTS_DTYPE_FLOAT32; break;
    case MBOTS_EXPORT_PREV_HEALTH: p = t.phealth; dt = MBOTS_DTYPE_FLOAT32; break;
    case MBOTS_EXPORT_SURROUNDING: p = t.sur; dt = MBOTS_DTYPE_FLOAT32; cols = 2; break;
    case MBOTS_EXPORT_PREV_SURROUNDING: p = t.psur; dt = MBOTS_DTYPE_FLOAT32; cols = 2; break;
    case MBOTS_EXPORT_SENSOR_SEMANTIC:
        if ((rc = wait_sensor(h, st))) return rc;
        p = t.sem; dt = MBOTS_DTYPE_INT8; cols = kSensor; break;
    // SensorDepth exports the semantic buffer (sim.cpp:102-104, B.1) unless fixed
    case MBOTS_EXPORT_SENSOR_DEPTH:
        if ((rc = wait_sensor(h, st))) return rc;
        p = fixd ? (void *)t.depth : (void *)t.sem; dt = MBOTS_DTYPE_UINT8; cols = kSensor; break;
    case MBOTS_EXPORT_PREV_SENSOR_SEMANTIC: p = t.psem; dt = MBOTS_DTYPE_INT8; cols = kSensor; break;
    case MBOTS_EXPORT_PREV_SENSOR_DEPTH:
        p = fixd ? (void *)t.pdepth : (void *)t.psem; dt = MBOTS_DTYPE_UINT8; cols = kSensor; break;
    case MBOTS_EXPORT_STATS: p = t.stats; cols = 4; break;
    case MBOTS_EXPORT_PREV_STATS: p = t.pstats; cols = 4; break;
    case MBOTS_EXPORT_SENSOR_INDEX: {
        HIP_TRY(mbots::launch_sensor_index(h->S, h->sensor_index, st));
        HIP_TRY(hipStreamSynchronize(st));
        p = h->sensor_index;
        break;
    }
    case MBOTS_EXPORT_SPECIES_COUNT: p = h->S.scount; rows = h->cfg.num_worlds; cols = kNumSpecies; break;
    case MBOTS_EXPORT_SPECIES: p = t.species; break;
    case MBOTS_EXPORT_PREV_SPECIES: p = t.pspecies; break;
    default: return fail(MBOTS_E_INVALID, "unknown export id " + std::to_string(id));
    }
    out->data = p;
    out->dtype = dt;
    out->device = h->device;
    out->dims[0] = rows;
    out->dims[1] = cols;
    return MBOTS_OK;
}

int mbots_export(mbots_handle *h, int32_t id, mbots_tensor *out)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (h->cpu) return mbots_export_on(h, id, nullptr, out);
    // the reference's views are valid on any stream once the synchronous
    // step() returned (mgr.cpp:51-63): so are these, once this returns
    const int rc = mbots_export_on(h, id, h->last_stream, out);
    if (rc) return rc;
    if (!capturing(h->last_stream)) HIP_TRY(hipStreamSynchronize(h->last_stream));
    return MBOTS_OK;
}

int mbots_set_action(mbots_handle *h, uint32_t row, const int32_t action[6])
{
    if (!h || !action) return fail(MBOTS_E_INVALID, "null argument");
    uint32_t N = 0;
    int rc = mbots_num_agents(h, &N);
    if (rc) return rc;
    if (row >= N) return fail(MBOTS_E_RANGE, "agent row out of range");
    if (h->cpu) {
        memcpy(&h->cpu->table().action[(size_t)row * 6], action, 6 * sizeof(int32_t));
        return MBOTS_OK;
    }
    HIP_TRY(hipSetDevice(h->device));
    const int owed = pending_mask(h);
    hipStream_t st = h->last_stream;
    if ((rc = materialize_cur_ah(h, st, 1))) return rc;
    note_use(h, mbots::kMoveAH, owed);
    HIP_TRY(hipMemcpyAsync(h->T[h->tb].action + (size_t)row * 6, action, 6 * sizeof(int32_t),
                           hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    return MBOTS_OK;
}

int mbots_agent_offset_for_world(mbots_handle *h, uint32_t world, uint32_t *out)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (world >= h->cfg.num_worlds) return fail(MBOTS_E_RANGE, "world out of range");
    if (h->cpu) {
        *out = h->cpu->world_offset_of(world);
        return MBOTS_OK;
    }
    int rc = sync_totals(h);
    if (rc) return rc;
    int32_t v = 0;
    HIP_TRY(hipMemcpy(&v, h->S.world_off + world, sizeof(v), hipMemcpyDeviceToHost));
    *out = (uint32_t)v;
    return MBOTS_OK;
}

int mbots_write_synthetic_actions(mbots_handle *h, uint32_t seed, uint32_t step,
                                  int32_t write_hidden, void *stream)
{
    if (!h) return fail(MBOTS_E_INVALID, "null handle");
    if (h->cpu) {
        h->cpu->write_synthetic_actions(seed, step, write_hidden != 0);
        return MBOTS_OK;
    }
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = as_stream(stream);
    int rc = use_stream(h, st);
    if (rc) return rc;
    const int owed = pending_mask(h);
    // the writer rewrites every live row's Action (and HiddenState with
    // write_hidden): an aliased column of those is simply written, not copied
    if ((rc = materialize_cur_ah(h, st, 0))) return rc;
    note_use(h, mbots::kMoveAH, owed);
    rc = timed(h, MBOTS_TK_ACTIONS, st, [&] {
        return mbots::launch_synthetic_actions(h->S, h->T[h->tb], seed, step, write_hidden, st);
    });
    if (rc) return rc;
    h->a_alias[h->tb] = false;
    if (write_hidden) h->h_alias[h->tb] = false;
    return MBOTS_OK;
}

int mbots_construct_obs(mbots_handle *h, int32_t prev, float *out, uint64_t out_rows, void *stream)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (out_rows > 0xFFFFFFFFull) return fail(MBOTS_E_INVALID, "out_rows too large");
    if (h->cpu) {
        h->cpu->construct_obs(prev != 0, out, out_rows);
        return MBOTS_OK;
    }
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = as_stream(stream);
    int rc = use_stream(h, st);
    if (rc) return rc;
    const int owed = pending_mask(h);
    // current semantic rows come from K3b (and in K1-finder mode the prev ones too)
    if ((!prev || h->k1_finder) && (rc = wait_sensor(h, st))) return rc;
    // The previous rows' health / position / surrounding: while the step's
    // deferred move of the six Prev* columns is still owed, gathered from the
    // other half along src_of inside this launch (what the move would write,
    // nothing materialised: the shift that follows in training_loop.py:135
    // makes the six the current columns, so the move is never run); the prev
    // sensor is moved (and remembered for the next step's prefetch)
    const bool gather6 = prev && h->six_pending[h->tb];
    if (prev && (rc = materialize_psem(h, st))) return rc;
    if (prev) note_use(h, mbots::kMoveSensor, owed);
    return timed(h, MBOTS_TK_OBS, st, [&] {
        return mbots::launch_construct_obs(h->S, h->T[h->tb], prev, h->prev_lazy[h->tb] ? 1 : 0, out,
                                           (uint32_t)out_rows, st, gather6 ? &h->T[h->tb ^ 1] : nullptr,
                                           h->six_lazy[h->tb] ? 1 : 0);
    });
}

int mbots_rollout_record_bytes(mbots_handle *h, uint32_t *out)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    *out = (h->cfg.flags & MBOTS_FLAG_FIX_DEPTH_ALIAS) ? MBOTS_ROLLOUT_BYTES_DEPTH : MBOTS_ROLLOUT_BYTES;
    return MBOTS_OK;
}

int mbots_pack_rollout(mbots_handle *h, void *out, uint64_t out_rows, void *stream)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (out_rows > 0xFFFFFFFFull) return fail(MBOTS_E_INVALID, "out_rows too large");
    const bool fixd = (h->cfg.flags & MBOTS_FLAG_FIX_DEPTH_ALIAS) != 0;
    if (h->cpu) {
        const mbots::cpu::Table &t = h->cpu->table();
        const uint64_t n = std::min<uint64_t>(h->cpu->num_agents(), out_rows);
        pack_rollout_host(t.sem.data(), fixd ? t.depth.data() : nullptr, t.health.data(), t.pos.data(),
                          t.sur.data(), t.reward.data(), t.stats.data(), n, static_cast<uint8_t *>(out));
        return MBOTS_OK;
    }
    if ((reinterpret_cast<uintptr_t>(out) & 15u) != 0) return fail(MBOTS_E_INVALID, "out must be 16-byte aligned");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = as_stream(stream);
    int rc = use_stream(h, st);
    if (rc) return rc;
    if ((rc = wait_sensor(h, st))) return rc;   // the semantic / depth rows come from K3b
    return timed(h, MBOTS_TK_OBS, st, [&] {
        return mbots::launch_pack_rollout(h->S, h->T[h->tb], out, (uint32_t)out_rows, st);
    });
}

int mbots_learner_record_bytes(mbots_handle *h, uint32_t *out)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    *out = (h->cfg.flags & MBOTS_FLAG_FIX_DEPTH_ALIAS) ? MBOTS_LEARNER_BYTES_DEPTH : MBOTS_LEARNER_BYTES;
    return MBOTS_OK;
}

int mbots_pack_learner(mbots_handle *h, void *out, uint64_t out_rows, void *stream)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (out_rows > 0xFFFFFFFFull) return fail(MBOTS_E_INVALID, "out_rows too large");
    const bool fixd = (h->cfg.flags & MBOTS_FLAG_FIX_DEPTH_ALIAS) != 0;
    if (h->cpu) {
        pack_learner_host(h->cpu->table(), fixd, std::min<uint64_t>(h->cpu->num_agents(), out_rows),
                          static_cast<uint8_t *>(out));
        return MBOTS_OK;
    }
    if ((reinterpret_cast<uintptr_t>(out) & 15u) != 0) return fail(MBOTS_E_INVALID, "out must be 16-byte aligned");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = as_stream(stream);
    int rc = use_stream(h, st);
    if (rc) return rc;
    // every column the record carries in its storage: the step's deferred
    // moves the learner's reads need (and remembered, like the accessors', so
    // the next step prefetches them beside its sensor)
    const int owed = pending_mask(h);
    if ((rc = materialize_prev(h, st))) return rc;
    if ((rc = materialize_prev_ah(h, st))) return rc;
    if ((rc = materialize_cur_ah(h, st, 3))) return rc;
    if ((rc = materialize_psem(h, st))) return rc;
    note_use(h, mbots::kMovePrev6 | mbots::kMovePrevAH | mbots::kMoveAH | mbots::kMoveSensor, owed);
    if ((rc = wait_sensor(h, st))) return rc;   // the sensor rows (and what it moved)
    return timed(h, MBOTS_TK_OBS, st, [&] {
        return mbots::launch_pack_learner(h->S, h->T[h->tb], h->prev_lazy[h->tb] ? 1 : 0, out, (uint32_t)out_rows,
                                          st);
    });
}

int mbots_pack_learner_slim(mbots_handle *h, void *out, uint64_t out_rows, void *stream)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (out_rows > 0xFFFFFFFFull) return fail(MBOTS_E_INVALID, "out_rows too large");
    const bool fixd = (h->cfg.flags & MBOTS_FLAG_FIX_DEPTH_ALIAS) != 0;
    if (h->cpu) {
        pack_learner_slim_host(h->cpu->table(), h->cpu->src_of(), fixd,
                               std::min<uint64_t>(h->cpu->num_agents(), out_rows), static_cast<uint8_t *>(out));
        return MBOTS_OK;
    }
    if ((reinterpret_cast<uintptr_t>(out) & 15u) != 0) return fail(MBOTS_E_INVALID, "out must be 16-byte aligned");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = as_stream(stream);
    int rc = use_stream(h, st);
    if (rc) return rc;
    // the sensor rows (and in K1-finder mode the prev sensor rows it moved);
    // in the joined schedule the last sensor's rows, the source of a prev
    // sensor still owed, were waited for by this step's K1
    if ((rc = wait_sensor(h, st))) return rc;
    const int tb = h->tb;
    const mbots::ObsTable &last = h->T[tb ^ 1];
    return timed(h, MBOTS_TK_OBS, st, [&] {
        return mbots::launch_pack_learner_slim(h->S, h->T[tb], h->prev_lazy[tb] ? 1 : 0,
                                               h->six_pending[tb] ? &last : nullptr, h->six_lazy[tb] ? 1 : 0,
                                               h->psem_pending[tb] ? &last : nullptr, out, (uint32_t)out_rows, st);
    });
}

int mbots_unpack_learner_slim(const void *records, uint64_t rows, int32_t with_depth, int32_t device,
                              const mbots_learner_out *out, int32_t *src, void *stream)
{
    if (!out || (!records && rows)) return fail(MBOTS_E_INVALID, "null argument");
    if (out->action || out->hidden || out->prev_hidden)
        return fail(MBOTS_E_INVALID, "slim records carry no Action / HiddenState / PrevHiddenState");
    if (rows > 0xFFFFFFFFull) return fail(MBOTS_E_INVALID, "rows too large");
    if (device < 0) {
        unpack_learner_host(static_cast<const uint8_t *>(records), rows, with_depth != 0, *out, true, src);
        return MBOTS_OK;
    }
    if ((reinterpret_cast<uintptr_t>(records) & 15u) != 0)
        return fail(MBOTS_E_INVALID, "records must be 16-byte aligned");
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(mbots::launch_unpack_learner_slim(records, (uint32_t)rows, with_depth ? 1 : 0, *out, src,
                                              as_stream(stream)));
    return MBOTS_OK;
}

int mbots_rebuild_learner(const int32_t *src, uint64_t rows, const int64_t *cur_counts, const int64_t *last_counts,
                          uint32_t ranks, const int32_t *last_action, const float *last_memory,
                          const float *last_hidden, uint64_t last_rows, int32_t *action, float *hidden,
                          float *prev_hidden, int32_t device, void *stream)
{
    if (!cur_counts || !last_counts || (rows && (!src || !action || !hidden || !prev_hidden)) ||
        (last_rows && (!last_action || !last_memory || !last_hidden)))
        return fail(MBOTS_E_INVALID, "null argument");
    if (ranks == 0 || ranks > MBOTS_MAX_LEARNER_RANKS)
        return fail(MBOTS_E_INVALID, "ranks must be in [1, " + std::to_string(MBOTS_MAX_LEARNER_RANKS) + "]");
    uint64_t cur = 0, last = 0;
    for (uint32_t i = 0; i < 4 * ranks; ++i) {
        if (cur_counts[i] < 0 || last_counts[i] < 0) return fail(MBOTS_E_INVALID, "negative row count");
        cur += (uint64_t)cur_counts[i];
        last += (uint64_t)last_counts[i];
    }
    if (cur != rows) return fail(MBOTS_E_INVALID, "cur_counts do not sum to rows");
    if (last != last_rows) return fail(MBOTS_E_INVALID, "last_counts do not sum to last_rows");
    if (rows > 0x7FFFFFFFull || last_rows > 0x7FFFFFFFull) return fail(MBOTS_E_INVALID, "rows too large");
    const mbots::RebuildPlan p = mbots::rebuild_plan(cur_counts, last_counts, ranks);
    if (device < 0) {
        // (a provenance outside the owning rank's last rows is refused, not read)
        for (uint64_t r = 0; r < rows; ++r) {
            const int32_t g = mbots::rebuild_row(p, (int32_t)r, src[r]);
            if (g >= (int64_t)last_rows) return fail(MBOTS_E_RANGE, "provenance outside the last table");
            for (int k = 0; k < 6; ++k) action[r * 6 + k] = g >= 0 ? last_action[(size_t)g * 6 + k] : 0;
            for (int k = 0; k < mbots::kHidden; ++k) {
                hidden[r * mbots::kHidden + k] = g >= 0 ? last_memory[(size_t)g * mbots::kHidden + k] : 0.0f;
                prev_hidden[r * mbots::kHidden + k] = g >= 0 ? last_hidden[(size_t)g * mbots::kHidden + k] : 0.0f;
            }
        }
        return MBOTS_OK;
    }
    for (const void *q : {(const void *)src, (const void *)last_action, (const void *)last_memory,
                          (const void *)last_hidden, (const void *)action, (const void *)hidden,
                          (const void *)prev_hidden})
        if (reinterpret_cast<uintptr_t>(q) & 7u) return fail(MBOTS_E_INVALID, "arrays must be 8-byte aligned");
    for (const void *q : {(const void *)last_memory, (const void *)last_hidden, (const void *)hidden,
                          (const void *)prev_hidden})
        if (reinterpret_cast<uintptr_t>(q) & 15u) return fail(MBOTS_E_INVALID, "float arrays must be 16-byte aligned");
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(mbots::launch_rebuild_learner(p, src, (uint32_t)rows, (uint32_t)last_rows, last_action, last_memory,
                                          last_hidden, action, hidden, prev_hidden, as_stream(stream)));
    return MBOTS_OK;
}

int mbots_unpack_learner(const void *records, uint64_t rows, int32_t with_depth, int32_t device,
                         const mbots_learner_out *out, void *stream)
{
    if (!out || (!records && rows)) return fail(MBOTS_E_INVALID, "null argument");
    if (rows > 0xFFFFFFFFull) return fail(MBOTS_E_INVALID, "rows too large");
    if (device < 0) {
        unpack_learner_host(static_cast<const uint8_t *>(records), rows, with_depth != 0, *out);
        return MBOTS_OK;
    }
    if ((reinterpret_cast<uintptr_t>(records) & 15u) != 0)
        return fail(MBOTS_E_INVALID, "records must be 16-byte aligned");
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(mbots::launch_unpack_learner(records, (uint32_t)rows, with_depth ? 1 : 0, *out, as_stream(stream)));
    return MBOTS_OK;
}

int mbots_max_population(mbots_handle *h, uint32_t *out)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (h->cpu) {
        *out = h->cpu->max_population();
        return MBOTS_OK;
    }
    HIP_TRY(hipSetDevice(h->device));
    if (!h->S.track_maxpop) {   // the first call: K2 publishes the tile maxima from the next step on
        h->S.track_maxpop = 1u;
        h->maxpop_stale = true;
    }
    if (h->maxpop_stale) {   // (after a checkpoint load or before tracking, until the next step's K2)
        HIP_TRY(hipDeviceSynchronize());
        std::vector<int32_t> n(h->S.W);
        HIP_TRY(hipMemcpy(n.data(), h->S.n, n.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
        int32_t mx = 0;
        for (int32_t v : n) mx = std::max(mx, v);
        *out = (uint32_t)mx;
        return MBOTS_OK;
    }
    // the last step's K2 published each tile's largest world with the row
    // counts: waiting for it waits for K2 only, not for the step's sensor or
    // the caller's chain
    if (int rc = sync_totals(h)) return rc;
    uint32_t mx = 0;
    for (uint32_t t = 0; t < h->S.ntiles; ++t)
        mx = std::max(mx, __atomic_load_n(&h->h_totals[mbots::kTotMaxPop + t], __ATOMIC_RELAXED));
    *out = mx;
    return MBOTS_OK;
}

int mbots_num_rows(mbots_handle *h, uint32_t *out)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (h->cpu) {
        *out = h->cpu->num_rows();
        return MBOTS_OK;
    }
    int rc = sync_totals(h);
    if (rc) return rc;
    *out = h->h_totals[mbots::kTotRows];
    return MBOTS_OK;
}

int mbots_write_actions(mbots_handle *h, const int32_t *action, const float *hidden, uint64_t rows, void *stream)
{
    if (!h) return fail(MBOTS_E_INVALID, "null handle");
    uint32_t N = 0, R = 0;
    int rc = mbots_num_agents(h, &N);
    if (!rc) rc = mbots_num_rows(h, &R);
    if (rc) return rc;
    if (rows != N && rows != R) return fail(MBOTS_E_INVALID, "rows must be num_agents() or num_rows()");
    if (h->cpu) {
        mbots::cpu::Table &t = h->cpu->table();
        if (action && rows) memcpy(t.action.data(), action, rows * 6 * sizeof(int32_t));
        if (hidden && rows) memcpy(t.hidden.data(), hidden, rows * mbots::kHidden * sizeof(float));
        return MBOTS_OK;
    }
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = as_stream(stream);
    if ((rc = use_stream(h, st))) return rc;
    const int tb = h->tb;
    const int owed = pending_mask(h);
    // a column written only in part keeps its other rows: copied out of an
    // aliased Prev storage first; a column written whole is simply written
    const int part = (action && rows < R && h->a_alias[tb] ? 1 : 0) | (hidden && rows < R && h->h_alias[tb] ? 2 : 0);
    if ((rc = materialize_cur_ah(h, st, part))) return rc;
    note_use(h, mbots::kMoveAH, owed);
    const mbots::ObsTable &t = h->T[tb];
    if (action && rows) HIP_TRY(hipMemcpyAsync(t.action, action, rows * 6 * sizeof(int32_t), hipMemcpyDefault, st));
    if (hidden && rows)
        HIP_TRY(hipMemcpyAsync(t.hidden, hidden, rows * mbots::kHidden * sizeof(float), hipMemcpyDefault, st));
    if (action) h->a_alias[tb] = false;
    if (hidden) h->h_alias[tb] = false;
    return MBOTS_OK;
}

int mbots_unpack_rollout(const void *records, uint64_t rows, int32_t with_depth, int32_t device, float *obs,
                         float *reward, int32_t *stats, void *stream)
{
    if ((!records || !obs) && rows) return fail(MBOTS_E_INVALID, "null argument");
    if (rows > 0xFFFFFFFFull) return fail(MBOTS_E_INVALID, "rows too large");
    if (device < 0) {
        unpack_rollout_host(static_cast<const uint8_t *>(records), rows, with_depth != 0, obs, reward, stats);
        return MBOTS_OK;
    }
    if ((stats && (reinterpret_cast<uintptr_t>(stats) & 15u)) || (reinterpret_cast<uintptr_t>(records) & 15u))
        return fail(MBOTS_E_INVALID, "records and stats must be 16-byte aligned");
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(mbots::launch_unpack_rollout(records, (uint32_t)rows, with_depth ? 1 : 0, obs, reward, stats,
                                         as_stream(stream)));
    return MBOTS_OK;
}

int mbots_join(mbots_handle *h, void *stream)
{
    if (!h) return fail(MBOTS_E_INVALID, "null handle");
    if (h->cpu) return MBOTS_OK;   // synchronous: nothing outstanding
    HIP_TRY(hipSetDevice(h->device));
    int rc = use_stream(h, as_stream(stream));
    if (rc) return rc;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    unsigned long long cid = 0;
    HIP_TRY(hipStreamGetCaptureInfo(as_stream(stream), &cs, &cid));
    // the table halves and the host's deferred-move bookkeeping alternate per
    // step: a graph of an odd number of steps would leave them out of step
    // with the device after every replay
    if (cs == hipStreamCaptureStatusActive && cid == h->cap_seen && (h->cap_steps & 1))
        return fail(MBOTS_E_INVALID, "a captured sequence must hold an even number of steps (" +
                                         std::to_string(h->cap_steps) + " recorded)");
    if (h->last_join >= 0) HIP_TRY(hipStreamWaitEvent(as_stream(stream), h->ev_join[h->last_join], 0));
    return MBOTS_OK;
}

int mbots_record_sensor_done(mbots_handle *h, void *event)
{
    if (!h || !event) return fail(MBOTS_E_INVALID, "null argument");
    if (h->cpu || h->last_join < 0) return fail(MBOTS_E_INVALID, "no sensor launched on the device");
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipEventRecord(static_cast<hipEvent_t>(event), h->aux));
    return MBOTS_OK;
}

int mbots_agent_steps(mbots_handle *h, uint64_t *out)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (h->cpu) {
        *out = h->cpu->agent_steps();
        return MBOTS_OK;
    }
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long v = 0;
    HIP_TRY(hipMemcpy(&v, h->S.agent_steps, sizeof(v), hipMemcpyDeviceToHost));
    *out = v;
    return MBOTS_OK;
}

int mbots_overflow(mbots_handle *h, uint64_t *out)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (h->cpu) {
        *out = h->cpu->overflow();
        return MBOTS_OK;
    }
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipDeviceSynchronize());
    std::vector<uint32_t> v(h->cfg.num_worlds);
    HIP_TRY(hipMemcpy(v.data(), h->S.overflow, v.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    uint64_t s = 0;
    for (uint32_t x : v) s += x;
    *out = s;
    return MBOTS_OK;
}

// ---- checkpoint / restore (absent in the reference) ----
// Blob: header + the live state after the last step: agent SoA columns (all
// W x cap slots), per-world arrays, and the first N rows of every column of the
// current export table.  Restoring into a manager of the same configuration
// puts the table in half 0, clears the scan tiles and continues bit-exactly.
int mbots_checkpoint_size(mbots_handle *h, uint64_t *out)
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (h->cpu) {
        *out = h->cpu->checkpoint_bytes();
        return MBOTS_OK;
    }
    int rc = sync_totals(h);
    if (rc) return rc;
    *out = ckpt_bytes(ckpt_segments(h, h->T[h->tb], h->h_totals[mbots::kTotRows]));
    return MBOTS_OK;
}

int mbots_save_checkpoint(mbots_handle *h, void *dst, uint64_t bytes)
{
    if (!h || !dst) return fail(MBOTS_E_INVALID, "null argument");
    if (h->cpu) {
        std::string err;
        const int r = h->cpu->save(dst, bytes, err);
        return r ? fail(r, err) : MBOTS_OK;
    }
    HIP_TRY(hipSetDevice(h->device));
    if (int rc = capture_guard(h, h->last_stream)) return rc;
    int rc0 = materialize_prev(h, h->last_stream);
    if (!rc0) rc0 = materialize_prev_ah(h, h->last_stream);
    if (!rc0) rc0 = materialize_cur_ah(h, h->last_stream, 3);
    if (!rc0) rc0 = materialize_psem(h, h->last_stream);
    if (rc0) return rc0;
    HIP_TRY(hipDeviceSynchronize());   // the sensor's finder / semantic rows included
    int rc = sync_totals(h);
    if (rc) return rc;
    const uint32_t n_rows = h->h_totals[mbots::kTotRows];   // the shard ghost's rows included
    const auto segs = ckpt_segments(h, h->T[h->tb], n_rows);
    const size_t need = ckpt_bytes(segs);
    if (bytes < need) return fail(MBOTS_E_INVALID, "checkpoint buffer too small");
    CkptHeader hd{};
    memcpy(hd.magic, "MBOTSCK", 8);
    hd.version = kCkptVersion;
    hd.num_worlds = h->cfg.num_worlds;
    hd.cap = h->cfg.agent_capacity;
    hd.A = h->cfg.init_num_agents_per_world;
    hd.world_offset = h->cfg.world_offset;
    hd.flags = h->cfg.flags;
    hd.seed = h->cfg.rand_seed;
    hd.n_rows = n_rows;
    hd.bytes = need;
    hd.sensed = h->sensed ? 1u : 0u;
    char *p = static_cast<char *>(dst);
    memcpy(p, &hd, sizeof(hd));
    p += sizeof(hd);
    for (const Seg &s : segs) {
        if (s.bytes) HIP_TRY(hipMemcpy(p, s.p, s.bytes, hipMemcpyDeviceToHost));
        p += s.bytes;
    }
    return MBOTS_OK;
}

int mbots_load_checkpoint(mbots_handle *h, const void *src, uint64_t bytes)
{
    if (!h || !src) return fail(MBOTS_E_INVALID, "null argument");
    if (h->cpu) {
        std::string err;
        const int r = h->cpu->load(src, bytes, err);
        if (r) return fail(r, err);
        h->ovf_reported = (uint32_t)std::min<uint64_t>(h->cpu->overflow(), 0xFFFFFFFFu);
        return MBOTS_OK;
    }
    if (bytes < sizeof(CkptHeader)) return fail(MBOTS_E_INVALID, "checkpoint truncated");
    CkptHeader hd;
    memcpy(&hd, src, sizeof(hd));
    if (memcmp(hd.magic, "MBOTSCK", 8) != 0 || hd.version != kCkptVersion)
        return fail(MBOTS_E_INVALID, "not a checkpoint of this version");
    // (another agent_capacity is fine when every world of the blob fits this
    // manager's: its per-slot columns are re-laid out, world by world -- a
    // learner growing its worlds' capacity, SimManager(agent_capacity="auto"))
    if (hd.num_worlds != h->cfg.num_worlds || hd.cap < 4 || hd.cap > (uint32_t)mbots::kMaxCap ||
        hd.A != h->cfg.init_num_agents_per_world || hd.world_offset != h->cfg.world_offset ||
        hd.flags != h->cfg.flags || hd.seed != h->cfg.rand_seed)
        return fail(MBOTS_E_INVALID, "checkpoint configuration differs from the manager's");
    const uint32_t cap = h->cfg.agent_capacity, cap_src = hd.cap;
    if (hd.n_rows > (uint64_t)h->S.W * cap)
        return fail(MBOTS_E_INVALID, "checkpoint row count out of range");
    if (int rc = capture_guard(h, h->last_stream)) return rc;
    const auto segs = ckpt_segments(h, h->T[0], hd.n_rows);
    const auto segs_src = ckpt_segments(h, h->T[0], hd.n_rows, cap_src);
    if (bytes < ckpt_bytes(segs_src) || hd.bytes != ckpt_bytes(segs_src))
        return fail(MBOTS_E_INVALID, "checkpoint size mismatch");
    {
        // the blob's own totals must agree with its header before anything is
        // overwritten (a mismatch used to leave the manager half
        // restored), and every world's population must fit this capacity
        const char *q = static_cast<const char *>(src) + sizeof(hd);
        for (const Seg &s : segs_src) {
            if (s.p == h->S.totals) {
                uint32_t tot[8];
                memcpy(tot, q, sizeof(tot));
                if (tot[mbots::kTotRows] != hd.n_rows || tot[0] > hd.n_rows)
                    return fail(MBOTS_E_INVALID, "checkpoint row count disagrees with its saved totals");
            }
            if (s.p == h->S.n) {
                for (size_t w = 0; w < h->S.W; ++w) {
                    int32_t n;
                    memcpy(&n, q + 4 * w, 4);
                    if (n < 0 || (uint32_t)n > cap)
                        return fail(MBOTS_E_INVALID, "a world of the checkpoint holds " + std::to_string(n) +
                                                         " agents, more than agent_capacity " + std::to_string(cap));
                }
            }
            q += s.bytes;
        }
    }
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipDeviceSynchronize());
    const char *p = static_cast<const char *>(src) + sizeof(hd);
    for (size_t i = 0; i < segs.size(); ++i) {
        const Seg &s = segs[i];
        if (i < kSlotSegs && cap != cap_src) {   // [world][cap_src] -> [world][cap]
            HIP_TRY(hipMemcpy2D(s.p, (size_t)cap * 4, p, (size_t)cap_src * 4, (size_t)std::min(cap, cap_src) * 4,
                                h->S.W, hipMemcpyHostToDevice));
        } else if (s.bytes) {
            HIP_TRY(hipMemcpy(s.p, p, s.bytes, hipMemcpyHostToDevice));
        }
        p += segs_src[i].bytes;
    }
    HIP_TRY(hipMemset(h->S.tiles, 0, (size_t)2 * h->S.ntiles * mbots::kTileBuckets * 5 * sizeof(int32_t)));
    if (h->S.mixed) {
        // the first K1 after the load (parity 0) reads the class list of slot 1
        HIP_TRY(hipMemset(h->S.big_cnt, 0, 4 * sizeof(uint32_t)));
        HIP_TRY(mbots::launch_build_lists(h->S, 1, nullptr));
    }
    h->tb = 0;
    h->parity = 0;
    h->last_join = -1;
    h->prev_join = -1;
    h->waited_serial = h->sensor_serial;   // (the device is idle)
    h->join_epoch = 0;
    h->prev_lazy[0] = h->prev_lazy[1] = false;
    h->ah_pending[0] = h->ah_pending[1] = false;
    h->six_pending[0] = h->six_pending[1] = false;
    h->cur_ah_pending[0] = h->cur_ah_pending[1] = false;
    h->psem_pending[0] = h->psem_pending[1] = false;
    h->a_alias[0] = h->a_alias[1] = h->h_alias[0] = h->h_alias[1] = false;
    h->forced = 0;
    h->prefetched = 0;
    h->steps = 1;
    h->sensed = hd.sensed != 0;
    hipStream_t st = nullptr;
    h->last_stream = st;
    h->totals_ok = false;
    int rc = record_totals(h, st);
    if (rc) return rc;
    HIP_TRY(hipDeviceSynchronize());
    h->ovf_reported = h->h_totals[mbots::kTotOverflow];   // drops before the checkpoint were reported then
    h->maxpop_stale = true;
    return MBOTS_OK;
}

int mbots_world_state(mbots_handle *h, uint32_t world, float *xy_rwrz, int32_t *sp_hp_finder,
                      uint64_t *food, uint32_t *food_rot, int32_t *n_out)
{
    using namespace mbots;
    if (!h || !xy_rwrz || !sp_hp_finder || !food || !n_out) return fail(MBOTS_E_INVALID, "null argument");
    if (world >= h->cfg.num_worlds) return fail(MBOTS_E_INVALID, "world out of range");
    if (h->cpu) {
        h->cpu->world_state(world, xy_rwrz, sp_hp_finder, food, food_rot, n_out);
        return MBOTS_OK;
    }
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipDeviceSynchronize());
    const SimState &S = h->S;
    const size_t cap = h->cfg.agent_capacity, base = (size_t)world * cap;
    std::vector<float> f(cap);
    std::vector<int32_t> v(cap);
    const float *fc[4] = {S.x, S.y, S.rw, S.rz};
    for (int c = 0; c < 4; ++c) {
        HIP_TRY(hipMemcpy(f.data(), fc[c] + base, cap * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < cap; ++i) xy_rwrz[i * 4 + c] = f[i];
    }
    const int32_t *ic[3] = {S.species, S.health, S.finder};
    for (int c = 0; c < 3; ++c) {
        HIP_TRY(hipMemcpy(v.data(), ic[c] + base, cap * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < cap; ++i) sp_hp_finder[i * 3 + c] = v[i];
    }
    HIP_TRY(hipMemcpy(food, S.food + (size_t)world * kNumChunks, kNumChunks * 8, hipMemcpyDeviceToHost));
    if (food_rot)
        HIP_TRY(hipMemcpy(food_rot, S.food_rot + (size_t)world * kNumPkg, kNumPkg * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(n_out, S.n + world, 4, hipMemcpyDeviceToHost));
    return MBOTS_OK;
}

int mbots_enable_kernel_timing(mbots_handle *h, int32_t enable)
{
    if (!h) return fail(MBOTS_E_INVALID, "null handle");
    if (h->cpu) return MBOTS_OK;   // no kernels
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipDeviceSynchronize());
    for (auto &p : h->pending) { h->pool.push_back(p.a); h->pool.push_back(p.b); }
    h->pending.clear();
    for (int k = 0; k < MBOTS_TK_COUNT; ++k) { h->acc_ms[k] = 0.0; h->acc_n[k] = 0; }
    h->timing = enable != 0;
    return MBOTS_OK;
}

int mbots_schedule_info(mbots_handle *h, uint32_t out[4])
{
    if (!h || !out) return fail(MBOTS_E_INVALID, "null argument");
    if (h->cpu) {
        out[0] = out[1] = out[2] = 0;
        out[3] = (uint32_t)h->steps;
        return MBOTS_OK;
    }
    out[0] = (h->k1_finder ? 1u : 0u) | (h->sig_fork ? 2u : 0u) | (h->sig_join ? 4u : 0u) | (h->swap ? 8u : 0u) |
             (h->S.mixed ? 16u : 0u);
    out[1] = h->epoch;
    out[2] = h->epoch_wraps;
    out[3] = (uint32_t)h->steps;
    return MBOTS_OK;
}

int mbots_kernel_times(mbots_handle *h, double ms[MBOTS_TK_COUNT], uint64_t launches[MBOTS_TK_COUNT])
{
    if (!h) return fail(MBOTS_E_INVALID, "null handle");
    if (h->cpu) {
        for (int k = 0; k < MBOTS_TK_COUNT; ++k) {
            if (ms) ms[k] = 0.0;
            if (launches) launches[k] = 0;
        }
        return MBOTS_OK;
    }
    HIP_TRY(hipSetDevice(h->device));
    for (auto &p : h->pending) {
        HIP_TRY(hipEventSynchronize(p.b));
        float t = 0.0f;
        HIP_TRY(hipEventElapsedTime(&t, p.a, p.b));
        h->acc_ms[p.kind] += t;
        h->acc_n[p.kind] += 1;
        h->pool.push_back(p.a);
        h->pool.push_back(p.b);
    }
    h->pending.clear();
    for (int k = 0; k < MBOTS_TK_COUNT; ++k) {
        if (ms) ms[k] = h->acc_ms[k];
        if (launches) launches[k] = h->acc_n[k];
    }
    return MBOTS_OK;
}

}  // extern "C"
