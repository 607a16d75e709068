// mbots_kernels.hip -- hand-written gfx950 kernels of the per-step ECS sweep.
//
// Layout: agent state is SoA, [world][slot] with a
// per-world slot capacity `cap`; one wave64 owns one world (4 worlds per
// 256-thread workgroup, waves never wait on each other except at the very end
// of K1), staging the world in LDS.  The exported observation table is
// species-major (species, world, slot) and written into the other half of a
// double-buffered table every step.
//
// step() = K1 world_step (ECS systems, per-world compaction into the other
// state half, per-tile species counts) -> K2 scan (species-major row offsets)
// -> fork: K3b sensor (raycast + finder, internal stream)  ||  K3a export_rows
// (current observations, reward, old->new row map) -> K4 move (Action, Hidden,
// Prev*, prev sensor to the new rows).  shift_observations() = K5 shift.
// DESIGN.md section 4 has the schedule and each kernel's bound.
// Probe switches (MB_COUNT, MB_SKIP_*, MB_PROBE_ALL_DEEP) build instruction-
// count and timing probes whose rows are wrong.  They need MB_PROBE_BUILD,
// which only scripts/build_var.sh probe builds pass (the Makefile refuses it).
#if (defined(MB_COUNT) || defined(MB_SKIP_WIDE) || defined(MB_SKIP_P2) || defined(MB_SKIP_OUT) || \
     defined(MB_PROBE_ALL_DEEP)) && !defined(MB_PROBE_BUILD)
#error "probe switches give wrong rows: build probes into build_var/ with -DMB_PROBE_BUILD, never the product"
#endif
#include <hip/hip_ext.h>
#include "mbots_kernels.hpp"
#include <stdlib.h>
#include <algorithm>
#include <type_traits>
#include "mbots_ray.hpp"

namespace mbots {

constexpr int kWorldsPerBlock = 4;
constexpr int kTileWorlds = 1024;             // worlds per scan tile (K2 block)

#ifndef MB_SHIFT_UNROLL
#define MB_SHIFT_UNROLL 2   // items per thread per pass of the fused shift (2 vs 1: the
                            // driver's window -1.5 %, steady state +-0; 4 and 8 with
                            // proportionally fewer blocks +1 / +7 %: DESIGN_EXPERIMENTS r6)
#endif
#ifndef MB_NT
#define MB_NT 35  // non-temporal stores: 1 K4, 2 K5, 4 K3a, 8 sensor output;
                  // non-temporal loads: 32 K4 sources, 64 K5 sources
#endif
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// a 4-byte store written through to memory (MB_WT: system scope, the L2 keeps
// no dirty copy; else a plain store)
#ifndef MB_WT
#define MB_WT 1
#endif
template <typename T>
__device__ __forceinline__ void st_wt(T *p, T v)
{
    static_assert(sizeof(T) == 4, "4-byte columns");
    if (MB_WT) __hip_atomic_store(reinterpret_cast<uint32_t *>(p), __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else *p = v;
}
__device__ __forceinline__ void st_stream(uint32_t *p, uint32_t v, bool nt)
{
    if (nt) __builtin_nontemporal_store(v, p);
    else *p = v;
}
__device__ __forceinline__ void st_stream(int32_t *p, int32_t v, bool nt)
{
    if (nt) __builtin_nontemporal_store(v, p);
    else *p = v;
}
__device__ __forceinline__ void st_stream(float *p, float v, bool nt)
{
    if (nt) __builtin_nontemporal_store(v, p);
    else *p = v;
}
__device__ __forceinline__ void st_stream(uint2 *p, uint2 v, bool nt)
{
    if (nt) __builtin_nontemporal_store(u32x2{v.x, v.y}, reinterpret_cast<u32x2 *>(p));
    else *p = v;
}
__device__ __forceinline__ void st_stream(float2 *p, float2 v, bool nt)
{
    st_stream(reinterpret_cast<uint2 *>(p), make_uint2(__float_as_uint(v.x), __float_as_uint(v.y)), nt);
}
__device__ __forceinline__ void st_stream(uint4 *p, uint4 v, bool nt)
{
    if (nt) __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4 *>(p));
    else *p = v;
}
__device__ __forceinline__ void st_stream(int4 *p, int4 v, bool nt)
{
    st_stream(reinterpret_cast<uint4 *>(p), make_uint4(v.x, v.y, v.z, v.w), nt);
}
// loads of data read once
__device__ __forceinline__ uint32_t ld_stream(const uint32_t *p, bool nt)
{
    return nt ? __builtin_nontemporal_load(p) : *p;
}
__device__ __forceinline__ uint2 ld_stream(const uint2 *p, bool nt)
{
    if (!nt) return *p;
    const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(p));
    return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint4 ld_stream(const uint4 *p, bool nt)
{
    if (!nt) return *p;
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}


// ---------------------------------------------------------------------------
// Food packages: HBM keeps one 8-byte record per chunk (5 x (x | y << 4) bytes,
// live mask in byte 5: kMaxFoodPerPackage = 1, so numFood is a bit);
// LDS keeps one u16 per package: x | y << 4 | numFood << 8.
// ---------------------------------------------------------------------------
constexpr uint32_t kPkgLive = 1u << 8;
__device__ __forceinline__ void food_unpack(uint64_t rec, uint16_t *pk)
{
#pragma unroll
    for (int k = 0; k < kMaxPkg; ++k) {
        const uint32_t xy = (uint32_t)(rec >> (8 * k)) & 0xFFu;
        const uint32_t live = (uint32_t)(rec >> (40 + k)) & 1u;
        pk[k] = (uint16_t)(xy | (live << 8));
    }
}
__device__ __forceinline__ uint64_t food_pack(const uint16_t *pk)
{
    uint64_t rec = 0;
#pragma unroll
    for (int k = 0; k < kMaxPkg; ++k) {
        const uint32_t p = pk[k];
        rec |= (uint64_t)(p & 0xFFu) << (8 * k);
        rec |= (uint64_t)((p >> 8) & 1u) << (40 + k);
    }
    return rec;
}

// ---------------------------------------------------------------------------
// Per-world LDS image used by the world-step kernel
// ---------------------------------------------------------------------------
// kCap: the slot capacity class (128: the default, 8 blocks per CU; 256)
template <int kCap>
struct WorldLDS {
    float x[kCap], y[kCap], rw[kCap], rz[kCap];
    int32_t accum[kCap];
    int16_t finder[kCap];
    int8_t species[kCap];
    uint8_t flags[kCap];
    // healthSync's cell keys / package takes (slots < n0) share storage with the
    // surroundings written after it (children/respawns, slots >= n0, only
    // touch the sur half)
    union {
        struct { int32_t key[kCap]; int32_t take[kCap]; };
        struct { float sur0[kCap]; float sur1[kCap]; };
    };
    uint16_t food[kNumPkg];
    uint32_t chunk[kNumChunks];   // ChunkInfo: numAgents << 16 | totalSpeed (<= 256 x 2)
    uint32_t cnt[kNumSpecies], hsum[kNumSpecies];
    int32_t need[kNumSpecies];
    int32_t scount[kNumSpecies];
    int32_t consumed;
};

// flags bits
constexpr uint32_t F_HIT_FRIENDLY = 1u << 0;
constexpr uint32_t F_HIT_ENEMY = 1u << 1;
constexpr uint32_t F_ATE = 1u << 2;
constexpr uint32_t F_REPRO = 1u << 3;
constexpr uint32_t F_ALIVE = 1u << 4;
constexpr uint32_t F_BREED = 1u << 5;
constexpr uint32_t F_STATS = 0xFu;


__device__ __forceinline__ uint32_t rng_draw(uint2 key, uint32_t ctr)
{
    return threefry2x32(key.x, key.y, ctr, 0u).x;
}

template <int kCap>
__device__ __forceinline__ void init_slot(WorldLDS<kCap> &L, int s, float x, float y, int32_t sp,
                                          int32_t h)
{
    L.x[s] = x;
    L.y[s] = y;
    L.rw[s] = 1.0f;
    L.rz[s] = 0.0f;
    L.species[s] = (int8_t)sp;
    L.accum[s] = h;
    L.finder[s] = -1;
    L.flags[s] = (uint8_t)F_ALIVE;
    L.sur0[s] = 0.0f;
    L.sur1[s] = 0.0f;
}

// ---------------------------------------------------------------------------
// K1: world step -- resetChunkInfoSystem, addFoodSystem, actionSystem,
// healthSync, updateSurroundingObservation, speciesTrackerUpdate,
// speciesInfoSync + respawn, and the per-world compaction of
// SortArchetypeNode<Agent, WorldID> (sim.cpp:1061-1132).
// ---------------------------------------------------------------------------
template <int kCap>
struct FinderScratch;
template <int kCap, bool kFinder, bool kSkipBig = false>
__device__ bool world_step(SimState &S, const ObsTable &cur, WorldLDS<kCap> &L, FinderScratch<kCap> &F,
                           uint32_t w, uint32_t lane);

#ifndef MB_K1_WPB
#define MB_K1_WPB 8   // 4: K1 +2.5 %, and +7 % step at 4096 worlds; 16: +30 % K1
#endif
constexpr int kK1Worlds = MB_K1_WPB;          // worlds (waves) per K1 block
// per capacity class: the 512 / 1024 / 2048 / 4096-slot images (17 / 34 / 66 /
// 131 KB of LDS a world) take 4 / 2 / 1 / 1 worlds a block (the 4096 image is the
// largest the CU's 160 KB hold)
template <int kCap>
constexpr int k1_worlds() { return kCap <= 256 ? kK1Worlds : kCap == 512 ? 4 : kCap == 1024 ? 2 : 1; }
template <int kCap>
constexpr int k1_min_blocks() { return kCap <= 128 ? 32 / kK1Worlds : kCap <= 256 ? 16 / kK1Worlds : kCap == 512 ? 2 : 1; }
// SGPRs capped at 80: the compiler's own choice (99, no spill at 80) admits only
// 6 waves per SIMD (800 SGPRs per SIMD in 16-register granules plus 16), one
// block in four fewer: K1 87 -> 78 us, step -1.7 %
// kFinder: the finder slots this step reads computed here (world_finders)
// instead of read from the last step's sensor, so K1 need not wait for it
// (small world counts, where the step is a latency chain)
// kSkipBig (mixed classes): worlds whose step could outgrow this class are
// left to world_step_list_kernel
template <int kCap, bool kFinder, bool kSkipBig = false>
__global__ __launch_bounds__(64 * k1_worlds<kCap>(), k1_min_blocks<kCap>())
__attribute__((amdgpu_num_sgpr(80))) void world_step_kernel(
    SimState S, ObsTable cur, int parity)
{
    constexpr int kW1 = k1_worlds<kCap>();
    __shared__ WorldLDS<kCap> lds[kW1];
    __shared__ FinderScratch<kCap> fsc[kFinder ? kW1 : 1];
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = uniform(blockIdx.x * kW1 + wv);
    // (mixed classes: a world whose step could outgrow the small class is the
    // class kernel's, world_step_list_kernel)
    const bool run = w < S.W && world_step<kCap, kFinder, kSkipBig>(S, cur, lds[wv], fsc[kFinder ? wv : 0], w, lane);
    // counter-major tile buckets: [counter][tile][bucket] (K2 reads one
    // counter's buckets as contiguous 16-B words)
    const size_t nent = (size_t)S.ntiles * kTileBuckets;
    int32_t *tiles = S.tiles + (size_t)parity * 5 * nent;
    if constexpr (kW1 == 1) {
        // one world per block: its species/agent counts go straight to the K2
        // scan tile (no block barrier: a block's LDS frees as its world ends)
        if ((!kSkipBig || run) && w < S.Wx && lane < 5) {   // (a shard ghost, w >= Wx, is not counted)
            const int32_t *sc = lds[0].scount;
            atomicAdd(&tiles[lane * nent + (w / kTileWorlds) * kTileBuckets + blockIdx.x % kTileBuckets],
                      lane < 4 ? sc[lane] : sc[0] + sc[1] + sc[2] + sc[3]);
        }
    } else {
        __shared__ int32_t blk[kW1][5];
        // per-block species/agent counts -> the K2 scan tile (one atomic per counter)
        if (lane < 5) {   // (a shard ghost, w >= Wx, is not counted: its rows follow the table's)
            const int32_t *sc = lds[wv].scount;
            blk[wv][lane] = ((!kSkipBig || run) && w < S.Wx) ? (lane < 4 ? sc[lane] : sc[0] + sc[1] + sc[2] + sc[3])
                                                              : 0;
        }
        __syncthreads();
        if (threadIdx.x < 5) {
            int32_t v = 0;
#pragma unroll
            for (int k = 0; k < kW1; ++k) v += blk[k][threadIdx.x];
            const uint32_t tile = (blockIdx.x * kW1) / kTileWorlds;
            atomicAdd(&tiles[threadIdx.x * nent + tile * kTileBuckets + blockIdx.x % kTileBuckets], v);
        }
    }
}

// K1 of the class kernel (mixed classes): the worlds the last K2 listed
// (S.big_k1 of the other parity), a wave per world in a grid-stride loop,
// each world's species / agent counts added to its scan tile itself
template <int kCap>
__global__ __launch_bounds__(64 * k1_worlds<kCap>(), k1_min_blocks<kCap>()) void world_step_list_kernel(
    SimState S, ObsTable cur, int parity)
{
    constexpr int kW1 = k1_worlds<kCap>();
    __shared__ WorldLDS<kCap> lds[kW1];
    __shared__ FinderScratch<kCap> fsc[1];
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lp = (uint32_t)parity ^ 1u;
    const uint32_t cnt = uniform(S.big_cnt[lp * 2]);
    const size_t nent = (size_t)S.ntiles * kTileBuckets;
    int32_t *tiles = S.tiles + (size_t)parity * 5 * nent;
    for (uint32_t i = blockIdx.x * kW1 + wv; i < cnt; i += gridDim.x * kW1) {
        const uint32_t w = uniform((uint32_t)S.big_k1[(size_t)lp * S.W + i]);
        world_step<kCap, false>(S, cur, lds[wv], fsc[0], w, lane);
        if (w < S.Wx && lane < 5) {
            const int32_t *sc = lds[wv].scount;
            atomicAdd(&tiles[lane * nent + (w / kTileWorlds) * kTileBuckets + w % kTileBuckets],
                      lane < 4 ? sc[lane] : sc[0] + sc[1] + sc[2] + sc[3]);
        }
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// K1's finder pass (small world counts): the finder slots this step's actions
// read -- what the last step's sensor computed for its centre ray
// (sim.cpp:1183-1188, read by actionSystem / healthSync :434-454, :547-569;
// the forward ray u = 0, the nearest object by (depth, order)
// beyond the near sphere, an agent's slot if it beats the wall) -- evaluated
// here on the world as K1 staged it (the state the sensor saw) with the
// sensor's predicates (finder_key for discs, box_hit at u = 0 for food
// squares, its wall resolution), so this K1 need not wait for that sensor.
// Only the agents that shoot or breed read their slot: they are the cameras
// (every slot past 64 too, whose action row is loaded later).  A P1-style cull
// of every (camera, object) pair -- |l| <= 1.45 and f >= -0.35 are necessary
// for either kind: a disc is hit only where |l| <= R and f >= 1.1 - R, a
// square only where |l| <= |p| + |q| <= sqrt 2 and f + ext >= 1.1 -- then the
// exact test of the survivors (about one per camera), atomicMin of their keys.
// ---------------------------------------------------------------------------
constexpr float kFinderCullL = 1.45f, kFinderCullF = -0.35f;

template <int kCap>
struct FinderScratch {
    uint32_t queue[128];   // cull survivors: camera | object << 8 (flushed at >= 64)
    uint8_t cam[kCap];     // the cameras' slots
};

template <int kCap>
__device__ void world_finders(const SimState &S, WorldLDS<kCap> &L, FinderScratch<kCap> &F, uint32_t lane,
                              int n0, uint64_t food_rec, const uint32_t (&rot)[kMaxPkg], bool want0)
{
    constexpr int kG = kCap / 64;
    static_assert(kCap * 4 >= 2 * kMaxFood * 8, "food scratch in the take array");
    // scratch: healthSync's arrays, free until it runs
    uint32_t *const fkey = reinterpret_cast<uint32_t *>(L.key);   // [ncam] min key per camera
    float2 *const fobj = reinterpret_cast<float2 *>(L.take);      // [na] food positions (NaN gap)
    float2 *const frot = fobj + kMaxFood;                         // [nf] food (cos, sin)

    // ---- cameras: the slots that shoot or breed (and every slot past 64) ----
    int ncam = 0;
#pragma unroll
    for (int g = 0; g < kG; ++g) {
        const int sl = 64 * g + (int)lane;
        if (64 * g >= n0) break;
        const bool want = sl < n0 && (g > 0 || want0);
        const uint64_t m = ballot64(want);
        if (want) F.cam[ncam + (int)rank_below(m)] = (uint8_t)sl;
        ncam += __popcll(m);
        if (sl < n0) L.finder[sl] = -1;
    }
    // ---- live food packages in (chunk, package) order (the sensor's objects) ----
    const uint32_t live = lane < kNumChunks ? (uint32_t)(food_rec >> 40) & 31u : 0u;
    const int cnt = __popc(live);
    int off = 0, tot = 0;
#pragma unroll
    for (int bt = 0; bt < 3; ++bt) {
        const uint64_t m = ballot64((cnt >> bt) & 1);
        off += (int)rank_below(m) << bt;
        tot += __popcll(m) << bt;
    }
    const int nf = min(tot, kMaxFood);
    const int na = (nf + 7) & ~7;
    {
        const float bx = (float)((lane % kChunksX) * kChunkW), by = (float)((lane / kChunksX) * kChunkW);
        int so = off;
#pragma unroll
        for (int k = 0; k < kMaxPkg; ++k) {
            if ((live >> k) & 1u) {
                const uint32_t xy = (uint32_t)(food_rec >> (8 * k)) & 0xFFu;
                if (so < kMaxFood) {
                    fobj[so] = make_float2((float)(xy & 15u) + bx, (float)(xy >> 4) + by);
                    frot[so].x = __uint_as_float(rot[k]);
                }
                ++so;
            }
        }
    }
    if ((int)lane >= nf && (int)lane < na) fobj[lane] = make_float2(__builtin_nanf(""), __builtin_nanf(""));
    wave_sync();
    // every camera's heading (camera c in lane c % 64, register c / 64) and key
    float hx[kG], hy[kG];
#pragma unroll
    for (int g = 0; g < kG; ++g) {
        hx[g] = hy[g] = 0.0f;
        const int c = 64 * g + (int)lane;
        if (c < ncam) {
            const int sl = F.cam[c];
            heading(L.rw[sl], L.rz[sl], hx[g], hy[g]);
            fkey[c] = kNoKey;
        }
    }
    if ((int)lane < nf) frot[lane] = food_cs(__float_as_uint(frot[lane].x));
    wave_sync();
    if (ncam == 0) return;

    // camera c's heading, from its lane (every lane shuffles)
    auto head = [&](int c, float &ahx, float &ahy) {
        ahx = __shfl(hx[0], c & 63);
        ahy = __shfl(hy[0], c & 63);
#pragma unroll
        for (int g = 1; g < kG; ++g) {
            const float gx = __shfl(hx[g], c & 63), gy = __shfl(hy[g], c & 63);
            if ((c >> 6) == g) { ahx = gx; ahy = gy; }
        }
    };
    const NearPt fnp = finder_np();
    // the exact test of the queued pairs [q0, q0 + cntq), one per lane
    auto exact = [&](int q0, int cntq) {
        const int ln = (int)lane;
        const uint32_t code = ln < cntq ? F.queue[q0 + ln] : 0u;
        const int ic = (int)(code & 0xFFu), j = (int)(code >> 8);
        const int sl = F.cam[ic];
        float ahx, ahy;
        head(ic, ahx, ahy);
        if (ln < cntq) {
            const bool food = j < na;
            const float2 p = food ? fobj[j] : make_float2(L.x[j - na], L.y[j - na]);
            // pair_fl / the oracle's raster: the exact (f, l)
            const float vx = p.x - L.x[sl], vy = p.y - L.y[sl];
            const float f = vx * ahx + vy * ahy;
            const float l = vx * ahy - vy * ahx;
            uint32_t kv;
            if (food) {
                const FoodBox b = box_setup(f, l, frot[j], make_float2(ahx, ahy));
                kv = box_hit(b, 0.0f, true, fnp.c) ? zkey(box_z(b, true), kOrderFood + (uint32_t)j) : kNoKey;
            } else {
                kv = finder_key(f, l, kOrderAgent + (uint32_t)(j - na));
            }
            if (kv != kNoKey) atomicMin(&fkey[ic], kv);
        }
    };

    // ---- the cull: lane = (camera a0 + a, object jb + o) ----
    int nq = 0;
    const int a = (int)lane >> 3, o = (int)lane & 7;
    for (int a0 = 0; a0 < ncam; a0 += 8) {   // wave-uniform
        const int nc = min(8, ncam - a0);
        const int ic = a0 + min(a, nc - 1);
        const int sl = F.cam[ic];
        float ahx, ahy;
        head(ic, ahx, ahy);
        const float cxp = a < nc ? L.x[sl] : __builtin_nanf(""), cyp = L.y[sl];
        // (P1's hoisted projections: f, l within ~1e-5, far inside the margins)
        const float pc = __builtin_fmaf(cxp, ahx, cyp * ahy);
        const float pd = __builtin_fmaf(cxp, ahy, -(cyp * ahx));
        auto cull = [&](int j, float2 p, bool ok) {
            const float f = __builtin_fmaf(p.x, ahx, __builtin_fmaf(p.y, ahy, -pc));
            const float l = __builtin_fmaf(p.x, ahy, __builtin_fmaf(-p.y, ahx, -pd));
            const bool keep = ok & (fabsf(l) <= kFinderCullL) & (f >= kFinderCullF);
            const uint64_t m = ballot64(keep);
            if (keep) F.queue[nq + (int)rank_below(m)] = (uint32_t)ic | ((uint32_t)j << 8);
            nq += __popcll(m);
            if (nq >= 64) {
                wave_sync();
                exact(nq - 64, 64);
                wave_sync();
                nq -= 64;
            }
        };
        // (each iteration's object loaded one iteration ahead: the LDS latency
        // overlaps the previous pair's tests instead of stalling each one)
        if (na > 0) {
            float2 pn = fobj[o];
            for (int jb = 0; jb < na; jb += 8) {
                const float2 p = pn;
                if (jb + 8 < na) pn = fobj[jb + 8 + o];
                cull(jb + o, p, true);
            }
        }
        {
            int tn = min(o, n0 - 1);
            float2 pn = make_float2(L.x[tn], L.y[tn]);
            for (int jb = 0; jb < n0; jb += 8) {
                const float2 p = pn;
                if (jb + 8 < n0) {
                    tn = min(jb + 8 + o, n0 - 1);
                    pn = make_float2(L.x[tn], L.y[tn]);
                }
                cull(na + jb + o, p, (jb + o < n0) & (jb + o != sl));
            }
        }
    }
    if (nq > 0) {
        wave_sync();
        exact(0, nq);
    }
    wave_sync();

    // ---- per camera: the sensor's wall resolution of its finder ray ----
#pragma unroll
    for (int g = 0; g < kG; ++g) {
        const int c = 64 * g + (int)lane;
        if (c >= ncam) break;
        const int sl = F.cam[c];
        const uint32_t kv = fkey[c];
        const uint32_t order = kv & kOrderMask;
        const float z = __uint_as_float(kv & ~kOrderMask);
        const float px = L.x[sl], py = L.y[sl];
        const float ch_x = hx[g], ch_y = hy[g];
        const float fx = fnp.c * ch_x + fnp.s * ch_y, fy = fnp.c * ch_y + fnp.s * (-ch_x);
        const int fcls = wall_class(px + fx, py + fy);
        const bool edge = !strictly_inside(px, py);
        bool see;
        if ((fcls != kWallInner) | edge)
            see = (fcls == kWallNone) | ((fcls == kWallInner) && beats_wall(px, py, ch_x, ch_y, z));
        else
            see = beats_wall_in(kInLo - px, kInHiX - px, kInLo - py, kInHiY - py, ch_x, ch_y, z);
        const bool agent = (kv != kNoKey) & (order >= kOrderAgent) & see;
        L.finder[sl] = (int16_t)(agent ? (int32_t)(order - kOrderAgent) : -1);
    }
    wave_sync();
}

// returns false, having done nothing, for a world kSkipBig leaves to the
// class kernel
template <int kCap, bool kFinder, bool kSkipBig>
__device__ bool world_step(SimState &S, const ObsTable &cur, WorldLDS<kCap> &L, FinderScratch<kCap> &F,
                           uint32_t w, uint32_t lane)
{
    constexpr int kG = kCap / 64;   // 64-slot groups
    const uint32_t cap = S.cap;
    const size_t base = (size_t)w * cap;
    const int n0 = uniform(S.n[w]);
    if (kSkipBig && k1_needs_class(n0, S.A)) return false;

    // ---- stage the world in LDS; slot `lane`'s action row is fetched now and
    // consumed after addFood (its latency hides behind that serial phase) ----
    // The old export rows stay in registers (rows[g]: slot 64 g + lane): only
    // the slot's own lane reads them (action fetch, compaction).
    int2 pa0 = make_int2(0, 0), pa1 = pa0, pa2 = pa0;
    int32_t rows[kG];
#pragma unroll
    for (int g = 0; g < kG; ++g) rows[g] = -1;
    // per-world records: issued with the first batch (none depends on n0)
    const uint64_t food_rec = lane < kNumChunks ? S.food[(size_t)w * kNumChunks + lane] : 0ull;
    // (kFinder) the food squares' rotations: the chunk's package 0 with the
    // record, the others where the record says live
    uint32_t frot_ld[kMaxPkg];
#pragma unroll
    for (int k = 0; k < kMaxPkg; ++k) frot_ld[k] = 0u;
    if (kFinder && lane < kNumChunks) frot_ld[0] = S.food_rot[(size_t)w * kNumPkg + lane];
    const uint2 key = S.key[w];
    uint32_t ctr = S.ctr[w];
    int32_t cur_food = S.cur_food[w];
    {
        // slots < min(n0, 64) (n0 is one scalar load; the first wave round is
        // bandwidth-bound, so the ~half of the lanes past n0 stay idle: K1 -2.4 %)
        // -- except the export rows, loaded for every lane beside n0 so that the
        // action rows they point at are fetched in the same round as the slot
        // columns, not after them
        const bool in = (int)lane < n0;
        const size_t i = base + lane;
        const int32_t row_any = lane < cap ? __builtin_nontemporal_load(S.obsrow + i) : -1;
        const int32_t row = in ? row_any : -1;
        const float x = in ? S.x[i] : 0.0f, y = in ? S.y[i] : 0.0f;
        const float rw = in ? S.rw[i] : 0.0f, rz = in ? S.rz[i] : 0.0f;
        const int32_t sp = in ? S.species[i] : 0, hp = in ? S.health[i] : 0;
        // (kFinder: the finder slots are world_finders', not the last sensor's --
        // except before any sensor ran, when S.finder holds the init's "none")
        const int32_t fd = (in && (!kFinder || S.finder_from_state)) ? S.finder[i] : -1;
        if ((int)lane < n0) {
            rows[0] = row;
            if (row >= 0) {
                const int2 *ap = reinterpret_cast<const int2 *>(cur.action + (size_t)row * 6);
                pa0 = ap[0]; pa1 = ap[1]; pa2 = ap[2];
            }
            L.x[lane] = x;
            L.y[lane] = y;
            L.rw[lane] = rw;
            L.rz[lane] = rz;
            L.species[lane] = (int8_t)sp;
            L.accum[lane] = hp;
            L.finder[lane] = (int16_t)fd;
            L.flags[lane] = (uint8_t)F_ALIVE;
        }
    }
#pragma unroll
    for (int g = 1; g < kG; ++g) {   // slots past 64
        const int i = 64 * g + (int)lane;
        if (64 * g >= n0) break;
        if (i < n0) {
            rows[g] = S.obsrow[base + i];
            L.x[i] = S.x[base + i];
            L.y[i] = S.y[base + i];
            L.rw[i] = S.rw[base + i];
            L.rz[i] = S.rz[base + i];
            L.species[i] = (int8_t)S.species[base + i];
            L.accum[i] = S.health[base + i];
            L.finder[i] = (kFinder && !S.finder_from_state) ? (int16_t)-1 : (int16_t)S.finder[base + i];
            L.flags[i] = (uint8_t)F_ALIVE;
        }
    }
    if (kFinder && lane < kNumChunks) {
        const uint32_t lv = (uint32_t)(food_rec >> 40) & 31u;
#pragma unroll
        for (int k = 1; k < kMaxPkg; ++k)
            if ((lv >> k) & 1u) frot_ld[k] = S.food_rot[(size_t)w * kNumPkg + k * kNumChunks + lane];
    }
    if (lane < kNumChunks) food_unpack(food_rec, &L.food[lane * kMaxPkg]);
    if (lane < kNumChunks) L.chunk[lane] = 0u;   // resetChunkInfoSystem
    if (lane < kNumSpecies) { L.cnt[lane] = 0u; L.hsum[lane] = 0u; L.scount[lane] = 0; }
    if (lane == 0) L.consumed = 0;
    wave_sync();
    // the finder slots the shoot / breed actions read (kFinder: computed here)
    if constexpr (kFinder) {
        if (!S.finder_from_state) world_finders<kCap>(S, L, F, lane, n0, food_rec, frot_ld, (pa2.x | pa2.y) != 0);
    }
#ifdef MB_FINDER_CHECK   // debug build: the computed slots against the last sensor's (run serialised)
    if (kFinder && !S.finder_from_state) {
        for (int i = lane; i < n0; i += 64) {
            const bool cam = i >= 64 || ((pa2.x | pa2.y) != 0);
            const int mine = L.finder[i], sens = S.finder[base + i];
            if (cam && mine != sens)
                printf("FINDER w %u slot %d n0 %d mine %d sensor %d pos %.3f %.3f rot %.4f %.4f\n", w, i, n0, mine, sens,
                       L.x[i], L.y[i], L.rw[i], L.rz[i]);
        }
    }
#endif

    // ---- addFoodSystem (sim.cpp:363-387) + addFoodToChunk (:308-361) ----
    // The serial draw sequence uses at most 2 + 3 x 7 = 23 counters: lane k
    // computes draw ctr + k up front and the (wave-uniform) logic reads them
    // with readlane.  The draws past the ones addFood takes are the respawns'
    // (speciesInfoSync below continues the same counter), so the 64 lanes'
    // draws serve both phases: one Threefry per wave where there were three.
    const uint32_t ctr0 = ctr;
    const uint32_t dl = rng_draw(key, ctr + lane);
    {
        auto D = [&](uint32_t k) { return (uint32_t)__builtin_amdgcn_readlane((int)dl, (int)k); };
        uint32_t k = 0;
        if (sample_i32(D(k++), 0, 10) == 0) {
            uint32_t nfood = (uint32_t)sample_i32(D(k++), 1, 3);
            const uint32_t diff = (uint32_t)kFoodCap - (uint32_t)cur_food;
            if (diff < nfood) nfood = diff;
            for (uint32_t f = 0; f < nfood; ++f) {
                const uint32_t cx = (uint32_t)sample_i32(D(k++), 0, kChunksX);
                const uint32_t cy = (uint32_t)sample_i32(D(k++), 0, kChunksY);
                const int chunk = (int)(cx + cy * kChunksX);
                k += 2;   // two unused draws (sim.cpp:311-312)
                for (int q = 0; q < kMaxPkg; ++q) {
                    const uint32_t p = L.food[chunk * kMaxPkg + q];
                    if ((p & kPkgLive) == 0u) {
                        const uint32_t rx = (uint32_t)sample_i32(D(k++), 0, kChunkW);
                        const uint32_t ry = (uint32_t)sample_i32(D(k++), 0, kChunkW);
                        // food entity rotation angleAxis(2 pi U, z) (sim.cpp:338-341):
                        // its quarter-turn fraction, the low 22 bits of U's 24
                        const uint32_t rot = (D(k++) >> 8) & 0x3FFFFFu;
                        if (lane == 0) {
                            L.food[chunk * kMaxPkg + q] = (uint16_t)((rx & 15u) | ((ry & 15u) << 4) | kPkgLive);
                            S.food_rot[((size_t)w * kMaxPkg + q) * kNumChunks + chunk] = rot;
                        }
                        cur_food += 1;
                        break;
                    }
                }
                wave_sync();
            }
        }
        ctr += k;
    }

    // ---- actionSystem (sim.cpp:419-502) ----
#pragma unroll
    for (int g = 0; g < kG; ++g) {
        const int i = 64 * g + (int)lane;
        if (64 * g >= n0) break;
        if (i >= n0) continue;
        int2 a0 = pa0, a1 = pa1, a2 = pa2;
        const int32_t row = rows[g];
        if (g > 0 && row >= 0) {
            const int2 *ap = reinterpret_cast<const int2 *>(cur.action + (size_t)row * 6);
            a0 = ap[0]; a1 = ap[1]; a2 = ap[2];
        }
        const int32_t act[6] = {a0.x, a0.y, a1.x, a1.y, a2.x, a2.y};
        const int32_t sp = L.species[i];
        uint32_t fl = F_ALIVE | (act[5] ? F_BREED : 0u);
        const int32_t tgt = L.finder[i];
        if (act[4] && tgt >= 0) {
            atomicAdd(&L.accum[tgt], -50);
            fl |= (L.species[tgt] == sp) ? F_HIT_FRIENDLY : F_HIT_ENEMY;
        }
        float rw = L.rw[i], rz = L.rz[i];
        if (act[2]) {
            float nw = rw * kRotC - rz * kRotS;
            float nz = rw * kRotS + rz * kRotC;
            rw = nw; rz = nz;
        } else if (act[3]) {
            float nw = rw * kRotC - rz * (-kRotS);
            float nz = rw * (-kRotS) + rz * kRotC;
            rw = nw; rz = nz;
        }
        float x = L.x[i], y = L.y[i];
        const float ox = x, oy = y;
        float dx, dy;
        heading(rw, rz, dx, dy);
        if (act[0]) { x = x + dx; y = y + dy; }
        else if (act[1]) { x = x - dx; y = y - dy; }
        x = fmin_std(kLx - 1.0f, fmax_std(0.0f, x));
        y = fmin_std(kLy - 1.0f, fmax_std(0.0f, y));
        float ddx = x - ox, ddy = y - oy;
        float len = sqrtf(ddx * ddx + ddy * ddy);
        int32_t ci = chunk_index(floorf((x / 1.0f) / 16.0f), floorf((y / 1.0f) / 16.0f));
        atomicAdd(&L.chunk[ci], (1u << 16) + (uint32_t)(len * 2.0f));
        L.x[i] = x; L.y[i] = y; L.rw[i] = rw; L.rz[i] = rz;
        L.flags[i] = (uint8_t)fl;
    }
    wave_sync();

    // ---- healthSync (sim.cpp:505-581) ----
    // food: the k-th agent (slot order) standing on a cell takes the k-th live
    // package of that cell (serial consume() order made deterministic).
    for (int i = lane; i < n0; i += 64) {
        float chx = (L.x[i] / 1.0f) / 16.0f, chy = (L.y[i] / 1.0f) / 16.0f;
        uint32_t cx = (uint8_t)(16.0f * (chx - floorf(chx)));
        uint32_t cy = (uint8_t)(16.0f * (chy - floorf(chy)));
        int32_t ci = chunk_index(chx, chy);
        L.key[i] = (ci << 8) | (int32_t)(cy << 4) | (int32_t)cx;
    }
    wave_sync();
    for (int i = lane; i < n0; i += 64) {
        const int32_t kk = L.key[i];
        const int ci = kk >> 8;
        const uint32_t cx = (uint32_t)kk & 15u, cy = ((uint32_t)kk >> 4) & 15u;
        const uint32_t cell = cx | (cy << 4) | kPkgLive;   // a live package on this cell
        int navail = 0;
        for (int k = 0; k < kMaxPkg; ++k) navail += (uint32_t)L.food[ci * kMaxPkg + k] == cell ? 1 : 0;
        int take = -1;
        if (navail > 0) {
            int rank = 0;
            for (int j = 0; j < i; ++j) rank += (L.key[j] == kk) ? 1 : 0;
            if (rank < navail) {
                for (int k = 0; k < kMaxPkg; ++k) {
                    if ((uint32_t)L.food[ci * kMaxPkg + k] == cell) {
                        if (rank == 0) { take = ci * kMaxPkg + k; break; }
                        --rank;
                    }
                }
            }
        }
        L.take[i] = take;
    }
    wave_sync();
    int n1 = n0;
    uint32_t ovf = 0;
    for (int b = 0; b < n0; b += 64) {
        const int i = b + (int)lane;
        const bool active = i < n0;
        bool want_child = false;
        if (active) {
            int32_t h = L.accum[i];
            uint32_t fl = L.flags[i];
            const int take = L.take[i];
            if (take >= 0) {
                L.food[take] &= (uint16_t)0xFFu;   // numFood 1 -> 0
                atomicAdd(&L.consumed, 1);
                h = (int32_t)((float)h + 20.0f);
                fl |= F_ATE;
            }
            const int32_t tgt = L.finder[i];
            if ((fl & F_BREED) && h > 10 && tgt >= 0) {
                if (L.species[tgt] == L.species[i]) {
                    h -= 40;
                    fl |= F_REPRO;
                    want_child = true;
                }
            }
            if (h <= 0) fl &= ~F_ALIVE;
            L.accum[i] = h;
            L.flags[i] = (uint8_t)fl;
        }
        const uint64_t m = ballot64(want_child);
        if (want_child) {
            const int s = n1 + (int)rank_below(m);
            if (s < (int)cap) init_slot(L, s, L.x[i], L.y[i], L.species[i], 50);
        }
        const int made = __popcll(m);
        const int room = (int)cap - n1;
        if (made > room) { ovf += (uint32_t)(made - room); n1 = (int)cap; }
        else n1 += made;
    }
    wave_sync();
    cur_food -= L.consumed;
    // ---- updateSurroundingObservation (sim.cpp:583-654) + tracker (:719-734) ----
    for (int i = lane; i < n1; i += 64) {
        if (!(L.flags[i] & F_ALIVE)) continue;
        float cpx = L.x[i] / 1.0f, cpy = L.y[i] / 1.0f;
        cpx = cpx - 16.0f * 0.5f;
        cpy = cpy - 16.0f * 0.5f;
        float chx = cpx / 16.0f, chy = cpy / 16.0f;
        float x0 = floorf(chx), y0 = floorf(chy), x1 = ceilf(chx), y1 = ceilf(chy);
        int32_t i00 = chunk_index(x0, y0), i10 = chunk_index(x1, y0);
        int32_t i01 = chunk_index(x0, y1), i11 = chunk_index(x1, y1);
        float xi = chx - x0, yi = chy - y0;
        const uint32_t c00 = i00 >= 0 ? L.chunk[i00] : 0u, c10 = i10 >= 0 ? L.chunk[i10] : 0u;
        const uint32_t c01 = i01 >= 0 ? L.chunk[i01] : 0u, c11 = i11 >= 0 ? L.chunk[i11] : 0u;
        float n00 = (float)(c00 >> 16), n10 = (float)(c10 >> 16);
        float n01 = (float)(c01 >> 16), n11 = (float)(c11 >> 16);
        float s00 = (float)(c00 & 0xFFFFu), s10 = (float)(c10 & 0xFFFFu);
        float s01 = (float)(c01 & 0xFFFFu), s11 = (float)(c11 & 0xFFFFu);
        float nx0 = xi * n10 + (1.0f - xi) * n00;
        float nx1 = xi * n11 + (1.0f - xi) * n01;
        float sx0 = xi * s10 + (1.0f - xi) * s00;
        float sx1 = xi * s11 + (1.0f - xi) * s01;
        L.sur0[i] = yi * nx1 + (1.0f - yi) * nx0;
        L.sur1[i] = yi * sx1 + (1.0f - yi) * sx0;
        const int sp = L.species[i] - 1;
        atomicAdd(&L.cnt[sp], 1u);
        atomicAdd(&L.hsum[sp], (uint32_t)L.accum[i]);
    }
    wave_sync();

    // ---- speciesInfoSync (sim.cpp:791-838) ----
    const int A = (int)S.A;
    const uint32_t per_species = S.A / kNumSpecies;
    if (lane < kNumSpecies) {
        const uint32_t count = L.cnt[lane];
        float avg = (float)L.hsum[lane] / (float)count;
        if (count == 0) avg = 0.0f;
        S.sreward[(size_t)w * kNumSpecies + lane] = (float)count / (float)A + avg / 100.0f - 2.0f;
        L.need[lane] = count < per_species ? (int32_t)(per_species - count) : 0;
    }
    wave_sync();
    const int need0 = L.need[0], need1 = L.need[1], need2 = L.need[2], need3 = L.need[3];
    const int total_need = need0 + need1 + need2 + need3;
    // respawn k's draws ctr + 2k, ctr + 2k + 1: from the lanes of dl while they
    // lie within its 64 counters (all lanes shuffle, before the loop diverges)
    const uint32_t ox = (ctr - ctr0) + 2u * lane;
    const uint32_t dx0 = (uint32_t)__shfl((int)dl, (int)(ox & 63u));
    const uint32_t dy0 = (uint32_t)__shfl((int)dl, (int)((ox + 1u) & 63u));
    for (int k = lane; k < total_need; k += 64) {
        int sp = k < need0 ? 1 : (k < need0 + need1 ? 2 : (k < need0 + need1 + need2 ? 3 : 4));
        uint32_t bx = dx0, by = dy0;
        if (k != (int)lane || ox + 1u >= 64u) {
            bx = rng_draw(key, ctr + 2u * (uint32_t)k);
            by = rng_draw(key, ctr + 2u * (uint32_t)k + 1u);
        }
        float x = u01(bx) * kLx;
        float y = u01(by) * kLy;
        const int s = n1 + k;
        if (s < (int)cap) init_slot(L, s, x, y, sp, 100);
    }
    ctr += 2u * (uint32_t)total_need;
    int n2 = n1 + total_need;
    if (n2 > (int)cap) { ovf += (uint32_t)(n2 - (int)cap); n2 = (int)cap; }
    wave_sync();

    // ---- compaction (SortArchetypeNode<Agent, WorldID>, sim.cpp:1129) ----
    int nn = 0;
#pragma unroll
    for (int g = 0; g < kG; ++g) {
        const int b = 64 * g;
        if (b >= n2) break;
        const int i = b + (int)lane;
        const bool alive = i < n2 && (L.flags[i] & F_ALIVE);
        const uint64_t m = ballot64(alive);
        if (alive) {
            const size_t d = base + nn + rank_below(m);
            // write-through (system-scope vector stores): no dirty lines left
            // for the end-of-kernel write-back, which K2 waits for (-1.5 % at
            // 4096 worlds, where the step is that latency chain; +-0 at 65536)
            st_wt(S.x_out + d, L.x[i]);
            st_wt(S.y_out + d, L.y[i]);
            st_wt(S.rw_out + d, L.rw[i]);
            st_wt(S.rz_out + d, L.rz[i]);
            st_wt(S.species_out + d, (int32_t)L.species[i]);
            st_wt(S.health + d, L.accum[i]);
            st_wt(S.obsrow_out + d, i < n0 ? rows[g] : -1);   // newborns: no row
            st_wt(S.sur0 + d, L.sur0[i]);
            st_wt(S.sur1 + d, L.sur1[i]);
            st_wt(S.stats + d, (uint32_t)(L.flags[i] & F_STATS));
            atomicAdd(&L.scount[L.species[i] - 1], 1);
        }
        nn += __popcll(m);
    }
    if (lane < kNumChunks) S.food_out[(size_t)w * kNumChunks + lane] = food_pack(&L.food[lane * kMaxPkg]);
    wave_sync();
    if (lane < kNumSpecies) S.scount[(size_t)w * kNumSpecies + lane] = L.scount[lane];
    if (lane == 0) {
        S.n_out[w] = nn;
        S.ctr[w] = ctr;
        S.cur_food[w] = cur_food;
        if (ovf) {
            S.overflow[w] += ovf;
            // the running total the host checks after each step (MBOTS_W_CAPACITY);
            // a shard ghost's drops belong to the next shard
            if (w < S.Wx) atomicAdd(&S.totals[kTotOverflow], ovf);
        }
    }
    return true;
}

// ---------------------------------------------------------------------------
// K2: species-major row offsets (SortArchetypeNode<Obs, SpeciesObservation>,
// sim.cpp:1147-1149, made deterministic: rows ordered by (species, world,
// slot)).  row_base[w][s] = sum_{s'<s} total[s'] + sum_{w'<w} count[w'][s];
// world_off[w] = sum_{w'<w} n[w'] (agentOffsetForWorld).  One 1024-thread
// block per tile of 1024 worlds; tile sums come from K1's atomics (buffer
// `parity`), the other parity's buffer is cleared for the next step.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int wave_incl_scan(int v)
{
    const int lane = (int)__lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(v, d);
        if (lane >= d) v += y;
    }
    return v;
}

// a wave's `take` lanes appended to list (one returning atomic per wave)
__device__ __forceinline__ void list_append(bool take, int32_t *list, uint32_t *count, uint32_t w)
{
    const uint64_t m = ballot64(take);
    if (m == 0ull) return;
    const int lead = (int)__builtin_ctzll(m);
    uint32_t base = 0;
    if ((int)__lane_id() == lead) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, lead);
    if (take) list[base + rank_below(m)] = (int32_t)w;
}

__global__ __launch_bounds__(1024) void scan_kernel(SimState S, int parity)
{
    __shared__ int32_t s_pre[5], s_tot[5];
    __shared__ int32_t s_wave[16][5];
    __shared__ int32_t s_hist[256];
    __shared__ int32_t s_max[16];
    const int t = threadIdx.x, b = blockIdx.x;
    const int wv = t >> 6, lane = t & 63;
    const uint32_t nent = S.ntiles * kTileBuckets;   // a multiple of 8: 16-B words
    const int32_t *tiles = S.tiles + (size_t)parity * 5 * nent;
    // wave k < 5 sums counter k over the tiles' buckets, four contiguous
    // buckets (of one tile) per 16-B load, 256 per pass
    if (wv < 5) {
        int32_t pre = 0, tot = 0;
        const int4 *tk = reinterpret_cast<const int4 *>(tiles + (size_t)wv * nent);
#pragma unroll 4
        for (uint32_t q = lane; q < nent / 4; q += 64) {
            const int4 v4 = tk[q];
            const int32_t v = v4.x + v4.y + v4.z + v4.w;
            if ((int)(q / (kTileBuckets / 4)) < b) pre += v;
            tot += v;
        }
        pre = wave_incl_scan(pre);
        tot = wave_incl_scan(tot);
        if (lane == 63) { s_pre[wv] = pre; s_tot[wv] = tot; }
    }
    const uint32_t w = (uint32_t)b * kTileWorlds + (uint32_t)t;
    int32_t c[5] = {0, 0, 0, 0, 0};
    if (w < S.W) {
        const int4 sc = reinterpret_cast<const int4 *>(S.scount)[w];
        c[0] = sc.x; c[1] = sc.y; c[2] = sc.z; c[3] = sc.w;
        c[4] = sc.x + sc.y + sc.z + sc.w;
    }
    if (S.mixed) {   // the class lists of this parity (their counts cleared by the last K2)
        const bool bk = w < S.W && k1_needs_class(c[4], S.A);
        const bool bs = w < S.W && c[4] > kSmallCap;
        list_append(bk, S.big_k1 + (size_t)parity * S.W, S.big_cnt + parity * 2, w);
        list_append(bs, S.big_s + (size_t)parity * S.W, S.big_cnt + parity * 2 + 1, w);
        if (b == 0 && t < 2) S.big_cnt[(parity ^ 1) * 2 + t] = 0u;   // the next K2's
    }
    int32_t inc[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) inc[k] = wave_incl_scan(c[k]);
    if (S.track_maxpop) {   // the tile's largest world (kTotMaxPop: mbots_max_population)
        int32_t mx = c[4];
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
        if (lane == 0) s_max[wv] = mx;
    }
    if (lane == 63) {
#pragma unroll
        for (int k = 0; k < 5; ++k) s_wave[wv][k] = inc[k];
    }
    // the sensor's dispatch order (S.sorder, when set): the tile's worlds by
    // descending population, a counting sort on 255 - min(n, 255) (ties in any
    // order: a world's rows do not depend on when it is rendered)
    int key = 0, slot = 0;
    if (S.sorder) {
        if (t < 256) s_hist[t] = 0;
        __syncthreads();
        if (w < S.W) {
            key = 255 - min(c[4], 255);
            slot = atomicAdd(&s_hist[key], 1);
        }
    }
    __syncthreads();
    if (t == 32 && S.totals_host && S.track_maxpop) {   // this tile's largest world into the pinned mirror
        int32_t mx = 0;
        for (int i = 0; i < 16; ++i) mx = max(mx, s_max[i]);
        __hip_atomic_store(S.totals_host + kTotMaxPop + b, (uint32_t)mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
    }
    if (t < 5) {
        int32_t run = 0;
        for (int i = 0; i < 16; ++i) { const int32_t v = s_wave[i][t]; s_wave[i][t] = run; run += v; }
    }
    if (S.sorder && wv == 15) {   // exclusive scan of the 256 bins, four per lane
        const int4 h4 = reinterpret_cast<const int4 *>(s_hist)[lane];
        const int sum = h4.x + h4.y + h4.z + h4.w;
        const int ex = wave_incl_scan(sum) - sum;
        reinterpret_cast<int4 *>(s_hist)[lane] = make_int4(ex, ex + h4.x, ex + h4.x + h4.y, ex + h4.x + h4.y + h4.z);
    }
    __syncthreads();
    if (S.sorder && w < S.W) S.sorder[(size_t)b * kTileWorlds + s_hist[key] + slot] = (int32_t)w;
    if (w < S.W) {
        int32_t ex[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) ex[k] = s_pre[k] + s_wave[wv][k] + inc[k] - c[k];
        int4 rb;
        rb.x = ex[0];
        rb.y = s_tot[0] + ex[1];
        rb.z = s_tot[0] + s_tot[1] + ex[2];
        rb.w = s_tot[0] + s_tot[1] + s_tot[2] + ex[3];
        int32_t off = ex[4];
        if (w >= S.Wx) {   // the shard ghost: its rows after every exported row
            rb.x = s_tot[4];
            rb.y = rb.x + c[0];
            rb.z = rb.y + c[1];
            rb.w = rb.z + c[2];
            off = s_tot[4];
        }
        reinterpret_cast<int4 *>(S.row_base)[w] = rb;
        S.world_off[w] = off;
    }
    if (t < 5 * kTileBuckets)   // this tile's buckets of the other parity, for the next step
        S.tiles[(size_t)(parity ^ 1) * 5 * nent + (size_t)(t / kTileBuckets) * nent + (size_t)b * kTileBuckets +
                t % kTileBuckets] = 0;
    if (b == 0 && t == 0) {
        S.totals[0] = (uint32_t)s_tot[4];
        for (int k = 0; k < 4; ++k) S.totals[1 + k] = (uint32_t)s_tot[k];
        // [5]: every table row, the shard ghost's included (they follow row N):
        // the row moves, the shift and checkpoints carry the ghost's
        // Action / HiddenState like every other row's
        uint32_t rows = (uint32_t)s_tot[4];
        if (S.W > S.Wx) {
            const int4 g = reinterpret_cast<const int4 *>(S.scount)[S.Wx];
            rows += (uint32_t)(g.x + g.y + g.z + g.w);
        }
        S.totals[kTotRows] = rows;
        *S.agent_steps += (unsigned long long)s_tot[4];
        // the host reads the row counts straight from pinned memory once the
        // event after K2 completes (no D2H copy on the step's stream)
        if (S.totals_host) {
#pragma unroll
            for (int k = 0; k < 5; ++k)
                __hip_atomic_store(S.totals_host + k, k ? (uint32_t)s_tot[k - 1] : (uint32_t)s_tot[4],
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(S.totals_host + kTotRows, rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(S.totals_host + kTotOverflow, S.totals[kTotOverflow], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            // make the mirror visible before the dispatch's completion signal,
            // whatever scope the runtime gives that signal's release
            __threadfence_system();
        }
    }
    if (S.epoch) {
        // the fork as a value wait ("Small world counts"): every
        // block writes its outputs back (agent-scope release) before it counts
        // itself done, and the last one stores the step's epoch into the
        // signal word the sensor's queue waits on (its dispatch acquires)
        __syncthreads();
        if (t == 0) {
            __threadfence();
            if (atomicAdd(S.fork_ctr, 1u) == gridDim.x - 1u) {
                atomicExch(S.fork_ctr, 0u);
                __hip_atomic_store(S.sig_fork, S.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// init-only: tile sums straight from scount (no K1 ran yet)
__global__ __launch_bounds__(1024) void tile_sum_kernel(SimState S, int parity)
{
    __shared__ int32_t s_wave[16][5];
    const int t = threadIdx.x, b = blockIdx.x;
    const uint32_t w = (uint32_t)b * kTileWorlds + (uint32_t)t;
    int32_t c[5] = {0, 0, 0, 0, 0};
    if (w < S.Wx) {
        const int4 sc = reinterpret_cast<const int4 *>(S.scount)[w];
        c[0] = sc.x; c[1] = sc.y; c[2] = sc.z; c[3] = sc.w;
        c[4] = sc.x + sc.y + sc.z + sc.w;
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const int32_t v = wave_incl_scan(c[k]);
        if ((t & 63) == 63) s_wave[t >> 6][k] = v;
    }
    __syncthreads();
    if (t < 5 * kTileBuckets) {   // the tile's sum in bucket 0, the other buckets and parity cleared
        const size_t nent = (size_t)S.ntiles * kTileBuckets;
        const int k = t / kTileBuckets, bk = t % kTileBuckets;
        int32_t run = 0;
        if (bk == 0)
            for (int i = 0; i < 16; ++i) run += s_wave[i][k];
        const size_t e = (size_t)k * nent + (size_t)b * kTileBuckets + bk;
        S.tiles[(size_t)parity * 5 * nent + e] = run;
        S.tiles[(size_t)(parity ^ 1) * 5 * nent + e] = 0;
    }
}

// mixed classes after a checkpoint load: the K1 class list of `slot` from S.n
// (its count zeroed by the host beforehand)
__global__ __launch_bounds__(256) void build_lists_kernel(SimState S, int slot)
{
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    const bool bk = w < S.W && k1_needs_class(S.n[w], S.A);
    list_append(bk, S.big_k1 + (size_t)slot * S.W, S.big_cnt + slot * 2, w);
}

// ---------------------------------------------------------------------------
// K3a: export rows, one wave per world -- updateObservations (sim.cpp:687-717)
// into the world's species-major rows of the next table and rewardSystem
// setting 8 (sim.cpp:840-983; faithful rewards[speciesID] off-by-one unless
// fixed).  The old row of each agent (the obs row travels through the species
// sort with its Action / HiddenState / Prev* columns and the prev sensor,
// updateSensorOutputIdx sim.cpp:736-789) is recorded in src_of[new_row] for
// the K4 move stream.
// ---------------------------------------------------------------------------
template <bool kInit>
__device__ __forceinline__ void export_world(const SimState &S, const ObsTable &nxt, uint32_t w, uint32_t lane)
{
    constexpr bool init = kInit;
    const size_t base = (size_t)w * S.cap;
    const int n = uniform(S.n[w]);
    // slot `lane`'s species loaded beside the count (rows past n are stale
    // and never used)
    const int32_t sp0 = (int)lane < (int)S.cap ? S.species[base + lane] : 0;
    const int4 rb = reinterpret_cast<const int4 *>(S.row_base)[w];
    const float4 rew = reinterpret_cast<const float4 *>(S.sreward)[w];
    const bool fixed = (S.flags & kFlagRewardFixed) != 0;
    // faithful B.3: rewards[4] reads the next SpeciesInfo row's rewards[0]
    const float next_r0 = (w + 1 < S.W) ? S.sreward[(size_t)(w + 1) * kNumSpecies] : 0.0f;
    int carry0 = 0, carry1 = 0, carry2 = 0, carry3 = 0;
    for (int b = 0; b < n; b += 64) {
        const int i = b + (int)lane;
        const bool active = i < n;
        const int32_t sp = active ? (b == 0 ? sp0 : S.species[base + i]) : 0;
        // every column of the slot loaded with its species (one memory round
        // trip per 64 slots: the wave holds its slot for less time beside the
        // sensor)
        float x = 0.0f, y = 0.0f, s0 = 0.0f, s1 = 0.0f;
        int32_t h = 0, old = -1;
        uint32_t st = 0u;
        if (active) {
            x = S.x[base + i];
            y = S.y[base + i];
            h = S.health[base + i];
            if (!init) {
                s0 = S.sur0[base + i];
                s1 = S.sur1[base + i];
                st = S.stats[base + i];
            }
            old = S.obsrow_out[base + i];
        }
        const uint64_t m1 = ballot64(sp == 1), m2 = ballot64(sp == 2);
        const uint64_t m3 = ballot64(sp == 3), m4 = ballot64(sp == 4);
        int32_t row = 0;
        if (sp == 1) row = rb.x + carry0 + (int32_t)rank_below(m1);
        else if (sp == 2) row = rb.y + carry1 + (int32_t)rank_below(m2);
        else if (sp == 3) row = rb.z + carry2 + (int32_t)rank_below(m3);
        else if (sp == 4) row = rb.w + carry3 + (int32_t)rank_below(m4);
        carry0 += __popcll(m1); carry1 += __popcll(m2);
        carry2 += __popcll(m3); carry3 += __popcll(m4);
        if (!active) continue;
        const size_t r = (size_t)row;
        // old row: K1's obsrow_out (the sensor reads it beside this kernel);
        // the new row goes to obsrow, which the next K1 reads
        S.src_of[r] = old;
        S.obsrow[base + i] = row;
        constexpr bool nt = (MB_NT & 4) != 0;
        st_stream(nxt.species + r, sp, nt);
        st_stream(reinterpret_cast<float2 *>(nxt.pos) + r, make_float2(x, y), nt);
        st_stream(nxt.health + r, h, nt);
        st_stream(reinterpret_cast<float2 *>(nxt.sur) + r, make_float2(s0, s1), nt);
        const int4 stv = make_int4((int)(st & 1u), (int)((st >> 1) & 1u), (int)((st >> 2) & 1u),
                                   (int)((st >> 3) & 1u));
        st_stream(reinterpret_cast<int4 *>(nxt.stats) + r, stv, nt);
        float rv = 0.0f;
        if (!init) {
            float sr;
            if (fixed) sr = sp == 1 ? rew.x : sp == 2 ? rew.y : sp == 3 ? rew.z : rew.w;
            else sr = sp == 1 ? rew.y : sp == 2 ? rew.z : sp == 3 ? rew.w : next_r0;
            rv = sr + (float)h / 100.0f - 0.5f;
            if (stv.z) rv += 10.0f;
            if (stv.w) rv += 10.0f;
            if (stv.y) rv += 15.0f;
        }
        st_stream(nxt.reward + r, rv, nt);
    }
}

#ifndef MB_EXPORT_WPW
#define MB_EXPORT_WPW 1   // worlds per K3a wave (straight-line: each its own unrolled body)
#endif
template <bool kInit>
__global__ __launch_bounds__(256) void export_rows_kernel(SimState S, ObsTable nxt)
{
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    constexpr int kWpw = kInit ? 1 : MB_EXPORT_WPW;
#pragma unroll
    for (int k = 0; k < kWpw; ++k) {
        const uint32_t w = uniform((blockIdx.x * kWpw + k) * kWorldsPerBlock + wv);
        if (w < S.W) export_world<kInit>(S, nxt, w, lane);
    }
}

// ---------------------------------------------------------------------------
// K4: row move.  For every new row r with old row o = src_of[r] (-1: a newborn
// or respawned agent, zero-filled -- SURVEY B.13) copy the columns that travel
// with the observation row: Action, HiddenState, every Prev* column and the
// prev sensor (semantic, and depth when it is not aliased).  One grid-stride
// stream of 8/16-byte items over the new rows, so stores are fully coalesced
// and the gathered loads are contiguous wherever old rows are (most agents
// keep their species and relative order).
//
// A step launches only the prev-sensor part; the other parts are deferred
// (DESIGN.md "Deferred Prev moves") and run from the host's materialisation
// points, or fused with the shift (shift_move_kernel: Action / HiddenState into
// the Prev columns, the current ones left as their views).
// ---------------------------------------------------------------------------
struct MoveSeg {
    void *dst;
    const void *src;
    uint32_t width;   // bytes per item: 4, 8 or 16
    uint32_t ipr;     // items per row
    uint32_t xform;   // 1: the source is current AgentStats, apply the shift's
                      // prevStats.hitEnemy = stats.hitFriendly (sim.cpp:1034)
};
constexpr int kMaxMoveSegs = 13;
struct MoveArgs {
    MoveSeg seg[kMaxMoveSegs];
    int nseg;
};

template <typename T>
__device__ __forceinline__ void move_item(const MoveSeg &sg, uint32_t idx, int32_t o, uint32_t part, bool nt)
{
    T v{};
    if (o >= 0) v = ld_stream(reinterpret_cast<const T *>(sg.src) + (size_t)o * sg.ipr + part, (MB_NT & 32) != 0);
    st_stream(reinterpret_cast<T *>(sg.dst) + idx, v, nt);
}

__device__ __forceinline__ void move_rows(const uint32_t *totals, const int32_t *src_of,
                                          const MoveArgs &args)
{
    const uint32_t N = totals[kTotRows];   // the shard ghost's rows included
    const MoveSeg &sg = args.seg[blockIdx.y];
    const uint32_t items = N * sg.ipr;
    const uint32_t stride = gridDim.x * blockDim.x;
    const bool nt = (MB_NT & 1) != 0;
    for (uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x; idx < items; idx += stride) {
        uint32_t r = idx, part = 0;
        if (sg.ipr == 2) { r = idx >> 1; part = idx & 1u; }
        else if (sg.ipr == 3) { r = idx / 3u; part = idx - r * 3u; }
        else if (sg.ipr == 4) { r = idx >> 2; part = idx & 3u; }
        const int32_t o = src_of[r];
        if (sg.width == 16 && sg.xform) {
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (o >= 0) v = ld_stream(reinterpret_cast<const uint4 *>(sg.src) + o, (MB_NT & 32) != 0);
            v.y = v.x;
            st_stream(reinterpret_cast<uint4 *>(sg.dst) + idx, v, nt);
        } else if (sg.width == 16) move_item<uint4>(sg, idx, o, part, nt);
        else if (sg.width == 8) move_item<uint2>(sg, idx, o, part, nt);
        else move_item<uint32_t>(sg, idx, o, part, nt);
    }
}

__global__ __launch_bounds__(256) void move_kernel(const uint32_t *totals, const int32_t *src_of,
                                                   MoveArgs args)
{
    move_rows(totals, src_of, args);
}

// one segment of the fused shift, kU items per thread per pass: the kU
// src_of loads, then the kU gathered loads, then the stores (each instruction
// still coalesced over the wave: items idx + k * stride)
template <typename T, int kIpr>
__device__ __forceinline__ void gather_seg(const MoveSeg &sg, uint32_t N, const int32_t *src_of)
{
    constexpr int kU = MB_SHIFT_UNROLL;
    const uint32_t items = N * kIpr;
    const uint32_t stride = gridDim.x * blockDim.x;
    const bool ntl = (MB_NT & 32) != 0, nts = (MB_NT & 1) != 0;
    for (uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < items; i0 += kU * stride) {
        int32_t o[kU];
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            const uint32_t idx = i0 + k * stride;
            o[k] = idx < items ? src_of[idx / kIpr] : -2;
        }
        T v[kU];
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            const uint32_t idx = i0 + k * stride;
            v[k] = T{};
            if (o[k] >= 0) v[k] = ld_stream(reinterpret_cast<const T *>(sg.src) + (size_t)o[k] * kIpr + idx % kIpr, ntl);
        }
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            const uint32_t idx = i0 + k * stride;
            if (o[k] != -2) st_stream(reinterpret_cast<T *>(sg.dst) + idx, v[k], nts);
        }
    }
}

// the fused shift (DESIGN.md "Deferred Prev moves"): Action / HiddenState
// gathered from the other half into the Prev columns (the current ones are
// left as their views: DESIGN.md "Aliased current Action / HiddenState")
__global__ __launch_bounds__(256) void shift_move_kernel(const uint32_t *totals, const int32_t *src_of,
                                                         MoveArgs args)
{
    const MoveSeg &sg = args.seg[blockIdx.y];
    const uint32_t N = totals[kTotRows];
    if (sg.width == 8 && sg.ipr == 3) gather_seg<uint2, 3>(sg, N, src_of);
    else if (sg.width == 16 && sg.ipr == 4) gather_seg<uint4, 4>(sg, N, src_of);
    else if (sg.width == 16 && sg.ipr == 2) gather_seg<uint4, 2>(sg, N, src_of);
    else move_rows(totals, src_of, args);
}

// ---------------------------------------------------------------------------
// K3b sensor: 32-pixel raycast (24 forward + 8 backward) plus the finder ray
// (Madrona RenderingSystem, sim.cpp:1183-1188).  Build spec:
// agents are discs of radius R = 0.92, food packages rotated +-1 squares
// (FoodBox, mbots_ray.hpp); in an agent's frame (f along heading h, l along
// r = (hy, -hx)) ray h + u r meets a disc iff
//     q(u) = (A u - 2 l f) u + C <= 0,   A = f^2 - R^2,  C = l^2 - R^2,
// and sees it iff it leaves it beyond the near sphere (1.1 from the camera:
// the near point NearPt inside the disc, or the chord's midpoint beyond it);
// view depth z = f - R (>= 0, 14-bit mantissa).  Per ray the lexicographic
// minimum of (z, order) over objects (food 1 + k, agents 64 + slot) is seen
// iff it beats the wall, placed by where the ray's near point lies (inner
// rectangle: the exit from it; a wall box: the wall at the near point; beyond
// the walls: no wall, semantic -1).
//
// One wave per world, agents in chunks of kKeyAgents; per chunk:
//  P1  all (agent, object) pairs, one per lane: f, l, the wedge test
//      |l| <= |f| + sqrt(2) R' + 0.05 (necessary for any pixel, |u| < 1) and
//      for far pairs the angular cull; survivors ballot-compacted into a queue;
//  P2  per survivor: far pairs (beyond the near sphere's reach) get their hit
//      interval (disc roots / square corner slopes): the edge pixels and the
//      finder run the exact predicate, interior pixels are filled, each by
//      ds_min_u32 of the 32-bit key (z with its low 9 mantissa bits replaced
//      by the object order); near pairs go to a wide list;
//  W   wide pairs: two per wave, one lane per ray, every ray exact;
//  out per (agent, ray): key vs wall -> semantic / depth bytes; finder slot
//      (every ray as inner first, then a fix-up for the agents near walls).
// The exact predicate and depths use the same float expressions as
// oracle/mbots_oracle.c; culling only skips rays it proves cannot pass.
// ---------------------------------------------------------------------------
#ifndef MB_KEY_AGENTS
#define MB_KEY_AGENTS 8
#endif
constexpr int kKeyAgents = MB_KEY_AGENTS;     // agents per chunk (key rows)
constexpr int kKeyStride = 36;                // key row: 32 pixels, finder, pad (16-B rows)
constexpr int kQueueCap = 128;                // P1 survivors (flushed at >= 64)
// P1's wedge |l| <= |f| + R sqrt(2) + 0.05 is necessary for a radius-R disc
// (a food square: its circumscribed circle, R = 1.42) on a ray |u| < 1
constexpr float kUEps = 2e-3f;                // root-interval margin in u
// food squares lie inside their circumscribed circle, radius sqrt 2 (1.42 with
// margin): the wedge |l| <= |f| + sqrt(2) 1.42; candidate pixels from the
// corner slopes when |f| > kFoodFar (the square then lies wholly beyond the
// near sphere, on one side of the camera plane), every ray exactly (the wide
// list) otherwise; discs likewise beyond kCircleFar
// Far pairs need no near-sphere test: a disc with |f| > 1.5 is met only by
// rays whose chord midpoint lies >= sqrt(1.5^2 - 0.92^2) = 1.18 > 1.1 along
// them (so they leave it past the near sphere, and a near point inside it is
// on such a ray); every point of a square with |f| > 2.55 lies >= 2.55 -
// 1.4142 = 1.136 > 1.1 ahead.  The r2 kernel's split stands.
constexpr float kFoodFar = 2.55f;
constexpr float kCircleFar = 1.5f;
constexpr float kFarCull = 5.0f;               // P1 angular cull from this |f| on
constexpr float kInsideNear2 = 0.17f * 0.17f;  // disc centres this close are inside the near sphere
#ifndef MB_NEAR_CULL
#define MB_NEAR_CULL 1
#endif
#ifndef MB_SPLIT_FLUSH
#define MB_SPLIT_FLUSH 16   // food survivors flushed alone from this many on (24: +0.2 %, 40: +0.3 %, never: +1 %)
#endif

template <int kCap>
struct SensorLDS {
    // positions: food, then agents, then (kCap <= 128) 64 NaN sentinels that P1
    // reads past nobj unchecked (the larger classes keep their bounds checks:
    // 2 KB more per block would cost the 256-slot class a block per CU)
    float2 obj[kMaxFood + kCap + (kCap <= 128 ? 64 : 0)];
    float2 frot[kMaxFood];                    // food squares' (cos, sin)
    float2 hd[kCap];                          // agent headings
    int8_t sem_of[kOrderAgent + kCap];        // semantic byte by object order: food 6,
                                              // agent 64 + slot its species
    // 32-bit keys up to 256 slots (orders < 320 fit the low 9 bits), 64-bit
    // above (mbots_ray.hpp Key<>)
    using key_t = std::conditional_t<(kCap <= 256), uint32_t, uint64_t>;
    alignas(16) key_t key[kKeyAgents * kKeyStride];
    uint32_t qcode[kQueueCap + 1];            // P1 survivors: agent | object << 11 (+ a
                                              // sink slot for the branch-free write); a
                                              // survivor batch's wide pairs are compacted
                                              // into its own range
};

// per ray k (32 pixels, the finder at 32): offset u and near point NearPt
// {c, s, e} (near_pt), one table per block (every wave writes
// the same bits before reading it: no barrier needed)
struct RayTab {
    alignas(16) float u[36];
    alignas(16) float c[36];
    alignas(16) float s[36];
    alignas(16) float e[36];
};

// pinhole offsets u = (2k + 1) / 24 - 1 forward, (2k' + 1) / 8 - 1 backward,
// as the oracle's one rounding (2k - 23) (1/24) / exact (2k' - 7) / 8;
// computed in registers (a table in constant memory cost every wave a memory
// round trip before its first load)
__host__ __device__ constexpr float u_of(int k)
{
    return k < 24 ? (float)(2 * k - 23) * (1.0f / 24.0f) : (float)(2 * (k - 24) - 7) * 0.125f;
}

// wave-wide compare masks (VOPC results as 64-bit lane masks; every lane
// active) and a select by such a mask (v_cndmask on the SGPR pair)
#ifndef MB_P1_MASKS
#define MB_P1_MASKS 1
#endif
constexpr int kCmpOGT = 2, kCmpOLT = 4, kCmpOLE = 5, kCmpNE = 33, kCmpSLT = 40;
template <int kPred>
__device__ __forceinline__ uint64_t fcmp_mask(float a, float b)
{
    return __builtin_amdgcn_fcmpf(a, b, kPred);
}
template <int kPred>
__device__ __forceinline__ uint64_t icmp_mask(int a, int b)
{
    return __builtin_amdgcn_uicmp((unsigned)a, (unsigned)b, kPred);
}
__device__ __forceinline__ int select_by_mask(uint64_t m, int if_set, int if_clear)
{
    int r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(m));
    return r;
}

// (f, l) of object j in agent i's frame; order of the object (food at
// [0, nf), agents from na = nf rounded up to 8; the gap holds NaN, which no
// queued pair references, so j < na tells food from agents)
template <class LDS>
__device__ __forceinline__ void pair_fl(const LDS &L, int na, int i, int j, float &f,
                                        float &l, uint32_t &order)
{
    const float2 a = L.obj[na + i];
    const float2 h = L.hd[i];
    const float2 p = L.obj[j];
    order = j < na ? kOrderFood + (uint32_t)j : kOrderAgent + (uint32_t)(j - na);
    const float vx = p.x - a.x, vy = p.y - a.y;
    f = vx * h.x + vy * h.y;   // along the heading
    l = vx * h.y - vy * h.x;   // along r = (hy, -hx)
}

// W: wide pairs qcode[q0, q0 + cnt), two per wave (32 lanes each: rays 0..31,
// lane 0 of each half also takes the finder ray)
// (MB_COUNT = k: counting-probe builds, scripts/probe_counts.py; event k's
// wave-uniform count summed into the overflow column)
#ifdef MB_COUNT
#define MB_CNT(k, v) do { if (MB_COUNT == (k)) mbc += (uint32_t)(v); } while (0)
#else
#define MB_CNT(k, v) do { } while (0)
#endif

template <class LDS>
__device__ __forceinline__ void run_wide(LDS &L, const RayTab &R, int na, int a0, int q0, int cnt, uint32_t &mbc)
{
    MB_CNT(6, (cnt + 1) / 2);
    using K = typename LDS::key_t;
    const int lane = (int)__lane_id();
    // ray k's offset and near point (the near sphere): loop invariant
    const int k = lane & 31;
    const float uk = R.u[k];
    const NearPt np{R.c[k], R.s[k], R.e[k]}, fnp{R.c[kSensor], R.s[kSensor], R.e[kSensor]};
    // a pair left alone (the common case: most batches hold one near pair) takes
    // 33 lanes, ray 32 being the finder (u = 0 and the finder's near point in
    // the ray table: the same predicate), so its round evaluates one test per
    // lane instead of a pixel's and the finder's
    const int cnt2 = cnt & ~1;
    if (cnt2 < cnt) {
        const int ks = (int)lane;
        if (ks <= kSensor) {
            const uint32_t code = L.qcode[q0 + cnt2];
            const int ic = (int)(code & 0x1Fu), j = (int)(code >> 11);
            float f, l;
            uint32_t order;
            pair_fl(L, na, a0 + ic, j, f, l, order);
            const float us = R.u[ks];
            const NearPt nps{R.c[ks], R.s[ks], R.e[ks]};
            const bool fw = (ks < 24) | (ks == kSensor);
            K kv;
            if (j < na) {
                const FoodBox b = box_setup(f, l, L.frot[j], L.hd[a0 + ic]);
                kv = box_hit(b, us, fw, nps.c) ? Key<K>::make(box_z(b, fw), order) : Key<K>::none;
            } else {
                kv = pixel_key<K>(f, l, us, nps, fw, order);
            }
            if (kv != Key<K>::none) atomicMin(&L.key[ic * kKeyStride + ks], kv);
        }
    }
    for (int e0 = 0; e0 < cnt2; e0 += 2) {
        const int e = e0 + (lane >> 5);
        if (e < cnt) {
            const uint32_t code = L.qcode[q0 + e];
            const int ic = (int)(code & 0x1Fu), j = (int)(code >> 11);
            float f, l;
            uint32_t order;
            pair_fl(L, na, a0 + ic, j, f, l, order);
            K *kr = L.key + ic * kKeyStride;
            K kv, kf;
            if (j < na) {   // food square: every ray exactly
                const FoodBox b = box_setup(f, l, L.frot[j], L.hd[a0 + ic]);
                kv = box_hit(b, uk, k < 24, np.c) ? Key<K>::make(box_z(b, k < 24), order) : Key<K>::none;
                kf = box_hit(b, 0.0f, true, fnp.c) ? Key<K>::make(box_z(b, true), order) : Key<K>::none;
            } else {
                kv = pixel_key<K>(f, l, uk, np, k < 24, order);
                kf = finder_key<K>(f, l, order);
            }
            if (kv != Key<K>::none) atomicMin(&kr[k], kv);
            if ((k == 0) & (kf != Key<K>::none)) atomicMin(&kr[kSensor], kf);
        }
    }
}

// P2: survivors [q0, q0 + cnt): the approximate hit interval bounds the
// candidate pixels; the edge pixels and the finder get the exact test inline,
// near pairs go to the wide list
template <class LDS>
__device__ __forceinline__ void run_survivors(LDS &L, const RayTab &R, int na, int a0, int q0, int cnt, uint32_t &mbc)
{
    MB_CNT(3, 1);
    MB_CNT(4, cnt);
    using K = typename LDS::key_t;
#ifdef MB_COUNT
    int mb_t = 0;
    bool mb_food = false, mb_disc = false;
#endif
    const int lane = (int)__lane_id();
    bool wide = false;
    uint32_t code = 0;
    float f = 0.0f, l = 0.0f;
    if (lane < cnt) {
        code = L.qcode[q0 + lane];
        const int ic = (int)(code & 0x1Fu), j = (int)(code >> 11);
        uint32_t order;
        pair_fl(L, na, a0 + ic, j, f, l, order);
        const bool food = j < na;
        const float r2 = f * f + l * l;
        if (fabsf(f) <= (food ? kFoodFar : kCircleFar)) {
            // a disc whose centre lies within 0.17 of the camera is wholly inside
            // the near sphere (0.17 + R = 1.09 < 1.1): no ray leaves it beyond
            // 1.1, so no ray sees it -- the exact predicate's near point then
            // lies >= 0.93 > R from the centre and the chord's midpoint < 0.17
            // along the ray, margins of 1e-2 against float errors of 1e-6.
            // Such pairs (a newborn on its parent, sim.cpp:561-564) skip the
            // wide round.
            wide = food | (r2 >= kInsideNear2) | !MB_NEAR_CULL;
        } else {
            // A far pair: the object lies on one side of the camera plane and
            // the near sphere clips none of its rays (circle: |f| > 1.5;
            // square: |f| > 2.55, so every corner has |X| >= 1.13; see
            // kFoodFar).  Its hit interval in u, approximately: the circle's
            // roots (lf -+ R sqrt(r^2 - R^2)) / (f^2 - R^2), or the square's
            // extreme corner slopes Y / X.
            const bool fwd = f > 0.0f;
            const float sc = fwd ? 12.0f : 4.0f;
            float ulo, uhi;
            FoodBox b{};
            if (food) {
                b = box_setup(f, l, L.frot[j], L.hd[a0 + ic]);
                // corner offsets +-(p - q, p + q), +-(p + q, q - p)
                const float ax = b.p - b.q, ay = b.p + b.q;
                const float s0 = (l + ay) * __builtin_amdgcn_rcpf(f + ax);
                const float s1 = (l - ay) * __builtin_amdgcn_rcpf(f - ax);
                const float s2 = (l - ax) * __builtin_amdgcn_rcpf(f + ay);
                const float s3 = (l + ax) * __builtin_amdgcn_rcpf(f - ay);
                ulo = fminf(fminf(s0, s1), fminf(s2, s3));
                uhi = fmaxf(fmaxf(s0, s1), fmaxf(s2, s3));
            } else {
                const float sq = __builtin_amdgcn_sqrtf(kAgentR2 * (r2 - kAgentR2));
                const float ia = __builtin_amdgcn_rcpf(f * f - kAgentR2);
                const float lf = l * f;
                ulo = (lf - sq) * ia;
                uhi = (lf + sq) * ia;
            }
            // widened by kUEps, in pixel coordinates s = (u + 1) sc - 0.5
            // (pixel k at s = k; FMA: an approximation bounded by the margin)
            const float lo = __builtin_fmaf(ulo, sc, fwd ? 12.0f * (1.0f - kUEps) - 0.5f : 4.0f * (1.0f - kUEps) - 0.5f);
            const float hi = __builtin_fmaf(uhi, sc, fwd ? 12.0f * (1.0f + kUEps) - 0.5f : 4.0f * (1.0f + kUEps) - 0.5f);
            const int kmax = fwd ? 23 : 7;
            int k0 = max((int)ceilf(lo), 0);
            const int k1 = min((int)floorf(hi), kmax);
            const int c = k1 - k0 + 1;
            k0 += fwd ? 0 : 24;
            K *kr = L.key + ic * kKeyStride;
            // The two edge pixels of [k0, k0 + c) get the exact predicate.
            // Interior pixels lie >= one pixel pitch minus 2 kUEps (>= 0.08 in
            // u) inside the true interval, where the approximate bounds are off
            // by ~1e-6: for a circle the float q(u) is then off by < 1e-4 of a
            // value <= -0.08; for a square every corner's S = Y - u X is
            // >= 1.13 x 0.08 from 0 (|X| >= 1.13), against a float error of the
            // line test < 1e-4.  They are hits carrying the object's key (a far
            // object lies beyond the near sphere: nothing of it is clipped).
            const int kl = k0 + max(c - 1, 0);
            const float ua = R.u[k0 & 31], ub = R.u[kl & 31];
            bool ha, hb, hf;
            K kin;
            if (food) {   // a far square: box_hit is the line test on its side
                ha = box_line_hit(b, ua);
                hb = box_line_hit(b, ub);
                hf = fwd & box_finder_hit(b);
                kin = Key<K>::make(box_z(b, fwd), order);
            } else {
                ha = far_pixel_hit(f, l, ua, fwd);
                hb = far_pixel_hit(f, l, ub, fwd);
                // finder ray (u = 0) of a far pair: q(0) = l^2 - R^2 <= 0 and f > 0
                hf = (l * l - kAgentR2 <= 0.0f) & fwd;
                kin = Key<K>::make(fwd ? f - kAgentR : -f - kAgentR, order);
            }
            if ((c > 0) & ha) atomicMin(&kr[k0], kin);
            if ((c > 1) & hb) atomicMin(&kr[kl], kin);
            if (hf) atomicMin(&kr[kSensor], kin);
            for (int k = k0 + 1; k < kl; ++k) atomicMin(&kr[k], kin);
#ifdef MB_COUNT
            mb_t = max(kl - k0 - 1, 0);
            mb_food = food;
            mb_disc = !food;
#endif
        }
    }
    // every lane read its code above: the wide ones compact in place
    const uint64_t wm = ballot64(wide);
    if (wide) L.qcode[q0 + (int)rank_below(wm)] = code;
    const int nw = __popcll(wm);
    MB_CNT(5, nw);
#ifdef MB_COUNT
    for (int o = 32; o > 0; o >>= 1) mb_t = max(mb_t, __shfl_xor(mb_t, o));
    MB_CNT(7, mb_t);
    MB_CNT(9, __popcll(ballot64(mb_food)));
    {
        // batches running the far-square path / the far-disc path / both
        const uint64_t fm = ballot64(mb_food), dm = ballot64(mb_disc);
        MB_CNT(10, fm != 0ull);
        MB_CNT(11, dm != 0ull);
        MB_CNT(12, (fm != 0ull) & (dm != 0ull));
    }
#endif
#ifndef MB_SKIP_WIDE   // (instruction-count probes only: MB_SKIP_* builds give wrong rows)
    if (nw > 0) {
        wave_sync();
        run_wide(L, R, na, a0, q0, nw, mbc);
        wave_sync();
    }
#endif
}

// the world's staged inputs, loaded as one batch of independent loads
struct SensorPrefetch {
    uint64_t food;             // lane < 48: packed chunk record
    uint32_t rot0;             // lane < 48: the rotation of the chunk's package 0 (where
                               // addFood places a chunk's first package; the others are
                               // read after the record's live mask, only where live)
    float x, y, rw, rz;        // lane < min(n, 64): agent slot `lane`
    int32_t sp;
    int n;
    int4 rb;                   // row_base[w]
};

__device__ __forceinline__ void sensor_prefetch(const SimState &S, uint32_t w, uint32_t lane,
                                                SensorPrefetch &p)
{
    p.n = uniform(S.n[w]);
    p.rb = reinterpret_cast<const int4 *>(S.row_base)[w];
    p.food = lane < kNumChunks ? S.food[(size_t)w * kNumChunks + lane] : 0ull;
    p.rot0 = lane < kNumChunks ? S.food_rot[(size_t)w * kNumPkg + lane] : 0u;
    // slots [0, min(cap, 64)), loaded without waiting for n (rows past n are
    // stale and never used; the fetch is by 128-B lines, so a 33-agent world
    // reads two per column either way: loading only slots < n measured no
    // fewer FETCH_SIZE bytes and +0.5 % step)
    const auto load = [&](uint32_t s) {
        const size_t i = (size_t)w * S.cap + s;
        p.x = S.x[i];
        p.y = S.y[i];
        p.rw = S.rw[i];
        p.rz = S.rz[i];
        p.sp = S.species[i];
    };
    if (lane < S.cap) load(lane);
}

// one wave per world, 4 worlds per block
#ifndef MB_SENSOR_WPB
#define MB_SENSOR_WPB 4
#endif
constexpr int kSensorWorlds = MB_SENSOR_WPB;   // worlds (waves) per sensor block
#ifndef MB_SENSOR_SPLIT_MAX
#define MB_SENSOR_SPLIT_MAX 4096   // world counts up to this use the split sensor
#endif
#ifndef MB_SENSOR_SPLIT
#define MB_SENSOR_SPLIT 4          // waves per world of the split sensor
#endif
#ifndef MB_SENSOR_SPLIT_WAVES
#define MB_SENSOR_SPLIT_WAVES MB_SENSOR_WPB   // waves per block of the split sensor
#endif
// the launch bounds' minimum waves per SIMD: 8 (<= 64 VGPRs) for the 128-slot
// class, 4 for the 256-slot one, 2 for the 512 / 1024 classes, 1 for 2048 / 4096 (LDS-bound there)
__host__ __device__ constexpr int sensor_min_waves(int cap) { return cap <= 128 ? 8 : cap <= 256 ? 4 : cap <= 1024 ? 2 : 1; }
// kDepth: fix_depth_alias (a depth byte per pixel besides the semantic one).
// kSplit: kSplit waves share one world, each taking every kSplit-th key chunk
// (each stages its own LDS image of the world).  Used at small world counts
// (<= 4096), where one wave per world leaves SIMDs idle and the step waits on
// the latency of one world's serial chunk loop (4 waves per world: step -8 % at
// 4096 worlds; 2 waves: -5 %; no gain at 8192).
template <bool kDepth, int kSplit, int kCap, bool kSkipBig = false>
__device__ __forceinline__ void sensor_world(const SimState &S, const ObsTable &nxt, SensorLDS<kCap> &L,
                                             RayTab &R, uint32_t w, uint32_t wv, uint32_t lane)
{
    constexpr int kG = kCap / 64;   // 64-slot groups
    constexpr int kChunkStep = kKeyAgents * kSplit;
    const int kChunk0 = (int)(wv % kSplit) * kKeyAgents;
    using K = typename SensorLDS<kCap>::key_t;
    constexpr bool depth = kDepth;
    SensorPrefetch pf;
    sensor_prefetch(S, w, lane, pf);
    // (mixed classes: a world past the small class is the class kernel's)
    if (kSkipBig && pf.n > kCap) return;
    // ray `lane`'s u and near point (the finder at 32: u = 0, {1.1, 0, 1.1}),
    // host-computed (upload_ray_table), loaded with the prefetch batch and
    // stored to the block's table after the staging below
    const float4 ray = lane <= (uint32_t)kSensor ? S.raytab[lane] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    {
    const size_t base = (size_t)w * S.cap;
    const SensorPrefetch cur = pf;
    const int n = cur.n;

    // ---- live food packages in (chunk, package) order -> objects [0, nf) ----
    uint32_t rot[kMaxPkg];
    {
        const uint32_t live = (uint32_t)(cur.food >> 40) & 31u;
        rot[0] = cur.rot0;
#pragma unroll
        for (int k = 1; k < kMaxPkg; ++k)
            rot[k] = (live >> k) & 1u ? S.food_rot[(size_t)w * kNumPkg + k * kNumChunks + lane] : 0u;
    }
    const int nf = stage_food(cur.food, rot, lane, L.obj, L.frot);
    // ---- agents -> objects [na, na + n), na = nf rounded up to 8: P1's
    // 8-object iterations are then all food or all agents (full chunks), so a
    // chunk's food survivors can be flushed as their own batch (below); the
    // gap holds NaN (every P1 test fails) ----
    const int na = (nf + 7) & ~7;
    if ((int)lane >= nf && (int)lane < na) L.obj[lane] = make_float2(__builtin_nanf(""), __builtin_nanf(""));
    L.sem_of[lane] = 6;   // orders < 64: wall 0 (unused), food 1 + k
    if ((int)lane < n) {
        float hx, hy;
        heading(cur.rw, cur.rz, hx, hy);
        L.obj[na + lane] = make_float2(cur.x, cur.y);
        L.hd[lane] = make_float2(hx, hy);
        L.sem_of[kOrderAgent + lane] = (int8_t)cur.sp;
    }
    // export rows (K3a's rule, computed here so the sensor need not wait for
    // K3a): row_base[w][species] + rank among the world's slots of that
    // species.  They stay in registers: rows[g] of lane s is slot 64 g + s.
    const int4 rb = cur.rb;
    int rows[kG];
    int c1 = 0, c2 = 0, c3 = 0, c4 = 0;
#pragma unroll
    for (int g = 0; g < kG; ++g) {
        rows[g] = 0;
        if (g > 0 && 64 * g >= n) continue;
        const int i = 64 * g + (int)lane;
        int sp = 0;
        if (g == 0) {
            sp = (int)lane < n ? cur.sp : 0;
        } else if (i < n) {   // slots past 64: loaded here
            float hx, hy;
            heading(S.rw[base + i], S.rz[base + i], hx, hy);
            L.obj[na + i] = make_float2(S.x[base + i], S.y[base + i]);
            L.hd[i] = make_float2(hx, hy);
            sp = S.species[base + i];
            L.sem_of[kOrderAgent + i] = (int8_t)sp;
        }
        const uint64_t m1 = ballot64(sp == 1), m2 = ballot64(sp == 2);
        const uint64_t m3 = ballot64(sp == 3), m4 = ballot64(sp == 4);
        rows[g] = sp == 1 ? rb.x + c1 + (int)rank_below(m1) : sp == 2 ? rb.y + c2 + (int)rank_below(m2)
                : sp == 3 ? rb.z + c3 + (int)rank_below(m3) : rb.w + c4 + (int)rank_below(m4);
        c1 += __popcll(m1); c2 += __popcll(m2); c3 += __popcll(m3); c4 += __popcll(m4);
    }
    // (K1-finder mode: the step's prev-sensor move, updateSensorOutputIdx
    // sim.cpp:736-789, done here -- each slot's last row is K1's obsrow_out,
    // the last sensor's rows precede this one on its stream -- so the caller's
    // stream needs no wait for that sensor; the first wave of a world does it)
    if (S.psem_src != nullptr && (kSplit == 1 || wv % kSplit == 0)) {
#pragma unroll
        for (int g = 0; g < kG; ++g) {
            const int i = 64 * g + (int)lane;
            if (i < n) {
                const int32_t o = S.obsrow_out[base + i];
                const size_t r = (size_t)rows[g];
                uint4 a = make_uint4(0u, 0u, 0u, 0u), b = a;
                if (o >= 0) {
                    a = reinterpret_cast<const uint4 *>(S.psem_src + (size_t)o * kSensor)[0];
                    b = reinterpret_cast<const uint4 *>(S.psem_src + (size_t)o * kSensor)[1];
                }
                reinterpret_cast<uint4 *>(nxt.psem + r * kSensor)[0] = a;
                reinterpret_cast<uint4 *>(nxt.psem + r * kSensor)[1] = b;
                if (depth) {
                    uint4 c = make_uint4(0u, 0u, 0u, 0u), d = c;
                    if (o >= 0) {
                        c = reinterpret_cast<const uint4 *>(S.pdepth_src + (size_t)o * kSensor)[0];
                        d = reinterpret_cast<const uint4 *>(S.pdepth_src + (size_t)o * kSensor)[1];
                    }
                    reinterpret_cast<uint4 *>(nxt.pdepth + r * kSensor)[0] = c;
                    reinterpret_cast<uint4 *>(nxt.pdepth + r * kSensor)[1] = d;
                }
            }
        }
    }
    const int nobj = na + n;
    // sentinels past the last object: a NaN position fails every P1 test, so
    // the pair loop needs no bounds check or clamped read (j < nobj + 63)
    constexpr bool kPad = kCap <= 128;
    if (kPad) L.obj[nobj + (int)lane] = make_float2(__builtin_nanf(""), __builtin_nanf(""));
    if (lane <= (uint32_t)kSensor) {   // every wave stores the same bits: no barrier
        R.u[lane] = ray.x;
        R.c[lane] = ray.y;
        R.s[lane] = ray.z;
        R.e[lane] = ray.w;
    }
    wave_sync();

    uint32_t mbc = 0;
    for (int a0 = kChunk0; a0 < n; a0 += kChunkStep) {
        const int nc = min(kKeyAgents, n - a0);
        MB_CNT(1, 1);
        for (int q = lane; q < nc * kKeyStride; q += 64) L.key[q] = Key<K>::none;
        wave_sync();
        // ---- P1: wedge pre-cull of the chunk's (agent, object) pairs.  Lane =
        // (agent a, object group o): the chunk's nc agents rounded up to P = 1,
        // 2, 4 or 8 and G = 64 / P object groups, objects j = o + G t ----
        int nq = 0;
        {
            const int P = nc > 4 ? 8 : nc > 2 ? 4 : nc > 1 ? 2 : 1;
            const int G = 64 / P, lgG = 6 - (P == 8 ? 3 : P == 4 ? 2 : P == 2 ? 1 : 0);
            const int a = (int)lane >> lgG, o = (int)lane & (G - 1);
            const int ia = a0 + min(a, nc - 1);
            // a lane past the chunk's agents gets a NaN camera: every test fails
            const float2 ap = a < nc ? L.obj[na + ia] : make_float2(__builtin_nanf(""), __builtin_nanf(""));
            const float2 ah = L.hd[ia];
            const int self = na + ia;
            // the camera's own projections, so (f, l) of an object p are two
            // FMAs each: f = p.h - c, l = p.r - d (r = (hy, -hx)).  An
            // approximation of pair_fl's (f, l) within ~1e-5 (|p|, |a| <= 160):
            // the wedge's + 0.05 and the angular cull's 1e-4 margin in u
            // (>= 1e-4 |f| in l) dwarf it; survivors recompute exactly.  (A NaN
            // camera gives NaN c, d: every test fails.)
            const float pc = __builtin_fmaf(ap.x, ah.x, ap.y * ah.y);
            const float pd = __builtin_fmaf(ap.x, ah.y, -(ap.y * ah.x));
            // body of one P1 iteration; kKind 0: every lane's object is food
            // (j + G <= na), 1: every one an agent (j >= na), 2: mixed -- the
            // radius and the self test then compile out of the uniform kinds
            auto p1_iter = [&](const int jb, auto kind_tag) {
                constexpr int kKind = decltype(kind_tag)::value;
                MB_CNT(2, 1);
                const int j = jb + o;
                // (j >= nobj reads a NaN sentinel: keep comes out false)
                const float2 p = L.obj[kPad ? j : min(j, nobj - 1)];
                const float f = __builtin_fmaf(p.x, ah.x, __builtin_fmaf(p.y, ah.y, -pc));
                const float l = __builtin_fmaf(p.x, ah.y, __builtin_fmaf(-p.y, ah.x, -pd));
                const bool food = kKind == 0 ? true : kKind == 1 ? false : j < na;
                const float af = fabsf(f);
                // the object's radius with the cull's 1.001 margin (the wedge's
                // half-width sqrt(2) rk + 0.05 >= sqrt(2) R + 0.05)
                const float rk = food ? 1.42f * 1.001f : kAgentR * 1.001f;
                const float wk = food ? 1.41421356f * (1.42f * 1.001f) + 0.05f
                                      : 1.41421356f * (kAgentR * 1.001f) + 0.05f;
#if MB_P1_MASKS
                // the keep mask straight from the compares (P1 runs with every
                // lane active): VOPC masks combined by scalar ops, and the queue
                // slot selected by the mask itself -- no per-lane bool turned
                // back into a ballot (2 VALU less per iteration)
                uint64_t m = fcmp_mask<kCmpOLE>(fabsf(l), af + wk);
                if (!kPad) m &= icmp_mask<kCmpSLT>(j, nobj);
                if (kKind != 0) m &= icmp_mask<kCmpNE>(j, self);
                {
                    // a far pair (|f| >= kFarCull) also needs a pixel centre, or
                    // forward the finder ray u = 0, within w of its centre's
                    // offset u_c = l / f: w bounds the bounding circle's roots,
                    // a (sqrt(1 + u_c^2) + a |u_c|) / (1 - a^2) with a = R / |f|
                    // (<= 0.284 here), plus the rcp / FMA error margin (56 % of
                    // the wedge's survivors go: step -3 %)
                    const float rf = __builtin_amdgcn_rcpf(f);
                    const float uc = l * rf;
                    // (ar carries the 1.001 margin itself: every factor only grows)
                    // The bound a (1 + u_c^2 / 2 + a |u_c|) (1 + 1.2 a^2) is taken
                    // as a (1 + u_c^2 / 2 + a (|u_c| + 2.9 a)), never smaller where
                    // it is used: 1.2 (1 + u_c^2 / 2 + a |u_c|) <= 2.9 for a <= 0.285
                    // and |u_c| <= 1 + 2.06 / 5 inside the wedge (5 ops, was 8)
                    const float ar = rk * fabsf(rf);
                    const float w = __builtin_fmaf(
                        ar, __builtin_fmaf(ar, __builtin_fmaf(2.9f, ar, fabsf(uc)), __builtin_fmaf(0.5f * uc, uc, 1.0f)),
                        1e-4f);
                    const float sc = f > 0.0f ? 12.0f : 4.0f;
                    const float s = __builtin_fmaf(uc, sc, sc - 0.5f);
                    // the nearest integer, not clamped to the pixels [0, 2 sc - 1]:
                    // off the range it is at least as near as the clamped one, so
                    // the test keeps a superset (a few more edge survivors for P2's
                    // exact test, 3 VALU less per iteration: step -0.9 %); s is
                    // finite for every far pair (|u_c| <= 1.42 in the wedge)
                    const float sn = __builtin_rintf(s);
                    m &= fcmp_mask<kCmpOLT>(af, kFarCull) | fcmp_mask<kCmpOLE>(fabsf(s - sn), sc * w) |
                         (fcmp_mask<kCmpOGT>(f, 0.0f) & fcmp_mask<kCmpOLE>(fabsf(uc), w));
                }
                L.qcode[select_by_mask(m, nq + (int)rank_below(m), kQueueCap)] = (uint32_t)a | ((uint32_t)j << 11);
                nq += __popcll(m);
#else   // (the per-lane form: the same tests as a bool, turned back into a ballot)
                bool keep = (kPad | (j < nobj)) & (kKind == 0 || j != self) & (fabsf(l) <= af + wk);
                {
                    const float rf = __builtin_amdgcn_rcpf(f);
                    const float uc = l * rf;
                    const float ar = rk * fabsf(rf);
                    const float w = __builtin_fmaf(
                        ar, __builtin_fmaf(ar, __builtin_fmaf(2.9f, ar, fabsf(uc)), __builtin_fmaf(0.5f * uc, uc, 1.0f)),
                        1e-4f);
                    const bool fwd = f > 0.0f;
                    const float sc = fwd ? 12.0f : 4.0f;
                    const float s = __builtin_fmaf(uc, sc, sc - 0.5f);
                    const float sn = __builtin_rintf(s);
                    const bool pix = fabsf(s - sn) <= sc * w;
                    const bool fin = fwd & (fabsf(uc) <= w);
                    keep = keep & ((af < kFarCull) | pix | fin);
                }
                const uint64_t m = ballot64(keep);
                // branch-free: culled lanes write the sink slot (+1 % step)
                L.qcode[keep ? nq + (int)rank_below(m) : kQueueCap] = (uint32_t)a | ((uint32_t)j << 11);
                nq += __popcll(m);
#endif
                if (nq >= 64) {
                    wave_sync();
#ifndef MB_SKIP_P2
                    run_survivors(L, R, na, a0, nq - 64, 64, mbc);
#endif
                    nq -= 64;
                }
            };
            // food iterations, the one straddling na (none for full chunks: G
            // = 8 divides na), agent iterations
            int jb = 0;
            for (; jb + G <= na; jb += G) p1_iter(jb, std::integral_constant<int, 0>{});
            if (jb < na) { p1_iter(jb, std::integral_constant<int, 2>{}); jb += G; }
            // the food survivors as a batch of their own when the agents'
            // would fill another anyway: a batch mixing far squares and far
            // discs runs both paths (and so do its near-pair rounds)
            if (nq >= MB_SPLIT_FLUSH) {
                wave_sync();
#ifndef MB_SKIP_P2
                run_survivors(L, R, na, a0, 0, nq, mbc);
#endif
                nq = 0;
            }
            for (; jb < nobj; jb += G) p1_iter(jb, std::integral_constant<int, 1>{});
        }
        if (nq > 0) {
            wave_sync();
#ifndef MB_SKIP_P2
            run_survivors(L, R, na, a0, 0, nq, mbc);
#endif
        }
        wave_sync();
#ifndef MB_SKIP_OUT
        // ---- output: keys vs walls; lane = (agent ci, pixels 4g .. 4g+3) ----
        {
            const int ci = (int)(lane >> 3), g = (int)(lane & 7u);
            const int cc = min(ci, nc - 1);
            const int i = a0 + cc;
            const float2 p = L.obj[na + i], h = L.hd[i];
            K kvs[4];
            if constexpr (sizeof(K) == 4) {
                const uint4 kv4 = *reinterpret_cast<const uint4 *>(&L.key[cc * kKeyStride + 4 * g]);
                kvs[0] = kv4.x; kvs[1] = kv4.y; kvs[2] = kv4.z; kvs[3] = kv4.w;
            } else {
                const ulonglong2 *kp = reinterpret_cast<const ulonglong2 *>(&L.key[cc * kKeyStride + 4 * g]);
                const ulonglong2 k01 = kp[0], k23 = kp[1];
                kvs[0] = k01.x; kvs[1] = k01.y; kvs[2] = k23.x; kvs[3] = k23.y;
            }
            const float4 u4 = *reinterpret_cast<const float4 *>(&R.u[4 * g]);
            // the chunk's 64-slot group (8 | 64: one group per chunk), a uniform branch
            int r;
            if constexpr (kG == 2) {
                r = a0 < 64 ? __shfl(rows[0], i & 63) : __shfl(rows[1], i & 63);
            } else {
                r = __shfl(rows[0], i & 63);
#pragma unroll
                for (int g = 1; g < kG; ++g)
                    if ((a0 >> 6) == g) r = __shfl(rows[g], i & 63);
            }
            // backward pixels look along -(h + u r): the sign folded into the
            // heading, sgn (h.x + u h.y) == (sgn h.x) + u (sgn h.y) exactly (IEEE
            // rounding is sign-symmetric)
            const bool fw = g < 6;
            const float hxs = fw ? h.x : -h.x, hys = fw ? h.y : -h.y;
            const float us[4] = {u4.x, u4.y, u4.z, u4.w};
            // every ray as if its near point lay in the inner rectangle (true
            // for every agent 1.2 inside it: the wall is the ray's exit) and
            // the agent strictly inside it; the rays of the others are redone
            // below
            const float lox = kInLo - p.x, hix = kInHiX - p.x, loy = kInLo - p.y, hiy = kInHiY - p.y;
            uint32_t semv = 0, depv = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float u = us[t];
                const float dx = hxs + u * hys, dy = hys + u * (-hxs);
                const K kv = kvs[t];
                const float oz = Key<K>::z(kv);
                const uint32_t order = Key<K>::order(kv);
                const bool obj = (kv != Key<K>::none) & beats_wall_in(lox, hix, loy, hiy, dx, dy, oz);
                // (read for any key: a miss's order bits 0x1FF clamp into the table)
                const int sem = obj ? (int)L.sem_of[min(order, (uint32_t)(kOrderAgent + kCap - 1))] : 5;
                semv |= (uint32_t)(uint8_t)(int8_t)sem << (8 * t);
                if (depth) {
                    const float z = obj ? oz : wall_z(p.x, p.y, dx, dy);
                    depv |= (uint32_t)depth_u8(z) << (8 * t);
                }
            }
            if (ci < nc) {
                constexpr bool nt = (MB_NT & 8) != 0;
                st_stream(reinterpret_cast<uint32_t *>(nxt.sem + (size_t)r * kSensor) + g, semv, nt);
                if (depth) st_stream(reinterpret_cast<uint32_t *>(nxt.depth + (size_t)r * kSensor) + g, depv, nt);
            }
        }
        bool shallow = false;   // lane a < nc: agent a0 + a is within 1.2 of the inner rectangle's edge
        if ((int)lane < nc) {
            const int i = a0 + (int)lane;
            const float2 p = L.obj[na + i], h = L.hd[i];
            const K kv = L.key[lane * kKeyStride + kSensor];
            const uint32_t order = Key<K>::order(kv);
#ifndef MB_PROBE_ALL_DEEP   // (instruction-count probe: wrong rows near the walls)
            shallow = !((p.x >= kInLo + 1.2f) & (p.x <= kInHiX - 1.2f) & (p.y >= kInLo + 1.2f) &
                        (p.y <= kInHiY - 1.2f));
#endif
            // (a shallow agent not strictly inside is redone below)
            const bool agent = (kv != Key<K>::none) & (order >= kOrderAgent) &&
                               beats_wall_in(kInLo - p.x, kInHiX - p.x, kInLo - p.y, kInHiY - p.y, h.x, h.y,
                                             Key<K>::z(kv));
            S.finder[base + i] = agent ? (int32_t)(order - kOrderAgent) : -1;
        }
        // ---- the agents near the walls: each ray's near point
        // P0 = o + c d placed -- in the inner rectangle (the pass above stands),
        // inside a wall box (the wall at view depth c: objects hidden) or beyond
        // the walls (a miss: semantic -1, objects seen); an agent not strictly
        // inside the rectangle has its inner rays redone too (beats_wall_in
        // assumed it); two agents per iteration, lane = (agent, ray), the
        // finder ray on lane 0 of each half
        uint64_t sm = ballot64(shallow);
        while (sm != 0ull) {   // wave-uniform
            const int a_lo = (int)__builtin_ctzll(sm);
            sm &= sm - 1ull;
            const int a_hi = sm != 0ull ? (int)__builtin_ctzll(sm) : -1;
            if (sm != 0ull) sm &= sm - 1ull;
            MB_CNT(8, 1);
            const int ca = lane < 32 ? a_lo : a_hi;
            const int i = a0 + max(ca, 0);
            int r = __shfl(rows[0], i & 63);
#pragma unroll
            for (int gg = 1; gg < kG; ++gg) {
                const int rg = __shfl(rows[gg], i & 63);
                if ((i >> 6) == gg) r = rg;
            }
            if (ca >= 0) {
                const int k = (int)(lane & 31u);
                const float2 p = L.obj[na + i], h = L.hd[i];
                const bool fw = k < 24;
                const float c = R.c[k], sn = R.s[k];
                const float ex = c * h.x + sn * h.y, ey = c * h.y + sn * (-h.x);
                const int cls = wall_class(fw ? p.x + ex : p.x - ex, fw ? p.y + ey : p.y - ey);
                const bool edge = !strictly_inside(p.x, p.y);
                if ((cls != kWallInner) | edge) {
                    const K kv = L.key[ca * kKeyStride + k];
                    const float oz = Key<K>::z(kv);
                    const uint32_t order = Key<K>::order(kv);
                    const bool none = cls == kWallNone, inner = cls == kWallInner;
                    const float u = R.u[k];
                    const float hxs = fw ? h.x : -h.x, hys = fw ? h.y : -h.y;
                    const float dx = hxs + u * hys, dy = hys + u * (-hxs);
                    const bool obj = (kv != Key<K>::none) & (none | (inner && beats_wall(p.x, p.y, dx, dy, oz)));
                    const int sem = obj ? (int)L.sem_of[min(order, (uint32_t)(kOrderAgent + kCap - 1))] : (none ? -1 : 5);
                    nxt.sem[(size_t)r * kSensor + k] = (int8_t)sem;
                    if (depth) {
                        const float z = obj ? oz : none ? __builtin_inff() : inner ? wall_z(p.x, p.y, dx, dy) : c;
                        nxt.depth[(size_t)r * kSensor + k] = depth_u8(z);
                    }
                }
                if (k == 0) {   // the finder ray (u = 0, near point 1.1 ahead)
                    const float fc = R.c[kSensor], fsn = R.s[kSensor];
                    const float fx = fc * h.x + fsn * h.y, fy = fc * h.y + fsn * (-h.x);
                    const int fcls = wall_class(p.x + fx, p.y + fy);
                    if ((fcls != kWallInner) | edge) {
                        const K kv = L.key[ca * kKeyStride + kSensor];
                        const uint32_t order = Key<K>::order(kv);
                        const bool see = (fcls == kWallNone) |
                                         ((fcls == kWallInner) &&
                                          beats_wall(p.x, p.y, h.x, h.y, Key<K>::z(kv)));
                        const bool agent = (kv != Key<K>::none) & (order >= kOrderAgent) & see;
                        S.finder[base + i] = agent ? (int32_t)(order - kOrderAgent) : -1;
                    }
                }
            }
        }
#endif
        wave_sync();
    }
#ifdef MB_COUNT
    if (lane == 0) S.overflow[w] += mbc;
#else
    (void)mbc;
#endif
    }
}

// kList (mixed classes): the worlds K2 listed as past the small class
// (S.big_s of this step's parity), a wave per world in a grid-stride loop;
// kSkipBig: the small class's launch beside it, which leaves those worlds
template <bool kDepth, int kSplit, int kCap, int kWaves, bool kList = false, bool kSkipBig = false>
__global__ __launch_bounds__(64 * kWaves, sensor_min_waves(kCap)) void sensor_kernel(SimState S,
                                                                                            ObsTable nxt)
{
    __shared__ SensorLDS<kCap> lds[kWaves];
    __shared__ RayTab R;
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    static_assert(kWaves % kSplit == 0, "split must divide the block's waves");
    if constexpr (kList) {
        static_assert(kSplit == 1, "the class kernel renders a world per wave");
        const uint32_t par = S.list_par;
        const uint32_t cnt = uniform(S.big_cnt[par * 2 + 1]);
        for (uint32_t i = blockIdx.x * kWaves + wv; i < cnt; i += gridDim.x * kWaves) {
            const uint32_t w = uniform((uint32_t)S.big_s[(size_t)par * S.W + i]);
            sensor_world<kDepth, 1, kCap>(S, nxt, lds[wv], R, w, wv, lane);
            wave_sync();
        }
    } else {
        constexpr uint32_t kWpb = kWaves / kSplit;   // worlds per block
        uint32_t w = blockIdx.x * kWpb + wv / kSplit;
        if (S.sorder) {
            // blocks in dispatch order take every tile's heaviest worlds first,
            // its lightest last (block b: tile b % ntiles, the tile's b / ntiles-th
            // group of kWpb worlds; used when every tile is full), so the kernel's
            // drain runs the cheapest worlds and a block's worlds cost about the same
            const uint32_t b = blockIdx.x, tile = b % S.ntiles, q = b / S.ntiles;
            w = (uint32_t)S.sorder[(size_t)tile * kTileWorlds + q * kWpb + wv / kSplit];
        }
        w = uniform(w);
        if (w >= S.W) return;
        sensor_world<kDepth, kSplit, kCap, kSkipBig>(S, nxt, lds[wv], R, w, wv, lane);
    }
}



// ---------------------------------------------------------------------------
// Learner observation rows (learn/util.py:14-29 construct_obs):
// out[r] = [depth 32 | health 1 | position 2 | semantic 32 | surrounding 2] as
// f32 -- torch.cat's promotion of the five exported views: depth bytes as
// uint8 (the semantic buffer when depth aliases it, B.1), health as the f32
// reinterpretation of its int32 bits (B.2), semantic bytes as int8.  All N rows
// (every species, species-major) in one pass.  A block takes 64 rows: their
// inputs are loaded coalesced into LDS (depth / semantic as 16-B granules),
// then the block's 64 x 69 contiguous output floats are written coalesced, four
// per thread as 16-B stores (HBM-bound: 84 B read + 276 B written per row).
// ---------------------------------------------------------------------------
#ifndef MB_OBS_NT
#define MB_OBS_NT 1   // non-temporal stores of the [N, 69] rows (written once, 600 MB at
                      // 65536 worlds: reference loop -2 % vs plain stores)
#endif
constexpr int kObsDim = 69;
constexpr int kObsRows = 64;
__global__ __launch_bounds__(256) void construct_obs_kernel(const uint32_t *totals,
                                                            const uint8_t *depth,
                                                            const int8_t *sem,
                                                            const int32_t *health,
                                                            const float *pos, const float *sur,
                                                            const int32_t *src_of,
                                                            float *out, uint32_t out_rows)
{
    __shared__ uint4 s_dep[kObsRows * 2], s_sem[kObsRows * 2];
    __shared__ int32_t s_hp[kObsRows];
    __shared__ float2 s_pos[kObsRows], s_sur[kObsRows];
    const uint32_t N = min(totals[0], out_rows);
    const uint32_t nblk = (N + kObsRows - 1) / kObsRows;
    const uint32_t t = threadIdx.x;
    const uint8_t *sd = reinterpret_cast<const uint8_t *>(s_dep);
    const int8_t *ss = reinterpret_cast<const int8_t *>(s_sem);
    // output float (r, c) of the block's rows from the LDS image
    auto val = [&](uint32_t i) {
        const uint32_t r = i / kObsDim, c = i - r * kObsDim;
        if (c < 32) return (float)sd[r * kSensor + c];
        if (c == 32) return __int_as_float(s_hp[r]);
        if (c < 35) return c == 33 ? s_pos[r].x : s_pos[r].y;
        if (c < 67) return (float)ss[r * kSensor + (c - 35)];
        return c == 67 ? s_sur[r].x : s_sur[r].y;
    };
    for (uint32_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        const uint32_t r0 = b * kObsRows, nr = min((uint32_t)kObsRows, N - r0);
        if (t < 2 * nr) s_dep[t] = reinterpret_cast<const uint4 *>(depth + (size_t)r0 * kSensor)[t];
        else if (t >= 128 && t - 128 < 2 * nr)
            s_sem[t - 128] = reinterpret_cast<const uint4 *>(sem + (size_t)r0 * kSensor)[t - 128];
        if (t < nr) {
            // (src_of: the deferred Prev move's gather, a newborn's row zero)
            const int32_t q = src_of ? src_of[r0 + t] : (int32_t)(r0 + t);
            int32_t hp = 0;
            float2 ps = make_float2(0.0f, 0.0f), su = ps;
            if (q >= 0) {
                hp = health[q];
                ps = reinterpret_cast<const float2 *>(pos)[q];
                su = reinterpret_cast<const float2 *>(sur)[q];
            }
            s_hp[t] = hp;
            s_pos[t] = ps;
            s_sur[t] = su;
        }
        __syncthreads();
        float *o = out + (size_t)r0 * kObsDim;
        if (nr == (uint32_t)kObsRows && (reinterpret_cast<uintptr_t>(out) & 15u) == 0) {
            // 64 x 69 floats = 1104 16-B granules
            for (uint32_t g = t; g < kObsRows * kObsDim / 4; g += 256)
                st_stream(reinterpret_cast<uint4 *>(o) + g,
                          make_uint4(__float_as_uint(val(4 * g)), __float_as_uint(val(4 * g + 1)),
                                     __float_as_uint(val(4 * g + 2)), __float_as_uint(val(4 * g + 3))),
                          MB_OBS_NT != 0);
        } else {
            for (uint32_t i = t; i < nr * kObsDim; i += 256) o[i] = val(i);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Rollout records for the learner-rank gather (BASELINE config 5):
// the raw columns learn/training_loop.py:43-57 reads, 64 B per export row --
// semantic 32 | health 4 | position 8 | surrounding 8 | reward 4 | stats as
// four bytes 4 | pad 4 -- plus the depth bytes (96 B) when the manager fixes
// the depth alias.  The gathered records become [N, 69] rows on the learner
// rank (unpack_rollout_kernel: construct_obs over records, bit-identical).
// One thread per record on the pack side (its 16-B granules are contiguous).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pack_rollout_kernel(const uint32_t *totals, ObsTable t, int fixd,
                                                           uint8_t *out, uint32_t out_rows)
{
    const uint32_t N = min(totals[0], out_rows);
    const uint32_t rec = fixd ? kRolloutBytesDepth : kRolloutBytes;
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < N; r += gridDim.x * blockDim.x) {
        uint4 *o = reinterpret_cast<uint4 *>(out + (size_t)r * rec);
        const uint4 *s = reinterpret_cast<const uint4 *>(t.sem + (size_t)r * kSensor);
        o[0] = s[0];
        o[1] = s[1];
        const float2 p = reinterpret_cast<const float2 *>(t.pos)[r];
        const float2 su = reinterpret_cast<const float2 *>(t.sur)[r];
        const int4 st = reinterpret_cast<const int4 *>(t.stats)[r];
        const uint32_t sb = (uint32_t)(st.x & 0xFF) | (uint32_t)(st.y & 0xFF) << 8 |
                            (uint32_t)(st.z & 0xFF) << 16 | (uint32_t)(st.w & 0xFF) << 24;
        o[2] = make_uint4((uint32_t)t.health[r], __float_as_uint(p.x), __float_as_uint(p.y),
                          __float_as_uint(su.x));
        o[3] = make_uint4(__float_as_uint(su.y), __float_as_uint(t.reward[r]), sb, 0u);
        if (fixd) {
            const uint4 *d = reinterpret_cast<const uint4 *>(t.depth + (size_t)r * kSensor);
            o[4] = d[0];
            o[5] = d[1];
        }
    }
}

// Learner side: records -> obs [N, 69] f32 (construct_obs: depth bytes as
// uint8 -- the semantic bytes when aliased, B.1 -- health's int32 bits as
// f32, B.2, position, semantic as int8, surroundings), reward [N], stats
// [N, 4] i32.  64 records per block staged in LDS, the block's 64 x 69 output
// floats written as coalesced 16-B stores (like construct_obs_kernel).
__global__ __launch_bounds__(256) void unpack_rollout_kernel(const uint8_t *recs, uint32_t N, int fixd,
                                                             float *obs, float *reward, int32_t *stats)
{
    constexpr int kW = kRolloutBytesDepth / 16;   // granules per staged record (the widest)
    __shared__ uint4 s_rec[kObsRows * kW];
    const uint32_t rec = fixd ? kRolloutBytesDepth : kRolloutBytes, gpr = rec / 16;
    const uint32_t nblk = (N + kObsRows - 1) / kObsRows;
    const uint32_t t = threadIdx.x;
    const uint8_t *sb = reinterpret_cast<const uint8_t *>(s_rec);
    auto val = [&](uint32_t i) {
        const uint32_t r = i / kObsDim, c = i - r * kObsDim;
        const uint8_t *q = sb + (size_t)r * kW * 16;
        if (c < 32) return (float)q[fixd ? 64 + c : c];
        if (c < 35) return __uint_as_float(reinterpret_cast<const uint32_t *>(q)[8 + (c - 32)]);
        if (c < 67) return (float)(int8_t)q[c - 35];
        return __uint_as_float(reinterpret_cast<const uint32_t *>(q)[11 + (c - 67)]);
    };
    for (uint32_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        const uint32_t r0 = b * kObsRows, nr = min((uint32_t)kObsRows, N - r0);
        for (uint32_t g = t; g < nr * gpr; g += 256) {
            const uint32_t r = g / gpr, k = g - r * gpr;
            s_rec[r * kW + k] = reinterpret_cast<const uint4 *>(recs + (size_t)r0 * rec)[g];
        }
        __syncthreads();
        float *o = obs + (size_t)r0 * kObsDim;
        if (nr == (uint32_t)kObsRows && (reinterpret_cast<uintptr_t>(obs) & 15u) == 0) {
            for (uint32_t g = t; g < kObsRows * kObsDim / 4; g += 256)
                st_stream(reinterpret_cast<uint4 *>(o) + g,
                          make_uint4(__float_as_uint(val(4 * g)), __float_as_uint(val(4 * g + 1)),
                                     __float_as_uint(val(4 * g + 2)), __float_as_uint(val(4 * g + 3))),
                          MB_OBS_NT != 0);
        } else {
            for (uint32_t i = t; i < nr * kObsDim; i += 256) o[i] = val(i);
        }
        if (t < nr) {
            const uint32_t *q = reinterpret_cast<const uint32_t *>(sb + (size_t)t * kW * 16);
            if (reward) reward[r0 + t] = __uint_as_float(q[13]);
            if (stats) {
                const uint32_t s4 = q[14];
                reinterpret_cast<int4 *>(stats)[r0 + t] =
                    make_int4((int)(s4 & 0xFF), (int)((s4 >> 8) & 0xFF), (int)((s4 >> 16) & 0xFF), (int)(s4 >> 24));
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Learner records (BASELINE config 5 round trip, include/mbots.h): everything
// learn/training_loop.py reads between step() and its writes -- the rollout
// record (current observation columns, reward, stats: :49-50, :58), the
// previous observation columns (:87), Action (:47, :93), HiddenState (:48,
// :58) and PrevHiddenState (:89) -- as one 272-B record per export row (336
// with real depth).  The columns are read after the manager materialised the
// step's deferred moves (`t` already holds each logical column's storage).
// ---------------------------------------------------------------------------
struct LearnerCols {
    const int8_t *sem, *psem;
    const uint8_t *depth, *pdepth;
    const int32_t *health, *phealth, *stats, *action;
    const float *pos, *ppos, *sur, *psur, *reward, *hidden, *phidden;
};

__global__ __launch_bounds__(256) void pack_learner_kernel(const uint32_t *totals, LearnerCols c, int fixd,
                                                           uint8_t *out, uint32_t out_rows)
{
    const uint32_t N = min(totals[0], out_rows);
    const uint32_t rec = fixd ? kLearnerBytesDepth : kLearnerBytes;
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < N; r += gridDim.x * blockDim.x) {
        uint4 *o = reinterpret_cast<uint4 *>(out + (size_t)r * rec);
        const uint4 *s = reinterpret_cast<const uint4 *>(c.sem + (size_t)r * kSensor);
        const uint4 *ps = reinterpret_cast<const uint4 *>(c.psem + (size_t)r * kSensor);
        o[0] = s[0];
        o[1] = s[1];
        const float2 p = reinterpret_cast<const float2 *>(c.pos)[r];
        const float2 su = reinterpret_cast<const float2 *>(c.sur)[r];
        const int4 st = reinterpret_cast<const int4 *>(c.stats)[r];
        const uint32_t sb = (uint32_t)(st.x & 0xFF) | (uint32_t)(st.y & 0xFF) << 8 |
                            (uint32_t)(st.z & 0xFF) << 16 | (uint32_t)(st.w & 0xFF) << 24;
        o[2] = make_uint4((uint32_t)c.health[r], __float_as_uint(p.x), __float_as_uint(p.y), __float_as_uint(su.x));
        o[3] = make_uint4(__float_as_uint(su.y), __float_as_uint(c.reward[r]), sb, 0u);
        o[4] = ps[0];
        o[5] = ps[1];
        const float2 pp = reinterpret_cast<const float2 *>(c.ppos)[r];
        const float2 psu = reinterpret_cast<const float2 *>(c.psur)[r];
        const int2 *a = reinterpret_cast<const int2 *>(c.action + (size_t)r * 6);
        const int2 a0 = a[0], a1 = a[1], a2 = a[2];
        o[6] = make_uint4((uint32_t)c.phealth[r], __float_as_uint(pp.x), __float_as_uint(pp.y), __float_as_uint(psu.x));
        o[7] = make_uint4(__float_as_uint(psu.y), (uint32_t)a0.x, (uint32_t)a0.y, (uint32_t)a1.x);
        o[8] = make_uint4((uint32_t)a1.y, (uint32_t)a2.x, (uint32_t)a2.y, 0u);
        const uint4 *hd = reinterpret_cast<const uint4 *>(c.hidden + (size_t)r * kHidden);
        const uint4 *phd = reinterpret_cast<const uint4 *>(c.phidden + (size_t)r * kHidden);
#pragma unroll
        for (int k = 0; k < 4; ++k) o[9 + k] = hd[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[13 + k] = phd[k];
        if (fixd) {
            const uint4 *d = reinterpret_cast<const uint4 *>(c.depth + (size_t)r * kSensor);
            const uint4 *pd = reinterpret_cast<const uint4 *>(c.pdepth + (size_t)r * kSensor);
            o[17] = d[0];
            o[18] = d[1];
            o[19] = pd[0];
            o[20] = pd[1];
        }
    }
}

// Slim learner records (include/mbots.h MBOTS_LEARNER_SLIM_BYTES): the learner
// record's observation part plus each row's provenance src_of[r] at byte 60;
// no Action / HiddenState / PrevHiddenState (the learner rank rebuilds them
// from its own writes, harness/gather.py).  The previous observation columns
// a step still owes (its deferred Prev moves, the lazy prev sensor) are
// gathered here along src_of from the last table -- what the move would write,
// zero for a newborn -- so a pack after step() launches nothing else.
struct LearnerSlimCols {
    const int8_t *sem;
    const uint8_t *depth;
    const int32_t *health, *stats, *src_of;
    const float *pos, *sur, *reward;
    const int8_t *psem;         // prev sensor: rows r, or old rows (gsem)
    const uint8_t *pdepth;
    const int32_t *phealth;     // prev health / position / surrounding: rows r, or old rows (g6)
    const float *ppos, *psur;
    int gsem, g6;
};

__global__ __launch_bounds__(256) void pack_learner_slim_kernel(const uint32_t *totals, LearnerSlimCols c, int fixd,
                                                                uint8_t *out, uint32_t out_rows)
{
    const uint32_t N = min(totals[0], out_rows);
    const uint32_t rec = fixd ? kLearnerSlimBytesDepth : kLearnerSlimBytes;
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < N; r += gridDim.x * blockDim.x) {
        uint4 *o = reinterpret_cast<uint4 *>(out + (size_t)r * rec);
        const int32_t src = c.src_of[r];
        const uint4 *s = reinterpret_cast<const uint4 *>(c.sem + (size_t)r * kSensor);
        o[0] = s[0];
        o[1] = s[1];
        const float2 p = reinterpret_cast<const float2 *>(c.pos)[r];
        const float2 su = reinterpret_cast<const float2 *>(c.sur)[r];
        const int4 st = reinterpret_cast<const int4 *>(c.stats)[r];
        const uint32_t sb = (uint32_t)(st.x & 0xFF) | (uint32_t)(st.y & 0xFF) << 8 |
                            (uint32_t)(st.z & 0xFF) << 16 | (uint32_t)(st.w & 0xFF) << 24;
        o[2] = make_uint4((uint32_t)c.health[r], __float_as_uint(p.x), __float_as_uint(p.y), __float_as_uint(su.x));
        o[3] = make_uint4(__float_as_uint(su.y), __float_as_uint(c.reward[r]), sb, (uint32_t)src);
        // the previous columns: this row's, or its old row's in the last table
        const int32_t ps = c.gsem ? src : (int32_t)r, p6 = c.g6 ? src : (int32_t)r;
        uint4 a = make_uint4(0u, 0u, 0u, 0u), b = a;
        if (ps >= 0) {
            a = reinterpret_cast<const uint4 *>(c.psem + (size_t)ps * kSensor)[0];
            b = reinterpret_cast<const uint4 *>(c.psem + (size_t)ps * kSensor)[1];
        }
        o[4] = a;
        o[5] = b;
        uint32_t ph = 0u;
        float2 pp = make_float2(0.0f, 0.0f), psu = pp;
        if (p6 >= 0) {
            ph = (uint32_t)c.phealth[p6];
            pp = reinterpret_cast<const float2 *>(c.ppos)[p6];
            psu = reinterpret_cast<const float2 *>(c.psur)[p6];
        }
        o[6] = make_uint4(ph, __float_as_uint(pp.x), __float_as_uint(pp.y), __float_as_uint(psu.x));
        o[7] = make_uint4(__float_as_uint(psu.y), 0u, 0u, 0u);
        if (fixd) {
            const uint4 *d = reinterpret_cast<const uint4 *>(c.depth + (size_t)r * kSensor);
            o[8] = d[0];
            o[9] = d[1];
            uint4 e = make_uint4(0u, 0u, 0u, 0u), f = e;
            if (ps >= 0) {
                e = reinterpret_cast<const uint4 *>(c.pdepth + (size_t)ps * kSensor)[0];
                f = reinterpret_cast<const uint4 *>(c.pdepth + (size_t)ps * kSensor)[1];
            }
            o[10] = e;
            o[11] = f;
        }
    }
}

// Learner side: records -> obs / prev_obs [N, 69] (construct_obs of the
// current / previous columns, bit-identical), reward [N], stats [N, 4],
// action [N, 6], hidden / prev_hidden [N, 16]; any output but obs may be null.
// 64 records per block staged in LDS, every output written as contiguous runs.
// (slim: the slim records -- depth at 128 / 160 -- and src [N] instead of
// action / hidden / prev_hidden)
__global__ __launch_bounds__(256) void unpack_learner_kernel(const uint8_t *recs, uint32_t N, int fixd,
                                                             mbots_learner_out o, int slim, int32_t *src)
{
    constexpr int kW = kLearnerBytesDepth / 16;   // granules per staged record (the widest)
    __shared__ uint4 s_rec[kObsRows * kW];
    const uint32_t rec = slim ? (fixd ? kLearnerSlimBytesDepth : kLearnerSlimBytes)
                              : (fixd ? kLearnerBytesDepth : kLearnerBytes),
                   gpr = rec / 16;
    // depth bytes: current at dc, previous at 64 + dp
    const uint32_t dc = slim ? 128u : 272u, dp = slim ? 96u : 240u;
    const uint32_t nblk = (N + kObsRows - 1) / kObsRows;
    const uint32_t t = threadIdx.x;
    const uint8_t *sb = reinterpret_cast<const uint8_t *>(s_rec);
    // obs column c of staged record r: the current (prev = 0) or previous part
    auto val = [&](uint32_t i, int prev) {
        const uint32_t r = i / kObsDim, c = i - r * kObsDim;
        const uint8_t *q = sb + (size_t)r * kW * 16 + (prev ? 64 : 0);
        const uint32_t *q32 = reinterpret_cast<const uint32_t *>(q);
        if (c < 32) return (float)q[fixd ? (prev ? dp : dc) + c : c];
        if (c < 35) return __uint_as_float(q32[8 + (c - 32)]);
        if (c < 67) return (float)(int8_t)q[c - 35];
        return __uint_as_float(q32[11 + (c - 67)]);
    };
    auto word = [&](uint32_t r, uint32_t byte) {
        return reinterpret_cast<const uint32_t *>(sb + (size_t)r * kW * 16 + byte)[0];
    };
    for (uint32_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        const uint32_t r0 = b * kObsRows, nr = min((uint32_t)kObsRows, N - r0);
        for (uint32_t g = t; g < nr * gpr; g += 256) {
            const uint32_t r = g / gpr, k = g - r * gpr;
            s_rec[r * kW + k] = reinterpret_cast<const uint4 *>(recs + (size_t)r0 * rec)[g];
        }
        __syncthreads();
#pragma unroll
        for (int prev = 0; prev < 2; ++prev) {
            float *out = prev ? o.prev_obs : o.obs;
            if (!out) continue;
            float *ob = out + (size_t)r0 * kObsDim;
            if (nr == (uint32_t)kObsRows && (reinterpret_cast<uintptr_t>(out) & 15u) == 0) {
                for (uint32_t g = t; g < kObsRows * kObsDim / 4; g += 256)
                    st_stream(reinterpret_cast<uint4 *>(ob) + g,
                              make_uint4(__float_as_uint(val(4 * g, prev)), __float_as_uint(val(4 * g + 1, prev)),
                                         __float_as_uint(val(4 * g + 2, prev)),
                                         __float_as_uint(val(4 * g + 3, prev))),
                              MB_OBS_NT != 0);
            } else {
                for (uint32_t i = t; i < nr * kObsDim; i += 256) ob[i] = val(i, prev);
            }
        }
        if (o.reward && t < nr) o.reward[r0 + t] = __uint_as_float(word(t, 52));
        if (o.stats && t < nr) {
            const uint32_t s4 = word(t, 56);
            o.stats[4 * (size_t)(r0 + t) + 0] = (int32_t)(s4 & 0xFF);
            o.stats[4 * (size_t)(r0 + t) + 1] = (int32_t)((s4 >> 8) & 0xFF);
            o.stats[4 * (size_t)(r0 + t) + 2] = (int32_t)((s4 >> 16) & 0xFF);
            o.stats[4 * (size_t)(r0 + t) + 3] = (int32_t)(s4 >> 24);
        }
        if (src && t < nr) src[r0 + t] = (int32_t)word(t, 60);
        if (o.action)
            for (uint32_t i = t; i < nr * 6; i += 256) {
                const uint32_t r = i / 6, k = i - r * 6;
                o.action[(size_t)r0 * 6 + i] = (int32_t)word(r, 116 + 4 * k);
            }
        if (o.hidden)
            for (uint32_t i = t; i < nr * kHidden; i += 256) {
                const uint32_t r = i / kHidden, k = i - r * kHidden;
                o.hidden[(size_t)r0 * kHidden + i] = __uint_as_float(word(r, 144 + 4 * k));
            }
        if (o.prev_hidden)
            for (uint32_t i = t; i < nr * kHidden; i += 256) {
                const uint32_t r = i / kHidden, k = i - r * kHidden;
                o.prev_hidden[(size_t)r0 * kHidden + i] = __uint_as_float(word(r, 208 + 4 * k));
            }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// K5: shiftObservationsSystem + shiftHiddenState (sim.cpp:1002-1048): Prev* <-
// current for rows [0, N).  Each column is a contiguous byte range, so the copy
// is one grid-stride stream of 16-byte granules over the concatenation of the
// columns (N is read on the device; granules past a column's end land in its
// 256-B allocation padding / unused capacity rows).  PrevStats rows get the
// reference's prevStats.hitEnemyAgent = stats.hitFriendlyAgent (sim.cpp:1034).
//
// Lazy shift: between shift_observations() and the next step() only the
// learner writes the table, and only its Action / HiddenState columns
// (training_loop.py:136-137).  So the shift copies those two eagerly
// (kShiftEager) and leaves Prev{Species, Position, Health, Surrounding,
// Reward, Stats} as a view of the current columns: the next step moves them
// from there, construct_obs reads them there, and an accessor of one of them
// materialises the copy first (kShiftRest).  kShiftAll copies all eight.
// A shift right after a step runs shift_move_kernel instead (the deferred
// Action / HiddenState move fused with this copy).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void shift_kernel(const uint32_t *totals, ObsTable t, int mode)
{
    const uint32_t N = totals[kTotRows];   // the shard ghost's rows included
    const bool eager = mode != kShiftRest, rest = mode != kShiftEager;
    const uint32_t g4 = rest ? (4u * N + 15u) >> 4 : 0u, g8 = rest ? (8u * N + 15u) >> 4 : 0u;
    const uint32_t g24 = eager ? (24u * N + 15u) >> 4 : 0u;
    const uint32_t gst = rest ? N : 0u, ghd = eager ? 4u * N : 0u;
    // segment ends (in granules): species, pos, health, sur, reward, action, stats, hidden
    const uint32_t e0 = g4, e1 = e0 + g8, e2 = e1 + g4, e3 = e2 + g8, e4 = e3 + g4,
                   e5 = e4 + g24, e6 = e5 + gst, e7 = e6 + ghd;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < e7; g += stride) {
        const uint4 *src;
        uint4 *dst;
        uint32_t k;
        if (g < e0) { src = (const uint4 *)t.species; dst = (uint4 *)t.pspecies; k = g; }
        else if (g < e1) { src = (const uint4 *)t.pos; dst = (uint4 *)t.ppos; k = g - e0; }
        else if (g < e2) { src = (const uint4 *)t.health; dst = (uint4 *)t.phealth; k = g - e1; }
        else if (g < e3) { src = (const uint4 *)t.sur; dst = (uint4 *)t.psur; k = g - e2; }
        else if (g < e4) { src = (const uint4 *)t.reward; dst = (uint4 *)t.preward; k = g - e3; }
        else if (g < e5) { src = (const uint4 *)t.action; dst = (uint4 *)t.paction; k = g - e4; }
        else if (g < e6) { src = (const uint4 *)t.stats; dst = (uint4 *)t.pstats; k = g - e5; }
        else { src = (const uint4 *)t.hidden; dst = (uint4 *)t.phidden; k = g - e6; }
        uint4 v = ld_stream(src + k, (MB_NT & 64) != 0);
        if (g >= e5 && g < e6) v.y = v.x;
        st_stream(dst + k, v, (MB_NT & 2) != 0);
    }
}

// ---------------------------------------------------------------------------
// World init: Sim::Sim + initWorld (sim.cpp:233-275, :1232-1256) and the Init
// graph's initializeChunks (sim.cpp:277-300).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void init_kernel(SimState S)
{
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = uniform(blockIdx.x * kWorldsPerBlock + wv);
    if (w >= S.W) return;
    const size_t base = (size_t)w * S.cap;
    const uint32_t gw = S.world_offset + w;
    const uint2 key = threefry2x32(S.seed, 0u, 0u, gw);   // split_i(initKey(seed), 0, world)
    const int A = (int)S.A;
    for (int i = lane; i < A; i += 64) {
        const float x = u01(rng_draw(key, 2u * (uint32_t)i)) * kLx;
        const float y = u01(rng_draw(key, 2u * (uint32_t)i + 1u)) * kLy;
        S.x[base + i] = x;
        S.y[base + i] = y;
        S.rw[base + i] = 1.0f;
        S.rz[base + i] = 0.0f;
        S.species[base + i] = (i % kNumSpecies) + 1;
        S.health[base + i] = 100;
        S.finder[base + i] = -1;
        S.obsrow[base + i] = -1;
        S.obsrow_out[base + i] = -1;   // the initial export's old rows: none
        S.sur0[base + i] = 0.0f;
        S.sur1[base + i] = 0.0f;
        S.stats[base + i] = 0u;
    }
    if (lane < kNumChunks) S.food[(size_t)w * kNumChunks + lane] = 0ull;
    if (lane < kNumSpecies) {
        S.scount[(size_t)w * kNumSpecies + lane] = A / kNumSpecies + ((int)lane < A % kNumSpecies ? 1 : 0);
        S.sreward[(size_t)w * kNumSpecies + lane] = 0.0f;
    }
    if (lane == 0) {
        S.key[w] = key;
        S.ctr[w] = 2u * (uint32_t)A;
        S.n[w] = A;
        S.cur_food[w] = 0;
        S.overflow[w] = 0u;
    }
}

// ---------------------------------------------------------------------------
// Harness: identity-keyed synthetic action stream
// ---------------------------------------------------------------------------
__device__ __forceinline__ void synthetic_actions_world(const SimState &S, const ObsTable &t, uint32_t seed,
                                                        uint32_t step, int write_hidden, uint32_t w, uint32_t lane)
{
    const size_t base = (size_t)w * S.cap;
    const uint32_t gw = S.world_offset + w;
    const int n = uniform(S.n[w]);
    // slot `lane`'s row loaded beside the count, and its draw computed while
    // both loads are in flight (rows past n are stale and never used)
    const int32_t r0 = (int)lane < (int)S.cap ? S.obsrow[base + lane] : 0;
    const uint32_t k0 = threefry2x32(seed, step, gw, lane).x % 6u;
    for (int i = lane; i < n; i += 64) {
        const size_t r = i < 64 ? (size_t)r0 : (size_t)S.obsrow[base + i];
        const uint32_t k = i < 64 ? k0 : threefry2x32(seed, step, gw, (uint32_t)i).x % 6u;
        int2 *ap = reinterpret_cast<int2 *>(t.action + r * 6);
        ap[0] = make_int2(k == 0, k == 1);
        ap[1] = make_int2(k == 2, k == 3);
        ap[2] = make_int2(k == 4, k == 5);
    }
    // the learner's memory: draw c of slot i (counter 8 i + c) fills
    // hidden[2c], hidden[2c + 1] of the slot's row; the n x 8 draws spread
    // over all 64 lanes (eight lanes per slot, one 64-B row), not eight per
    // slot lane -- the writer is Threefry-bound
    if (write_hidden) {
        constexpr uint32_t kDraws = kHidden / 2;
        const uint32_t nd = (uint32_t)n * kDraws;
        for (uint32_t u0 = 0; u0 < nd; u0 += 64) {   // wave-uniform trips (the shuffle)
            const uint32_t u = u0 + lane, i = u / kDraws, c = u % kDraws;
            const int32_t rs = __shfl(r0, (int)(i & 63u));
            if (u < nd) {
                const size_t r = i < 64 ? (size_t)rs : (size_t)S.obsrow[base + i];
                const uint2 d = threefry2x32(seed ^ 0x9E3779B9u, step, gw, u);
                reinterpret_cast<float2 *>(t.hidden + r * kHidden)[c] =
                    make_float2(u01(d.x) - 0.5f, u01(d.y) - 0.5f);
            }
        }
    }
}

#ifndef MB_ACT_WPW
#define MB_ACT_WPW 1   // worlds per writer wave (straight-line: each its own unrolled body)
#endif
__global__ __launch_bounds__(256) void synthetic_actions_kernel(SimState S, ObsTable t,
                                                                uint32_t seed, uint32_t step,
                                                                int write_hidden)
{
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int k = 0; k < MB_ACT_WPW; ++k) {
        const uint32_t w = uniform((blockIdx.x * MB_ACT_WPW + k) * kWorldsPerBlock + wv);
        if (w < S.W) synthetic_actions_world(S, t, seed, step, write_hidden, w, lane);
    }
}

// sensorIndexTensor (mgr.cpp:241-249): world-major agent order -> export row
__global__ __launch_bounds__(256) void sensor_index_kernel(SimState S, int32_t *out)
{
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = uniform(blockIdx.x * kWorldsPerBlock + wv);
    if (w >= S.W) return;
    const size_t base = (size_t)w * S.cap;
    const int n = uniform(S.n[w]), off = S.world_off[w];
    for (int i = lane; i < n; i += 64) out[off + i] = S.obsrow[base + i];
}

// ---------------------------------------------------------------------------
// Host-side launchers
// ---------------------------------------------------------------------------
static inline unsigned world_blocks(uint32_t W) { return (W + kWorldsPerBlock - 1) / kWorldsPerBlock; }

uint32_t scan_tiles(uint32_t W) { return (W + kTileWorlds - 1) / kTileWorlds; }
bool sensor_order_used(uint32_t W)
{
#ifdef MB_NO_SENSOR_ORDER
    return false;
#else
    static_assert(kTileWorlds % kSensorWorlds == 0 && kTileWorlds % (MB_SENSOR_SPLIT_WAVES / MB_SENSOR_SPLIT) == 0,
                  "a sensor block's worlds lie in one scan tile");
    return W % kTileWorlds == 0;
#endif
}

hipError_t upload_ray_table(const SimState &S, hipStream_t st)
{
    // the same float expressions on the host (IEEE sqrt / division, no
    // contraction): the table's bits are the ones the kernel computed itself
    static float4 tab[36];
    for (int k = 0; k < 36; ++k) {
        const float u = k < kSensor ? u_of(k) : 0.0f;
        const NearPt np = near_pt(u);
        tab[k] = make_float4(u, np.c, np.s, np.e);
    }
    return hipMemcpyAsync(S.raytab, tab, sizeof(tab), hipMemcpyHostToDevice, st);
}

hipError_t launch_init(const SimState &S, hipStream_t st)
{
    hipLaunchKernelGGL(init_kernel, dim3(world_blocks(S.W)), dim3(256), 0, st, S);
    return hipGetLastError();
}
// the join as a value wait (small world counts, mbots_step): one wave after the
// sensor on its queue stores the step's epoch (a vector store at system scope)
// into the signal word the next step's K1 queue polls
__global__ __launch_bounds__(64) void raise_flag_kernel(uint32_t *flag, uint32_t v)
{
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_raise_flag(uint32_t *flag, uint32_t v, hipStream_t st)
{
    hipLaunchKernelGGL(raise_flag_kernel, dim3(1), dim3(64), 0, st, flag, v);
    return hipGetLastError();
}

hipError_t launch_tile_sum(const SimState &S, int parity, hipStream_t st)
{
    hipLaunchKernelGGL(tile_sum_kernel, dim3(S.ntiles), dim3(1024), 0, st, S, parity);
    return hipGetLastError();
}
// the class kernels' fixed grids (mixed classes): blocks looping over the
// listed worlds -- a dispatch of them costs its empty blocks every step
#ifndef MB_K1_LIST_BLOCKS
#define MB_K1_LIST_BLOCKS 1024
#endif
#ifndef MB_SENSOR_LIST_BLOCKS
#define MB_SENSOR_LIST_BLOCKS 2048
#endif
hipError_t launch_world_step(const SimState &S, const ObsTable &cur, int parity, hipStream_t st, hipEvent_t done)
{
    auto go = [&](auto kern, int wpb) {
        const dim3 grid((S.W + wpb - 1) / wpb), blk(64 * wpb);
        if (!done) hipLaunchKernelGGL(kern, grid, blk, 0, st, S, cur, parity);
        else hipExtLaunchKernelGGL(kern, grid, blk, 0u, st, nullptr, done, 0u, S, cur, parity);   // on the packet
    };
    // (K1-finder mode is a <= 256-slot mode: its camera slots are bytes)
    if (S.cap <= 128 || S.mixed) {
        // mixed classes: the small kernel for every world that fits it, then the
        // class kernel over the worlds the last K2 listed (a fixed grid; `done`
        // rides on the last dispatch)
        if (!S.mixed)
            S.k1_finder ? go(world_step_kernel<128, true>, kK1Worlds) : go(world_step_kernel<128, false>, kK1Worlds);
        else {
            hipLaunchKernelGGL((world_step_kernel<128, false, true>), dim3((S.W + kK1Worlds - 1) / kK1Worlds),
                               dim3(64 * kK1Worlds), 0, st, S, cur, parity);
            auto list = [&](auto kern, int wpb) {
                const dim3 grid(std::max(1u, std::min((S.W + wpb - 1) / wpb, (unsigned)MB_K1_LIST_BLOCKS))),
                    blk(64 * wpb);
                if (!done) hipLaunchKernelGGL(kern, grid, blk, 0, st, S, cur, parity);
                else hipExtLaunchKernelGGL(kern, grid, blk, 0u, st, nullptr, done, 0u, S, cur, parity);
            };
            if (S.cap <= 256) list(world_step_list_kernel<256>, k1_worlds<256>());
            else if (S.cap <= 512) list(world_step_list_kernel<512>, k1_worlds<512>());
            else if (S.cap <= 1024) list(world_step_list_kernel<1024>, k1_worlds<1024>());
            else if (S.cap <= 2048) list(world_step_list_kernel<2048>, k1_worlds<2048>());
            else list(world_step_list_kernel<4096>, k1_worlds<4096>());
        }
    } else if (S.cap <= 256)
        S.k1_finder ? go(world_step_kernel<256, true>, kK1Worlds) : go(world_step_kernel<256, false>, kK1Worlds);
    else if (S.cap <= 512)
        go(world_step_kernel<512, false>, k1_worlds<512>());
    else if (S.cap <= 1024)
        go(world_step_kernel<1024, false>, k1_worlds<1024>());
    else if (S.cap <= 2048)
        go(world_step_kernel<2048, false>, k1_worlds<2048>());
    else
        go(world_step_kernel<4096, false>, k1_worlds<4096>());
    return hipGetLastError();
}
hipError_t launch_scan(const SimState &S, int parity, hipStream_t st, hipEvent_t done, bool plain_events)
{
    // `done` rides on the dispatch packet itself (no marker packet between K2
    // and the next kernel on this stream)
    if (!done) {
        hipLaunchKernelGGL(scan_kernel, dim3(S.ntiles), dim3(1024), 0, st, S, parity);
        return hipGetLastError();
    }
    if (plain_events) {   // stream capture: a capturable event record after the dispatch
        hipLaunchKernelGGL(scan_kernel, dim3(S.ntiles), dim3(1024), 0, st, S, parity);
        return hipEventRecord(done, st);
    }
    hipExtLaunchKernelGGL(scan_kernel, dim3(S.ntiles), dim3(1024), 0, st, nullptr, done, 0u, S, parity);
    return hipGetLastError();
}
hipError_t launch_build_lists(const SimState &S, int slot, hipStream_t st)
{
    hipLaunchKernelGGL(build_lists_kernel, dim3((S.W + 255) / 256), dim3(256), 0, st, S, slot);
    return hipGetLastError();
}
hipError_t launch_export_rows(const SimState &S, const ObsTable &nxt, int init, hipStream_t st)
{
    if (init) hipLaunchKernelGGL(export_rows_kernel<true>, dim3(world_blocks(S.W)), dim3(256), 0, st, S, nxt);
    else hipLaunchKernelGGL(export_rows_kernel<false>, dim3((world_blocks(S.W) + MB_EXPORT_WPW - 1) / MB_EXPORT_WPW),
                            dim3(256), 0, st, S, nxt);
    return hipGetLastError();
}
#if defined(MB_PROBE_SHIFT) && !defined(MB_PROBE_BUILD)
#error "MB_PROBE_SHIFT drops moves: a probe build (scripts/build_var.sh -DMB_PROBE_BUILD) only"
#endif
hipError_t launch_move(const SimState &S, const ObsTable &cur, const ObsTable &nxt, int prev_lazy,
                       int parts, hipStream_t st)
{
    MoveArgs m{};
    int k = 0;
    auto add = [&](void *d, const void *s, uint32_t width, uint32_t ipr, uint32_t xform = 0) {
        m.seg[k++] = MoveSeg{d, s, width, ipr, xform};
    };
    // after a lazy shift the six Prev* columns it left are the current ones
    const bool lz = prev_lazy != 0;
    if (parts & kMoveAH) {
        add(nxt.action, cur.action, 8, 3);
        add(nxt.hidden, cur.hidden, 16, 4);
    } else if (parts & kMoveAHShift) {   // the fused shift: the Prev columns (the
                                        // current ones become their views)
#ifdef MB_PROBE_SHIFT   // timing probes (wrong rows): 1 HiddenState only, 2/3 no A/H (3: no prev sensor either)
        if (MB_PROBE_SHIFT == 1) add(nxt.phidden, cur.hidden, 16, 4);
        if (MB_PROBE_SHIFT == 3) parts &= ~kMoveSensor;
#else
        add(nxt.paction, cur.action, 8, 3);
        add(nxt.phidden, cur.hidden, 16, 4);
#endif
    }
    if (parts & kMoveSensor) {
        add(nxt.psem, cur.sem, 16, 2);                   // prev sensor <- last step's sensor
        if (S.flags & kFlagFixDepth) add(nxt.pdepth, cur.depth, 16, 2);
    }
    if (parts & kMovePrev6) {
        add(nxt.pspecies, lz ? cur.species : cur.pspecies, 4, 1);
        add(nxt.ppos, lz ? cur.pos : cur.ppos, 8, 1);
        add(nxt.phealth, lz ? cur.health : cur.phealth, 4, 1);
        add(nxt.psur, lz ? cur.sur : cur.psur, 8, 1);
        add(nxt.preward, lz ? cur.reward : cur.preward, 4, 1);
        add(nxt.pstats, lz ? cur.stats : cur.pstats, 16, 1, lz ? 1u : 0u);
    }
    if (parts & kMovePrevAH) {
        add(nxt.paction, cur.paction, 8, 3);
        add(nxt.phidden, cur.phidden, 16, 4);
    }
    if (k == 0) return hipSuccess;
    m.nseg = k;
#ifndef MB_MOVE_BLOCKS
#define MB_MOVE_BLOCKS 8192   // +0.9 % vs 512 (4096: +0.6 %, 1024/2048 slower)
#endif
    // blocks per segment: a launch of few segments (the prev sensor alone, the
    // fused shift with or without the prev sensor) still needs enough waves in
    // flight to stream
    // (below 65536 worlds a block per two worlds, at most 2048 per segment,
    // covers a segment's items in one or two passes; more would be mostly
    // empty blocks holding wave slots the sensor beside it needs:
    // profiles/r04_shift_grid_small_ab.jsonl, r04_shift_grid_cap_ab.jsonl)
#ifndef MB_MOVE_SMALL
#define MB_MOVE_SMALL 1
#endif
#ifndef MB_MOVE_SMALL_CAP
#define MB_MOVE_SMALL_CAP 2048u
#endif
    const unsigned full = k <= 4 ? (unsigned)MB_MOVE_BLOCKS : 512u;
    const unsigned bx = MB_MOVE_SMALL && S.W < 65536u
                            ? std::max(256u, std::min(std::min(full, (unsigned)MB_MOVE_SMALL_CAP), S.W / 2u))
                            : full;
    if (parts & kMoveAHShift)
        hipLaunchKernelGGL(shift_move_kernel, dim3(bx, k), dim3(256), 0, st, S.totals, S.src_of, m);
    else
        hipLaunchKernelGGL(move_kernel, dim3(bx, k), dim3(256), 0, st, S.totals, S.src_of, m);
    return hipGetLastError();
}
// a dispatch whose completion records `done`: carried by the dispatch packet
// itself (no marker packet), or -- while the stream is being captured into a
// graph, where only event records are capturable -- an event record after it
#define MB_LAUNCH_EV(kern, grid, blk, st, done, plain, ...)                                   \
    do {                                                                                    \
        if (plain || !(done)) {                                                             \
            hipLaunchKernelGGL(kern, grid, blk, 0, st, __VA_ARGS__);                        \
            if (done) (void)hipEventRecord(done, st);                                       \
        } else {                                                                            \
            hipExtLaunchKernelGGL(kern, grid, blk, 0u, st, nullptr, done, 0u, __VA_ARGS__); \
        }                                                                                   \
    } while (0)

template <int kCap, bool kSkipBig = false>
static void launch_sensor_cap(const SimState &S, const ObsTable &nxt, hipStream_t st, hipEvent_t done,
                              bool plain_events)
{
    const bool fixd = (S.flags & kFlagFixDepth) != 0;
    if constexpr (kCap > 256) {
        // the large classes (11 / 21 / 38 / 71 KB of LDS a world at 512 / 1024 /
        // 2048 / 4096 slots): one wave per world, 2 / 1 / 1 / 1 worlds a block,
        // no split
        constexpr int kWv = kCap > 512 ? 1 : 2;
        const dim3 grid((S.W + kWv - 1) / kWv), blk(64 * kWv);
        if (fixd) MB_LAUNCH_EV((sensor_kernel<true, 1, kCap, kWv>), grid, blk, st, done, plain_events, S, nxt);
        else MB_LAUNCH_EV((sensor_kernel<false, 1, kCap, kWv>), grid, blk, st, done, plain_events, S, nxt);
    } else if (S.W <= (uint32_t)MB_SENSOR_SPLIT_MAX) {   // small: MB_SENSOR_SPLIT waves per world
        constexpr int kWv = MB_SENSOR_SPLIT_WAVES, kWpb = kWv / MB_SENSOR_SPLIT;
        const dim3 grid((S.W + kWpb - 1) / kWpb), blk(64 * kWv);
        if (fixd)
            MB_LAUNCH_EV((sensor_kernel<true, MB_SENSOR_SPLIT, kCap, kWv, false, kSkipBig>), grid, blk, st, done, plain_events, S, nxt);
        else
            MB_LAUNCH_EV((sensor_kernel<false, MB_SENSOR_SPLIT, kCap, kWv, false, kSkipBig>), grid, blk, st, done, plain_events, S, nxt);
    } else {
        const dim3 grid((S.W + kSensorWorlds - 1) / kSensorWorlds), blk(64 * kSensorWorlds);
        if (fixd)
            MB_LAUNCH_EV((sensor_kernel<true, 1, kCap, kSensorWorlds, false, kSkipBig>), grid, blk, st, done, plain_events, S, nxt);
        else
            MB_LAUNCH_EV((sensor_kernel<false, 1, kCap, kSensorWorlds, false, kSkipBig>), grid, blk, st, done, plain_events, S, nxt);
    }
}
// mixed classes: the class kernel over the worlds this step's K2 listed (a
// fixed grid of one-wave blocks looping over the list)
template <int kCap>
static void launch_sensor_list(const SimState &S, const ObsTable &nxt, hipStream_t st, hipEvent_t done,
                               bool plain_events)
{
    const dim3 grid(std::max(1u, std::min(S.W, (unsigned)MB_SENSOR_LIST_BLOCKS))), blk(64);
    if (S.flags & kFlagFixDepth)
        MB_LAUNCH_EV((sensor_kernel<true, 1, kCap, 1, true>), grid, blk, st, done, plain_events, S, nxt);
    else
        MB_LAUNCH_EV((sensor_kernel<false, 1, kCap, 1, true>), grid, blk, st, done, plain_events, S, nxt);
}
hipError_t launch_sensor(const SimState &S, const ObsTable &nxt, hipStream_t st, hipEvent_t done,
                         bool plain_events)
{
    if (S.mixed) {
        launch_sensor_cap<128, true>(S, nxt, st, nullptr, plain_events);
        if (S.cap <= 256) launch_sensor_list<256>(S, nxt, st, done, plain_events);
        else if (S.cap <= 512) launch_sensor_list<512>(S, nxt, st, done, plain_events);
        else if (S.cap <= 1024) launch_sensor_list<1024>(S, nxt, st, done, plain_events);
        else if (S.cap <= 2048) launch_sensor_list<2048>(S, nxt, st, done, plain_events);
        else launch_sensor_list<4096>(S, nxt, st, done, plain_events);
        return hipGetLastError();
    }
    if (S.cap <= 128) launch_sensor_cap<128>(S, nxt, st, done, plain_events);
    else if (S.cap <= 256) launch_sensor_cap<256>(S, nxt, st, done, plain_events);
    else if (S.cap <= 512) launch_sensor_cap<512>(S, nxt, st, done, plain_events);
    else if (S.cap <= 1024) launch_sensor_cap<1024>(S, nxt, st, done, plain_events);
    else if (S.cap <= 2048) launch_sensor_cap<2048>(S, nxt, st, done, plain_events);
    else launch_sensor_cap<4096>(S, nxt, st, done, plain_events);
    return hipGetLastError();
}
hipError_t launch_shift(const SimState &S, const ObsTable &t, int mode, hipStream_t st)
{
    hipLaunchKernelGGL(shift_kernel, dim3(4096), dim3(256), 0, st, S.totals, t, mode);
    return hipGetLastError();
}
hipError_t launch_synthetic_actions(const SimState &S, const ObsTable &t, uint32_t seed,
                                    uint32_t step, int write_hidden, hipStream_t st)
{
    hipLaunchKernelGGL(synthetic_actions_kernel, dim3((world_blocks(S.W) + MB_ACT_WPW - 1) / MB_ACT_WPW), dim3(256),
                       0, st, S, t, seed, step, write_hidden);
    return hipGetLastError();
}
hipError_t launch_construct_obs(const SimState &S, const ObsTable &t, int prev, int prev_lazy,
                                float *out, uint32_t out_rows, hipStream_t st, const ObsTable *six_src,
                                int six_lazy)
{
    // Prev{Health, Position, Surrounding} left lazy by the shift are the current ones
    const bool lz = prev && prev_lazy;
    const bool fixd = (S.flags & kFlagFixDepth) != 0;
    const int8_t *sem = prev ? t.psem : t.sem;
    const uint8_t *depth = fixd ? (prev ? t.pdepth : t.depth) : reinterpret_cast<const uint8_t *>(sem);
    const unsigned blocks = (unsigned)std::min<uint64_t>((out_rows + kObsRows - 1) / kObsRows, 16384);
    if (prev && six_src) {   // the step's deferred Prev move of the three columns, gathered here
        const ObsTable &o = *six_src;
        hipLaunchKernelGGL(construct_obs_kernel, dim3(std::max(blocks, 1u)), dim3(256), 0, st, S.totals, depth,
                           sem, six_lazy ? o.health : o.phealth, six_lazy ? o.pos : o.ppos,
                           six_lazy ? o.sur : o.psur, (const int32_t *)S.src_of, out, out_rows);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(construct_obs_kernel, dim3(std::max(blocks, 1u)), dim3(256), 0, st, S.totals, depth, sem,
                       prev && !lz ? t.phealth : t.health, prev && !lz ? t.ppos : t.pos,
                       prev && !lz ? t.psur : t.sur, (const int32_t *)nullptr,
                       out, out_rows);
    return hipGetLastError();
}
hipError_t launch_pack_rollout(const SimState &S, const ObsTable &t, void *out, uint32_t out_rows,
                               hipStream_t st)
{
    const int fixd = (S.flags & kFlagFixDepth) != 0;
    const unsigned blocks = (unsigned)std::min<uint64_t>((out_rows + 255) / 256, 8192);
    hipLaunchKernelGGL(pack_rollout_kernel, dim3(std::max(blocks, 1u)), dim3(256), 0, st, S.totals, t, fixd,
                       static_cast<uint8_t *>(out), out_rows);
    return hipGetLastError();
}
hipError_t launch_unpack_rollout(const void *recs, uint32_t n, int fixd, float *obs, float *reward,
                                 int32_t *stats, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<uint64_t>((n + kObsRows - 1) / kObsRows, 16384);
    hipLaunchKernelGGL(unpack_rollout_kernel, dim3(blocks), dim3(256), 0, st,
                       static_cast<const uint8_t *>(recs), n, fixd, obs, reward, stats);
    return hipGetLastError();
}
hipError_t launch_pack_learner(const SimState &S, const ObsTable &t, int prev_lazy, void *out, uint32_t out_rows,
                               hipStream_t st)
{
    const int fixd = (S.flags & kFlagFixDepth) != 0;
    const bool lz = prev_lazy != 0;
    LearnerCols c;
    c.sem = t.sem;
    c.psem = t.psem;
    c.depth = t.depth;
    c.pdepth = t.pdepth;
    c.health = t.health;
    c.phealth = lz ? t.health : t.phealth;
    c.stats = t.stats;
    c.action = t.action;
    c.pos = t.pos;
    c.ppos = lz ? t.pos : t.ppos;
    c.sur = t.sur;
    c.psur = lz ? t.sur : t.psur;
    c.reward = t.reward;
    c.hidden = t.hidden;
    c.phidden = t.phidden;
    const unsigned blocks = (unsigned)std::min<uint64_t>((out_rows + 255) / 256, 8192);
    hipLaunchKernelGGL(pack_learner_kernel, dim3(std::max(blocks, 1u)), dim3(256), 0, st, S.totals, c, fixd,
                       static_cast<uint8_t *>(out), out_rows);
    return hipGetLastError();
}
hipError_t launch_unpack_learner(const void *recs, uint32_t n, int fixd, const mbots_learner_out &o,
                                 hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<uint64_t>((n + kObsRows - 1) / kObsRows, 16384);
    hipLaunchKernelGGL(unpack_learner_kernel, dim3(blocks), dim3(256), 0, st, static_cast<const uint8_t *>(recs), n,
                       fixd, o, 0, (int32_t *)nullptr);
    return hipGetLastError();
}
hipError_t launch_pack_learner_slim(const SimState &S, const ObsTable &t, int prev_lazy, const ObsTable *six_src,
                                    int six_lazy, const ObsTable *sem_src, void *out, uint32_t out_rows,
                                    hipStream_t st)
{
    const int fixd = (S.flags & kFlagFixDepth) != 0;
    LearnerSlimCols c;
    c.sem = t.sem;
    c.depth = t.depth;
    c.health = t.health;
    c.stats = t.stats;
    c.src_of = S.src_of;
    c.pos = t.pos;
    c.sur = t.sur;
    c.reward = t.reward;
    c.gsem = sem_src != nullptr;
    c.psem = sem_src ? sem_src->sem : t.psem;
    c.pdepth = sem_src ? sem_src->depth : t.pdepth;
    c.g6 = six_src != nullptr;
    if (six_src) {
        const bool lz = six_lazy != 0;
        c.phealth = lz ? six_src->health : six_src->phealth;
        c.ppos = lz ? six_src->pos : six_src->ppos;
        c.psur = lz ? six_src->sur : six_src->psur;
    } else {
        const bool lz = prev_lazy != 0;
        c.phealth = lz ? t.health : t.phealth;
        c.ppos = lz ? t.pos : t.ppos;
        c.psur = lz ? t.sur : t.psur;
    }
    const unsigned blocks = (unsigned)std::min<uint64_t>((out_rows + 255) / 256, 8192);
    hipLaunchKernelGGL(pack_learner_slim_kernel, dim3(std::max(blocks, 1u)), dim3(256), 0, st, S.totals, c, fixd,
                       static_cast<uint8_t *>(out), out_rows);
    return hipGetLastError();
}
// one thread per gathered row: its old row in the last global table, then the
// 152 B of Action / memory / hidden gathered (rows keep their relative order
// through the sort, so the gathers are nearly contiguous)
__global__ __launch_bounds__(256) void rebuild_learner_kernel(RebuildPlan p, const int32_t *src, uint32_t rows,
                                                              uint32_t last_rows, const int32_t *last_action,
                                                              const float *last_memory,
                                                              const float *last_hidden, int32_t *action,
                                                              float *hidden, float *prev_hidden)
{
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += gridDim.x * blockDim.x) {
        int32_t g = rebuild_row(p, (int32_t)r, src[r]);
        if (g >= (int32_t)last_rows) g = -1;   // (a provenance the last table does not hold: never read)
        int2 a0 = make_int2(0, 0), a1 = a0, a2 = a0;
        uint4 m[4], hd[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) m[k] = hd[k] = make_uint4(0u, 0u, 0u, 0u);
        if (g >= 0) {
            const int2 *la = reinterpret_cast<const int2 *>(last_action + (size_t)g * 6);
            a0 = la[0];
            a1 = la[1];
            a2 = la[2];
            const uint4 *lm = reinterpret_cast<const uint4 *>(last_memory + (size_t)g * kHidden);
            const uint4 *lh = reinterpret_cast<const uint4 *>(last_hidden + (size_t)g * kHidden);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                m[k] = lm[k];
                hd[k] = lh[k];
            }
        }
        int2 *oa = reinterpret_cast<int2 *>(action + (size_t)r * 6);
        oa[0] = a0;
        oa[1] = a1;
        oa[2] = a2;
        uint4 *om = reinterpret_cast<uint4 *>(hidden + (size_t)r * kHidden);
        uint4 *oh = reinterpret_cast<uint4 *>(prev_hidden + (size_t)r * kHidden);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            om[k] = m[k];
            oh[k] = hd[k];
        }
    }
}

RebuildPlan rebuild_plan(const int64_t *cur, const int64_t *last, uint32_t ranks)
{
    RebuildPlan p{};
    p.ranks = (int32_t)ranks;
    int64_t base = 0;
    for (int s = 0; s < 4; ++s) {   // per species: rank-major segments
        for (uint32_t k = 0; k < ranks; ++k) {
            p.cur_g[k][s] = (int32_t)base;
            base += cur[k * 4 + s];
        }
        p.sp_end[s] = (int32_t)base;
    }
    int64_t lbase = 0;
    for (int s = 0; s < 4; ++s)
        for (uint32_t k = 0; k < ranks; ++k) {
            p.last_g[k][s] = (int32_t)lbase;
            lbase += last[k * 4 + s];
        }
    for (uint32_t k = 0; k < ranks; ++k) {
        int64_t l = 0;
        for (int s = 0; s < 4; ++s) {
            p.last_l[k][s] = (int32_t)l;
            l += last[k * 4 + s];
        }
    }
    return p;
}

hipError_t launch_rebuild_learner(const RebuildPlan &p, const int32_t *src, uint32_t rows, uint32_t last_rows,
                                  const int32_t *last_action, const float *last_memory, const float *last_hidden,
                                  int32_t *action, float *hidden, float *prev_hidden, hipStream_t st)
{
    if (rows == 0) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<uint64_t>((rows + 255) / 256, 16384);
    hipLaunchKernelGGL(rebuild_learner_kernel, dim3(blocks), dim3(256), 0, st, p, src, rows, last_rows, last_action,
                       last_memory, last_hidden, action, hidden, prev_hidden);
    return hipGetLastError();
}

hipError_t launch_unpack_learner_slim(const void *recs, uint32_t n, int fixd, const mbots_learner_out &o,
                                      int32_t *src, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<uint64_t>((n + kObsRows - 1) / kObsRows, 16384);
    hipLaunchKernelGGL(unpack_learner_kernel, dim3(blocks), dim3(256), 0, st, static_cast<const uint8_t *>(recs), n,
                       fixd, o, 1, src);
    return hipGetLastError();
}
hipError_t launch_sensor_index(const SimState &S, int32_t *out, hipStream_t st)
{
    hipLaunchKernelGGL(sensor_index_kernel, dim3(world_blocks(S.W)), dim3(256), 0, st, S, out);
    return hipGetLastError();
}

}  // namespace mbots
