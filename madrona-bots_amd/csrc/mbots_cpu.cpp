// mbots_cpu.cpp -- the CPU execution mode behind the same C ABI (mbots.h,
// MBOTS_EXEC_CPU): BASELINE config 1 ("64 worlds, ExecMode::CPU via
// learn/env.py, runs without a GPU"; learn/env.py:12-15 selects it when no
// GPU is present).  Systems follow the HIP kernels of mbots_kernels.hip
// system for system (sim.cpp:1061-1220), one world per task on host threads;
// every float expression is the shared host+device one (mbots_device.hpp,
// mbots_ray.hpp), so the results are bit-identical to the HIP path.
#include "mbots_cpu.hpp"
#include "mbots_ray.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <type_traits>

namespace mbots {
namespace cpu {

namespace {

constexpr uint32_t kLive = 1u << 8;   // per-package image: x | y << 4 | live << 8
constexpr uint8_t F_HIT_FRIENDLY = 1, F_HIT_ENEMY = 2, F_ATE = 4, F_REPRO = 8, F_ALIVE = 16,
                  F_BREED = 32;

// one world's working image (the K1 LDS image of mbots_kernels.hip)
struct Slot {
    float x, y, rw, rz, s0, s1;
    int32_t accum, row, sp, fd;
    uint8_t fl;
};

inline uint32_t rng_draw(uint2 key, uint32_t ctr) { return threefry2x32(key.x, key.y, ctr, 0u).x; }

// pinhole offsets u = (2k + 1) / 24 - 1 (forward), (2k' + 1) / 8 - 1 (backward)
// as one rounding, the kernels' u_of
inline float ray_u(int k)
{
    return k < 24 ? (float)(2 * k - 23) * (1.0f / 24.0f) : (float)(2 * (k - 24) - 7) * 0.125f;
}

template <typename T> void put(std::vector<T> &v, size_t n) { v.assign(n, T{}); }

}  // namespace

void Table::resize(size_t rows)
{
    put(species, rows); put(health, rows); put(action, rows * 6); put(stats, rows * 4);
    put(pspecies, rows); put(phealth, rows); put(paction, rows * 6); put(pstats, rows * 4);
    put(pos, rows * 2); put(sur, rows * 2); put(reward, rows); put(hidden, rows * kHidden);
    put(ppos, rows * 2); put(psur, rows * 2); put(preward, rows); put(phidden, rows * kHidden);
    put(sem, rows * kSensor); put(psem, rows * kSensor);
    put(depth, rows * kSensor); put(pdepth, rows * kSensor);
}

template <typename F> void Sim::for_worlds(F &&fn) const
{
    const unsigned T = std::max(1u, std::min<unsigned>(threads_, W_));
    if (T == 1) {
        for (uint32_t w = 0; w < W_; ++w) fn(w);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(T);
    for (unsigned t = 0; t < T; ++t) {
        const uint32_t lo = (uint32_t)((uint64_t)W_ * t / T), hi = (uint32_t)((uint64_t)W_ * (t + 1) / T);
        th.emplace_back([&fn, lo, hi] {
            for (uint32_t w = lo; w < hi; ++w) fn(w);
        });
    }
    for (auto &t : th) t.join();
}

Sim::Sim(const mbots_config &cfg)
    : cfg_(cfg), W_(cfg.num_worlds + ((cfg.flags & MBOTS_FLAG_SHARD_GHOST) ? 1u : 0u)), Wx_(cfg.num_worlds),
      cap_(cfg.agent_capacity), A_(cfg.init_num_agents_per_world)
{
    const char *e = getenv("MBOTS_CPU_THREADS");
    // default: the machine's threads up to 16 (a GPU box's per-GPU CPU share;
    // MBOTS_CPU_THREADS overrides, e.g. bench.py's all-core baseline).  Each
    // phase starts its threads on contiguous world ranges: a persistent pool
    // with dynamic chunks measured 2x slower on the GPU box (16-CPU cgroup)
    threads_ = e ? (unsigned)atoi(e) : std::min(16u, std::thread::hardware_concurrency());
    if (threads_ == 0) threads_ = 1;
    const size_t rows = (size_t)W_ * cap_;
    for (auto *v : {&x_, &y_, &rw_, &rz_, &sur0_, &sur1_}) put(*v, rows);
    for (auto *v : {&species_, &health_, &finder_, &obsrow_}) put(*v, rows);
    put(stats_, rows);
    for (auto *v : {&n_, &cur_food_, &world_off_}) put(*v, W_);
    put(scount_, (size_t)W_ * kNumSpecies);
    put(row_base_, (size_t)W_ * kNumSpecies);
    put(key_, W_);
    put(ctr_, W_);
    put(overflow_, W_);
    put(food_rot_, (size_t)W_ * kNumPkg);
    put(food_, (size_t)W_ * kNumChunks);
    put(sreward_, (size_t)W_ * kNumSpecies);
    T_[0].resize(rows);
    T_[1].resize(rows);
    put(zeros_rows_, rows);
    put(zeros_worlds_, W_);
    put(sensor_index_, rows);
    put(src_of_, rows);
    // Sim::Sim + initWorld (sim.cpp:1232-1256, :233-275), then the first export
    for_worlds([&](uint32_t w) { init_world(w); });
    scan();
    agent_steps_ = 0;   // the initial population is not a step
    for_worlds([&](uint32_t w) { export_world(w, T_[1], T_[0], true); });
    tb_ = 0;
}

void Sim::init_world(uint32_t w)
{
    const size_t base = (size_t)w * cap_;
    const uint2 key = threefry2x32(cfg_.rand_seed, 0u, 0u, cfg_.world_offset + w);
    for (uint32_t i = 0; i < A_; ++i) {
        x_[base + i] = u01(rng_draw(key, 2u * i)) * kLx;
        y_[base + i] = u01(rng_draw(key, 2u * i + 1u)) * kLy;
        rw_[base + i] = 1.0f;
        rz_[base + i] = 0.0f;
        species_[base + i] = (int32_t)(i % kNumSpecies) + 1;
        health_[base + i] = 100;
        finder_[base + i] = -1;
        obsrow_[base + i] = -1;
    }
    for (int s = 0; s < kNumSpecies; ++s)
        scount_[(size_t)w * kNumSpecies + s] = (int32_t)(A_ / kNumSpecies + ((uint32_t)s < A_ % kNumSpecies ? 1 : 0));
    key_[w] = key;
    ctr_[w] = 2u * A_;
    n_[w] = (int32_t)A_;
}

// resetChunkInfoSystem, addFoodSystem, actionSystem, healthSync,
// updateSurroundingObservation, speciesTrackerUpdate, speciesInfoSync +
// respawn, SortArchetypeNode<Agent, WorldID> (sim.cpp:1061-1132) -- K1
void Sim::world_step(uint32_t w, const Table &cur)
{
    const size_t base = (size_t)w * cap_;
    const int n0 = n_[w];
    thread_local std::vector<Slot> L;
    L.resize(cap_);
    for (int i = 0; i < n0; ++i) {
        const size_t s = base + i;
        L[i] = Slot{x_[s], y_[s], rw_[s], rz_[s], 0.0f, 0.0f, health_[s], obsrow_[s], species_[s],
                    finder_[s], F_ALIVE};
    }
    uint16_t pk[kNumPkg];
    uint32_t chunk[kNumChunks] = {};   // ChunkInfo: numAgents << 16 | totalSpeed
    for (int c = 0; c < kNumChunks; ++c) {
        const uint64_t rec = food_[(size_t)w * kNumChunks + c];
        for (int q = 0; q < kMaxPkg; ++q)
            pk[c * kMaxPkg + q] = (uint16_t)(((rec >> (8 * q)) & 0xFFu) | (((rec >> (40 + q)) & 1u) << 8));
    }
    const uint2 key = key_[w];
    uint32_t ctr = ctr_[w];
    int32_t cur_food = cur_food_[w];
    auto draw = [&] { return rng_draw(key, ctr++); };

    // ---- addFoodSystem (sim.cpp:363-387) + addFoodToChunk (:308-361) ----
    if (sample_i32(draw(), 0, 10) == 0) {
        uint32_t nfood = (uint32_t)sample_i32(draw(), 1, 3);
        const uint32_t diff = (uint32_t)kFoodCap - (uint32_t)cur_food;
        if (diff < nfood) nfood = diff;
        for (uint32_t f = 0; f < nfood; ++f) {
            const uint32_t cx = (uint32_t)sample_i32(draw(), 0, kChunksX);
            const uint32_t cy = (uint32_t)sample_i32(draw(), 0, kChunksY);
            const int c = (int)(cx + cy * kChunksX);
            draw();   // two unused draws (sim.cpp:311-312)
            draw();
            for (int q = 0; q < kMaxPkg; ++q) {
                if ((pk[c * kMaxPkg + q] & kLive) == 0u) {
                    const uint32_t rx = (uint32_t)sample_i32(draw(), 0, kChunkW);
                    const uint32_t ry = (uint32_t)sample_i32(draw(), 0, kChunkW);
                    // food entity rotation (sim.cpp:338-341): 22-bit quarter turn
                    food_rot_[((size_t)w * kMaxPkg + q) * kNumChunks + c] = (draw() >> 8) & 0x3FFFFFu;
                    pk[c * kMaxPkg + q] = (uint16_t)((rx & 15u) | ((ry & 15u) << 4) | kLive);
                    cur_food += 1;
                    break;
                }
            }
        }
    }

    // ---- actionSystem (sim.cpp:419-502) ----
    for (int i = 0; i < n0; ++i) {
        Slot &a = L[i];
        int32_t act[6] = {0, 0, 0, 0, 0, 0};
        if (a.row >= 0) memcpy(act, &cur.action[(size_t)a.row * 6], sizeof(act));
        uint8_t fl = F_ALIVE | (act[5] ? F_BREED : 0);
        if (act[4] && a.fd >= 0) {
            L[a.fd].accum += -50;
            fl |= (L[a.fd].sp == a.sp) ? F_HIT_FRIENDLY : F_HIT_ENEMY;
        }
        float rw = a.rw, rz = a.rz;
        if (act[2]) {
            const float nw = rw * kRotC - rz * kRotS, nz = rw * kRotS + rz * kRotC;
            rw = nw; rz = nz;
        } else if (act[3]) {
            const float nw = rw * kRotC - rz * (-kRotS), nz = rw * (-kRotS) + rz * kRotC;
            rw = nw; rz = nz;
        }
        float x = a.x, y = a.y;
        const float ox = x, oy = y;
        float dx, dy;
        heading(rw, rz, dx, dy);
        if (act[0]) { x = x + dx; y = y + dy; }
        else if (act[1]) { x = x - dx; y = y - dy; }
        x = fmin_std(kLx - 1.0f, fmax_std(0.0f, x));
        y = fmin_std(kLy - 1.0f, fmax_std(0.0f, y));
        const float ddx = x - ox, ddy = y - oy;
        const float len = sqrtf(ddx * ddx + ddy * ddy);
        const int32_t ci = chunk_index(floorf((x / 1.0f) / 16.0f), floorf((y / 1.0f) / 16.0f));
        chunk[ci] += (1u << 16) + (uint32_t)(len * 2.0f);
        a.x = x; a.y = y; a.rw = rw; a.rz = rz;
        a.fl = fl;
    }

    // ---- healthSync (sim.cpp:505-581): the agents on a cell consume its live
    // packages in slot order (FoodPackage::consume, sim.inl:76-99) ----
    int n1 = n0, consumed = 0;
    uint32_t ovf = 0;
    for (int i = 0; i < n0; ++i) {
        Slot &a = L[i];
        const float chx = (a.x / 1.0f) / 16.0f, chy = (a.y / 1.0f) / 16.0f;
        const uint32_t cx = (uint8_t)(16.0f * (chx - floorf(chx)));
        const uint32_t cy = (uint8_t)(16.0f * (chy - floorf(chy)));
        const int32_t ci = chunk_index(chx, chy);
        const uint32_t cell = cx | (cy << 4) | kLive;
        int32_t h = a.accum;
        uint8_t fl = a.fl;
        for (int q = 0; q < kMaxPkg; ++q) {
            if (pk[ci * kMaxPkg + q] == cell) {
                pk[ci * kMaxPkg + q] &= (uint16_t)0xFFu;   // numFood 1 -> 0
                consumed += 1;
                h = (int32_t)((float)h + 20.0f);
                fl |= F_ATE;
                break;
            }
        }
        if ((fl & F_BREED) && h > 10 && a.fd >= 0 && L[a.fd].sp == a.sp) {   // :547-569
            h -= 40;
            fl |= F_REPRO;
            if (n1 < (int)cap_) {
                L[n1] = Slot{a.x, a.y, 1.0f, 0.0f, 0.0f, 0.0f, 50, -1, a.sp, -1, F_ALIVE};
                n1 += 1;
            } else {
                ovf += 1;
            }
        }
        if (h <= 0) fl &= (uint8_t)~F_ALIVE;
        a.accum = h;
        a.fl = fl;
    }
    cur_food -= consumed;

    // ---- updateSurroundingObservation (sim.cpp:583-654) + tracker (:719-734) ----
    uint32_t cnt[kNumSpecies] = {}, hsum[kNumSpecies] = {};
    for (int i = 0; i < n1; ++i) {
        Slot &a = L[i];
        if (!(a.fl & F_ALIVE)) continue;
        float cpx = a.x / 1.0f, cpy = a.y / 1.0f;
        cpx = cpx - 16.0f * 0.5f;
        cpy = cpy - 16.0f * 0.5f;
        const float chx = cpx / 16.0f, chy = cpy / 16.0f;
        const float x0 = floorf(chx), y0 = floorf(chy), x1 = ceilf(chx), y1 = ceilf(chy);
        const int32_t i00 = chunk_index(x0, y0), i10 = chunk_index(x1, y0);
        const int32_t i01 = chunk_index(x0, y1), i11 = chunk_index(x1, y1);
        const float xi = chx - x0, yi = chy - y0;
        const uint32_t c00 = i00 >= 0 ? chunk[i00] : 0u, c10 = i10 >= 0 ? chunk[i10] : 0u;
        const uint32_t c01 = i01 >= 0 ? chunk[i01] : 0u, c11 = i11 >= 0 ? chunk[i11] : 0u;
        const float n00 = (float)(c00 >> 16), n10 = (float)(c10 >> 16);
        const float n01 = (float)(c01 >> 16), n11 = (float)(c11 >> 16);
        const float s00 = (float)(c00 & 0xFFFFu), s10 = (float)(c10 & 0xFFFFu);
        const float s01 = (float)(c01 & 0xFFFFu), s11 = (float)(c11 & 0xFFFFu);
        const float nx0 = xi * n10 + (1.0f - xi) * n00;
        const float nx1 = xi * n11 + (1.0f - xi) * n01;
        const float sx0 = xi * s10 + (1.0f - xi) * s00;
        const float sx1 = xi * s11 + (1.0f - xi) * s01;
        a.s0 = yi * nx1 + (1.0f - yi) * nx0;
        a.s1 = yi * sx1 + (1.0f - yi) * sx0;
        cnt[a.sp - 1] += 1u;
        hsum[a.sp - 1] += (uint32_t)a.accum;
    }

    // ---- speciesInfoSync (sim.cpp:791-838) + respawn ----
    const uint32_t per_species = A_ / kNumSpecies;
    int n2 = n1;
    for (int s = 0; s < kNumSpecies; ++s) {
        const uint32_t count = cnt[s];
        float avg = (float)hsum[s] / (float)count;
        if (count == 0) avg = 0.0f;
        sreward_[(size_t)w * kNumSpecies + s] = (float)count / (float)A_ + avg / 100.0f - 2.0f;
        for (uint32_t e = count; e < per_species; ++e) {
            const float x = u01(draw()) * kLx;
            const float y = u01(draw()) * kLy;
            if (n2 < (int)cap_) {
                L[n2] = Slot{x, y, 1.0f, 0.0f, 0.0f, 0.0f, 100, -1, s + 1, -1, F_ALIVE};
                n2 += 1;
            } else {
                ovf += 1;
            }
        }
    }

    // ---- compaction (SortArchetypeNode<Agent, WorldID>, sim.cpp:1129) ----
    int nn = 0;
    int32_t sc[kNumSpecies] = {};
    for (int i = 0; i < n2; ++i) {
        const Slot &a = L[i];
        if (!(a.fl & F_ALIVE)) continue;
        const size_t d = base + nn++;
        x_[d] = a.x; y_[d] = a.y; rw_[d] = a.rw; rz_[d] = a.rz;
        species_[d] = a.sp;
        health_[d] = a.accum;
        obsrow_[d] = i < n0 ? a.row : -1;   // newborns / respawns: no row yet
        sur0_[d] = a.s0; sur1_[d] = a.s1;
        stats_[d] = a.fl & 0xFu;
        sc[a.sp - 1] += 1;
    }
    for (int c = 0; c < kNumChunks; ++c) {
        uint64_t rec = 0;
        for (int q = 0; q < kMaxPkg; ++q) {
            const uint32_t p = pk[c * kMaxPkg + q];
            rec |= (uint64_t)(p & 0xFFu) << (8 * q);
            rec |= (uint64_t)((p >> 8) & 1u) << (40 + q);
        }
        food_[(size_t)w * kNumChunks + c] = rec;
    }
    for (int s = 0; s < kNumSpecies; ++s) scount_[(size_t)w * kNumSpecies + s] = sc[s];
    n_[w] = nn;
    ctr_[w] = ctr;
    cur_food_[w] = cur_food;
    overflow_[w] += ovf;
}

// species-major row offsets (SortArchetypeNode<Obs, Species>, sim.cpp:1147-1149,
// rows ordered (species, world, slot)); world-major agent offsets -- K2
void Sim::scan()
{
    int32_t tot[kNumSpecies] = {};
    for (uint32_t w = 0; w < Wx_; ++w)
        for (int s = 0; s < kNumSpecies; ++s) tot[s] += scount_[(size_t)w * kNumSpecies + s];
    int32_t run[kNumSpecies];
    int32_t acc = 0;
    for (int s = 0; s < kNumSpecies; ++s) { run[s] = acc; acc += tot[s]; }
    int32_t off = 0;
    for (uint32_t w = 0; w < Wx_; ++w) {
        for (int s = 0; s < kNumSpecies; ++s) {
            row_base_[(size_t)w * kNumSpecies + s] = run[s];
            run[s] += scount_[(size_t)w * kNumSpecies + s];
        }
        world_off_[w] = off;
        off += n_[w];
    }
    for (uint32_t w = Wx_; w < W_; ++w) {   // the shard ghost: rows after every exported row
        int32_t r = acc;
        for (int s = 0; s < kNumSpecies; ++s) {
            row_base_[(size_t)w * kNumSpecies + s] = r;
            r += scount_[(size_t)w * kNumSpecies + s];
        }
        world_off_[w] = acc;
    }
    N_ = (uint32_t)acc;
    totals_[0] = N_;
    for (int s = 0; s < kNumSpecies; ++s) totals_[1 + s] = (uint32_t)tot[s];
    agent_steps_ += N_;
}

// updateObservations (sim.cpp:687-717), rewardSystem setting 8 (:942-956), and
// the columns that travel with an observation row through the species sort
// (Action, HiddenState, Prev*, the prev sensor, updateSensorOutputIdx
// :736-789) -- K3a + K4, eager
void Sim::export_world(uint32_t w, const Table &cur, Table &nxt, bool init)
{
    const size_t base = (size_t)w * cap_;
    const int n = n_[w];
    const float *rew = &sreward_[(size_t)w * kNumSpecies];
    const bool fixed = (cfg_.flags & MBOTS_FLAG_REWARD_FIXED) != 0;
    const bool fixd = (cfg_.flags & MBOTS_FLAG_FIX_DEPTH_ALIAS) != 0;
    // faithful B.3: rewards[4] reads the next SpeciesInfo row's rewards[0]
    const float next_r0 = (w + 1 < W_) ? sreward_[(size_t)(w + 1) * kNumSpecies] : 0.0f;
    int32_t rank[kNumSpecies] = {};
    auto mv = [](auto &dst, const auto &src, size_t r, int32_t o, size_t k) {
        for (size_t c = 0; c < k; ++c) dst[r * k + c] = o >= 0 ? src[(size_t)o * k + c] : 0;
    };
    for (int i = 0; i < n; ++i) {
        const size_t s = base + i;
        const int32_t sp = species_[s];
        const size_t r = (size_t)(row_base_[(size_t)w * kNumSpecies + sp - 1] + rank[sp - 1]++);
        const int32_t o = obsrow_[s];
        const int32_t h = health_[s];
        const uint32_t st = init ? 0u : stats_[s];
        nxt.species[r] = sp;
        nxt.pos[r * 2] = x_[s];
        nxt.pos[r * 2 + 1] = y_[s];
        nxt.health[r] = h;
        nxt.sur[r * 2] = init ? 0.0f : sur0_[s];
        nxt.sur[r * 2 + 1] = init ? 0.0f : sur1_[s];
        for (int b = 0; b < 4; ++b) nxt.stats[r * 4 + b] = (int32_t)((st >> b) & 1u);
        float rv = 0.0f;
        if (!init) {
            const float sr = fixed ? rew[sp - 1] : (sp < kNumSpecies ? rew[sp] : next_r0);
            rv = sr + (float)h / 100.0f - 0.5f;
            if (st & F_ATE) rv += 10.0f;
            if (st & F_REPRO) rv += 10.0f;
            if (st & F_HIT_ENEMY) rv += 15.0f;
        }
        nxt.reward[r] = rv;
        mv(nxt.action, cur.action, r, o, 6);
        mv(nxt.hidden, cur.hidden, r, o, kHidden);
        mv(nxt.pspecies, cur.pspecies, r, o, 1);
        mv(nxt.ppos, cur.ppos, r, o, 2);
        mv(nxt.phealth, cur.phealth, r, o, 1);
        mv(nxt.psur, cur.psur, r, o, 2);
        mv(nxt.preward, cur.preward, r, o, 1);
        mv(nxt.paction, cur.paction, r, o, 6);
        mv(nxt.pstats, cur.pstats, r, o, 4);
        mv(nxt.phidden, cur.phidden, r, o, kHidden);
        mv(nxt.psem, cur.sem, r, o, kSensor);
        if (fixd) mv(nxt.pdepth, cur.depth, r, o, kSensor);
        src_of_[r] = o;
        obsrow_[s] = (int32_t)r;
    }
}

// the Sensor graph (sim.cpp:1183-1188; build spec DESIGN.md 3.6): every
// (agent, object, ray) through the exact predicates -- K3b
void Sim::sensor_world(uint32_t w, Table &nxt, int lo, int hi)
{
    const size_t base = (size_t)w * cap_;
    const int n = n_[w];
    if (hi < 0) hi = n;
    const bool fixd = (cfg_.flags & MBOTS_FLAG_FIX_DEPTH_ALIAS) != 0;
    // live food in (chunk, package) order: position and rotation
    float2 fp[kNumPkg], fr[kNumPkg];
    int nf = 0;
    for (int c = 0; c < kNumChunks; ++c) {
        const uint64_t rec = food_[(size_t)w * kNumChunks + c];
        for (int q = 0; q < kMaxPkg; ++q) {
            if (!((rec >> (40 + q)) & 1u)) continue;
            const uint32_t xy = (uint32_t)(rec >> (8 * q)) & 0xFFu;
            fp[nf] = make_float2((float)(xy & 15u) + (float)((c % kChunksX) * kChunkW),
                                 (float)(xy >> 4) + (float)((c / kChunksX) * kChunkW));
            fr[nf] = food_cs(food_rot_[((size_t)w * kMaxPkg + q) * kNumChunks + c]);
            ++nf;
        }
    }
    thread_local std::vector<float2> hd;
    hd.resize(cap_);
    // every ray's near point (nearSphere, mgr.cpp:133); the finder's at u = 0
    NearPt np[kRays];
    for (int k = 0; k < kSensor; ++k) np[k] = near_pt(ray_u(k));
    np[kSensor] = finder_np();
    for (int i = 0; i < n; ++i) heading(rw_[base + i], rz_[base + i], hd[i].x, hd[i].y);
    for (int i = lo; i < hi; ++i) {
        const float ax = x_[base + i], ay = y_[base + i];
        const float2 h = hd[i];
        // 64-bit keys in every capacity class (mbots_ray.hpp Key<>: the same
        // (depth, order) minimum as the device's 32-bit keys up to 256 slots)
        using K = uint64_t;
        K key[kRays];
        for (int k = 0; k < kRays; ++k) key[k] = Key<K>::none;
        auto fl_of = [&](float px, float py, float &f, float &l) {
            const float vx = px - ax, vy = py - ay;
            f = vx * h.x + vy * h.y;
            l = vx * h.y - vy * h.x;
        };
        for (int j = 0; j < nf; ++j) {
            float f, l;
            fl_of(fp[j].x, fp[j].y, f, l);
            const FoodBox b = box_setup(f, l, fr[j], h);
            const uint32_t order = kOrderFood + (uint32_t)j;
            for (int k = 0; k < kSensor; ++k) {
                const bool fwd = k < 24;
                if (box_hit(b, ray_u(k), fwd, np[k].c)) key[k] = std::min(key[k], Key<K>::make(box_z(b, fwd), order));
            }
            if (box_hit(b, 0.0f, true, np[kSensor].c))
                key[kSensor] = std::min(key[kSensor], Key<K>::make(box_z(b, true), order));
        }
        for (int j = 0; j < n; ++j) {
            if (j == i) continue;
            float f, l;
            fl_of(x_[base + j], y_[base + j], f, l);
            const uint32_t order = kOrderAgent + (uint32_t)j;
            for (int k = 0; k < kSensor; ++k)
                key[k] = std::min(key[k], pixel_key<K>(f, l, ray_u(k), np[k], k < 24, order));
            key[kSensor] = std::min(key[kSensor], finder_key<K>(f, l, order));
        }
        // each ray's near point: in the inner rectangle (the wall is the exit
        // from it), inside a wall box (the wall, at s0) or beyond (a miss)
        auto cls_of = [&](int k, bool fwd) {
            const float ex = np[k].c * h.x + np[k].s * h.y, ey = np[k].c * h.y + np[k].s * (-h.x);
            return wall_class(fwd ? ax + ex : ax - ex, fwd ? ay + ey : ay - ey);
        };
        const size_t r = (size_t)obsrow_[base + i];
        for (int k = 0; k < kSensor; ++k) {
            const bool fwd = k < 24;
            const float u = ray_u(k), sgn = fwd ? 1.0f : -1.0f;
            const float dx = sgn * (h.x + u * h.y), dy = sgn * (h.y + u * (-h.x));
            const K kv = key[k];
            const float oz = Key<K>::z(kv);
            const uint32_t order = Key<K>::order(kv);
            const int cls = cls_of(k, fwd);
            const bool obj = (kv != Key<K>::none) && (cls == kWallInner ? beats_wall(ax, ay, dx, dy, oz) : cls == kWallNone);
            nxt.sem[r * kSensor + k] = (int8_t)(obj ? (order < kOrderAgent ? 6 : species_[base + order - kOrderAgent])
                                                    : (cls == kWallNone ? -1 : 5));
            if (fixd)
                nxt.depth[r * kSensor + k] = depth_u8(obj ? oz
                                                      : cls == kWallInner ? wall_z(ax, ay, dx, dy)
                                                      : cls == kWallBox ? np[k].c : __builtin_inff());
        }
        const K kv = key[kSensor];
        const uint32_t order = Key<K>::order(kv);
        const int fcls = cls_of(kSensor, true);
        const bool agent = kv != Key<K>::none && order >= kOrderAgent &&
                           (fcls == kWallInner ? beats_wall(ax, ay, h.x, h.y, Key<K>::z(kv)) : fcls == kWallNone);
        finder_[base + i] = agent ? (int32_t)(order - kOrderAgent) : -1;
    }
}

void Sim::step()
{
    const Table &cur = T_[tb_];
    Table &nxt = T_[tb_ ^ 1];
    for_worlds([&](uint32_t w) { world_step(w, cur); });
    scan();
    if (W_ >= 2 * threads_) {
        for_worlds([&](uint32_t w) {
            export_world(w, cur, nxt, false);
            sensor_world(w, nxt);
        });
    } else {   // few (large) worlds: the sensor split by agents over the threads
        for_worlds([&](uint32_t w) { export_world(w, cur, nxt, false); });
        sensor_by_agents(nxt);
    }
    tb_ ^= 1;
}

// the sensor over every world's agents, split evenly by agent count: each
// agent writes only its own rows and finder slot
void Sim::sensor_by_agents(Table &nxt)
{
    uint64_t G = 0;
    for (uint32_t w = 0; w < W_; ++w) G += (uint64_t)n_[w];
    const unsigned T = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(threads_, G));
    auto run = [&](uint64_t lo, uint64_t hi) {
        uint64_t g = 0;
        for (uint32_t w = 0; w < W_ && g < hi; ++w) {
            const uint64_t n = (uint64_t)n_[w];
            const uint64_t a = lo > g ? lo - g : 0, b = std::min(hi - g, n);
            if (a < b) sensor_world(w, nxt, (int)a, (int)b);
            g += n;
        }
    };
    if (T == 1) {
        run(0, G);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(T);
    for (unsigned t = 0; t < T; ++t) th.emplace_back(run, G * t / T, G * (t + 1) / T);
    for (auto &t : th) t.join();
}

// shiftObservationsSystem + shiftHiddenState (sim.cpp:1002-1048)
void Sim::shift_observations()
{
    Table &t = T_[tb_];
    const size_t n = N_;
    std::copy_n(t.species.begin(), n, t.pspecies.begin());
    std::copy_n(t.pos.begin(), 2 * n, t.ppos.begin());
    std::copy_n(t.health.begin(), n, t.phealth.begin());
    std::copy_n(t.sur.begin(), 2 * n, t.psur.begin());
    std::copy_n(t.reward.begin(), n, t.preward.begin());
    std::copy_n(t.action.begin(), 6 * n, t.paction.begin());
    for (size_t r = 0; r < n; ++r) {
        t.pstats[r * 4 + 0] = t.stats[r * 4 + 0];
        t.pstats[r * 4 + 1] = t.stats[r * 4 + 0];   // :1034 hitEnemy <- hitFriendly
        t.pstats[r * 4 + 2] = t.stats[r * 4 + 2];
        t.pstats[r * 4 + 3] = t.stats[r * 4 + 3];
    }
    std::copy_n(t.hidden.begin(), kHidden * n, t.phidden.begin());
}

void Sim::write_synthetic_actions(uint32_t seed, uint32_t step, bool write_hidden)
{
    Table &t = T_[tb_];
    for_worlds([&](uint32_t w) {
        const size_t base = (size_t)w * cap_;
        const uint32_t gw = cfg_.world_offset + w;
        for (int i = 0; i < n_[w]; ++i) {
            const size_t r = (size_t)obsrow_[base + i];
            const uint32_t k = threefry2x32(seed, step, gw, (uint32_t)i).x % 6u;
            for (uint32_t j = 0; j < 6; ++j) t.action[r * 6 + j] = j == k ? 1 : 0;
            if (write_hidden)   // both words of each draw: hidden[2k], hidden[2k + 1]
                for (int q = 0; q < kHidden / 2; ++q) {
                    const uint2 d = threefry2x32(seed ^ 0x9E3779B9u, step, gw, (uint32_t)i * (kHidden / 2) + (uint32_t)q);
                    t.hidden[r * kHidden + 2 * q] = u01(d.x) - 0.5f;
                    t.hidden[r * kHidden + 2 * q + 1] = u01(d.y) - 0.5f;
                }
        }
    });
}

void Sim::sensor_index(int32_t *out) const
{
    for (uint32_t w = 0; w < Wx_; ++w)
        for (int i = 0; i < n_[w]; ++i) out[world_off_[w] + i] = obsrow_[(size_t)w * cap_ + i];
}

uint64_t Sim::overflow() const
{
    uint64_t s = 0;
    for (uint32_t w = 0; w < Wx_; ++w) s += overflow_[w];
    return s;
}

int Sim::export_tensor(int32_t id, mbots_tensor *out)
{
    Table &t = T_[tb_];
    const bool fixd = (cfg_.flags & MBOTS_FLAG_FIX_DEPTH_ALIAS) != 0;
    void *p = nullptr;
    int dt = MBOTS_DTYPE_INT32;
    int64_t rows = N_, cols = 1;
    switch (id) {
    case MBOTS_EXPORT_RESET: p = zeros_worlds_.data(); rows = Wx_; break;
    case MBOTS_EXPORT_ACTION: p = t.action.data(); cols = 6; break;
    case MBOTS_EXPORT_PREV_ACTION: p = t.paction.data(); cols = 6; break;
    case MBOTS_EXPORT_HIDDEN_STATE: p = t.hidden.data(); dt = MBOTS_DTYPE_FLOAT32; cols = kHidden; break;
    case MBOTS_EXPORT_PREV_HIDDEN_STATE: p = t.phidden.data(); dt = MBOTS_DTYPE_FLOAT32; cols = kHidden; break;
    case MBOTS_EXPORT_REWARD: p = t.reward.data(); dt = MBOTS_DTYPE_FLOAT32; break;
    case MBOTS_EXPORT_PREV_REWARD: p = t.preward.data(); dt = MBOTS_DTYPE_FLOAT32; break;
    case MBOTS_EXPORT_DONE: p = zeros_rows_.data(); break;
    case MBOTS_EXPORT_POSITION: p = t.pos.data(); dt = MBOTS_DTYPE_FLOAT32; cols = 2; break;
    case MBOTS_EXPORT_PREV_POSITION: p = t.ppos.data(); dt = MBOTS_DTYPE_FLOAT32; cols = 2; break;
    case MBOTS_EXPORT_HEALTH: p = t.health.data(); dt = MBOTS_DTYPE_FLOAT32; break;   // int32 bits (B.2)
    case MBOTS_EXPORT_PREV_HEALTH: p = t.phealth.data(); dt = MBOTS_DTYPE_FLOAT32; break;
    case MBOTS_EXPORT_SURROUNDING: p = t.sur.data(); dt = MBOTS_DTYPE_FLOAT32; cols = 2; break;
    case MBOTS_EXPORT_PREV_SURROUNDING: p = t.psur.data(); dt = MBOTS_DTYPE_FLOAT32; cols = 2; break;
    case MBOTS_EXPORT_SENSOR_SEMANTIC: p = t.sem.data(); dt = MBOTS_DTYPE_INT8; cols = kSensor; break;
    case MBOTS_EXPORT_SENSOR_DEPTH:   // the semantic buffer unless fixed (sim.cpp:102-112, B.1)
        p = fixd ? (void *)t.depth.data() : (void *)t.sem.data(); dt = MBOTS_DTYPE_UINT8; cols = kSensor; break;
    case MBOTS_EXPORT_PREV_SENSOR_SEMANTIC: p = t.psem.data(); dt = MBOTS_DTYPE_INT8; cols = kSensor; break;
    case MBOTS_EXPORT_PREV_SENSOR_DEPTH:
        p = fixd ? (void *)t.pdepth.data() : (void *)t.psem.data(); dt = MBOTS_DTYPE_UINT8; cols = kSensor; break;
    case MBOTS_EXPORT_STATS: p = t.stats.data(); cols = 4; break;
    case MBOTS_EXPORT_PREV_STATS: p = t.pstats.data(); cols = 4; break;
    case MBOTS_EXPORT_SENSOR_INDEX: sensor_index(sensor_index_.data()); p = sensor_index_.data(); break;
    case MBOTS_EXPORT_SPECIES_COUNT: p = scount_.data(); rows = Wx_; cols = kNumSpecies; break;
    case MBOTS_EXPORT_SPECIES: p = t.species.data(); break;
    case MBOTS_EXPORT_PREV_SPECIES: p = t.pspecies.data(); break;
    default: return MBOTS_E_INVALID;
    }
    out->data = p;
    out->dtype = dt;
    out->device = -1;
    out->dims[0] = rows;
    out->dims[1] = cols;
    return MBOTS_OK;
}

// learn/util.py:14-29 over all rows: depth | health bits | position | semantic | surrounding
void Sim::construct_obs(bool prev, float *out, uint64_t out_rows) const
{
    const Table &t = T_[tb_];
    const bool fixd = (cfg_.flags & MBOTS_FLAG_FIX_DEPTH_ALIAS) != 0;
    const int8_t *sem = prev ? t.psem.data() : t.sem.data();
    const uint8_t *dep = fixd ? (prev ? t.pdepth.data() : t.depth.data()) : reinterpret_cast<const uint8_t *>(sem);
    const int32_t *hp = prev ? t.phealth.data() : t.health.data();
    const float *pos = prev ? t.ppos.data() : t.pos.data();
    const float *sur = prev ? t.psur.data() : t.sur.data();
    const size_t n = std::min<uint64_t>(N_, out_rows);
    for (size_t r = 0; r < n; ++r) {
        float *o = out + r * 69;
        for (int k = 0; k < kSensor; ++k) o[k] = (float)dep[r * kSensor + k];
        o[32] = u2f((uint32_t)hp[r]);
        o[33] = pos[r * 2];
        o[34] = pos[r * 2 + 1];
        for (int k = 0; k < kSensor; ++k) o[35 + k] = (float)sem[r * kSensor + k];
        o[67] = sur[r * 2];
        o[68] = sur[r * 2 + 1];
    }
}

void Sim::world_state(uint32_t w, float *xy_rwrz, int32_t *sp_hp_finder, uint64_t *food,
                      uint32_t *food_rot, int32_t *n_out) const
{
    const size_t base = (size_t)w * cap_;
    for (uint32_t i = 0; i < cap_; ++i) {
        xy_rwrz[i * 4 + 0] = x_[base + i];
        xy_rwrz[i * 4 + 1] = y_[base + i];
        xy_rwrz[i * 4 + 2] = rw_[base + i];
        xy_rwrz[i * 4 + 3] = rz_[base + i];
        sp_hp_finder[i * 3 + 0] = species_[base + i];
        sp_hp_finder[i * 3 + 1] = health_[base + i];
        sp_hp_finder[i * 3 + 2] = finder_[base + i];
    }
    memcpy(food, &food_[(size_t)w * kNumChunks], kNumChunks * sizeof(uint64_t));
    if (food_rot) memcpy(food_rot, &food_rot_[(size_t)w * kNumPkg], kNumPkg * sizeof(uint32_t));
    *n_out = n_[w];
}

// ---- checkpoint: the config, every state array and the live table half ----
namespace {
constexpr char kMagic[8] = {'M', 'B', 'O', 'T', 'S', 'C', 'P', 'U'};
}  // namespace

#define MB_CPU_SLOT_ARRAYS(X)                                                                     \
    X(x_) X(y_) X(rw_) X(rz_) X(sur0_) X(sur1_) X(species_) X(health_) X(finder_) X(obsrow_)       \
    X(stats_)
#define MB_CPU_WORLD_ARRAYS(X)                                                                    \
    X(n_) X(cur_food_) X(scount_) X(row_base_) X(world_off_) X(key_) X(ctr_) X(overflow_)         \
    X(food_rot_) X(food_) X(sreward_)
#define MB_CPU_ARRAYS(X) MB_CPU_SLOT_ARRAYS(X) MB_CPU_WORLD_ARRAYS(X)
#define MB_CPU_TABLE(X)                                                                           \
    X(species) X(health) X(action) X(stats) X(pspecies) X(phealth) X(paction) X(pstats) X(pos)     \
    X(sur) X(reward) X(hidden) X(ppos) X(psur) X(preward) X(phidden) X(sem) X(psem) X(depth)      \
    X(pdepth)

uint64_t Sim::checkpoint_bytes() const
{
    uint64_t b = sizeof(kMagic) + sizeof(mbots_config) + sizeof(N_) + sizeof(totals_) + sizeof(agent_steps_);
#define X(v) b += v.size() * sizeof(v[0]);
    MB_CPU_ARRAYS(X)
#undef X
    const Table &t = T_[tb_];
#define X(c) b += t.c.size() * sizeof(t.c[0]);
    MB_CPU_TABLE(X)
#undef X
    return b;
}

int Sim::save(void *dst, uint64_t bytes, std::string &err) const
{
    if (bytes < checkpoint_bytes()) { err = "checkpoint buffer too small"; return MBOTS_E_INVALID; }
    char *p = static_cast<char *>(dst);
    auto w = [&](const void *s, size_t n) { memcpy(p, s, n); p += n; };
    w(kMagic, sizeof(kMagic));
    w(&cfg_, sizeof(cfg_));
    w(&N_, sizeof(N_));
    w(totals_, sizeof(totals_));
    w(&agent_steps_, sizeof(agent_steps_));
#define X(v) w(v.data(), v.size() * sizeof(v[0]));
    MB_CPU_ARRAYS(X)
#undef X
    const Table &t = T_[tb_];
#define X(c) w(t.c.data(), t.c.size() * sizeof(t.c[0]));
    MB_CPU_TABLE(X)
#undef X
    return MBOTS_OK;
}

int Sim::load(const void *src, uint64_t bytes, std::string &err)
{
    if (bytes < sizeof(kMagic) + sizeof(mbots_config)) { err = "checkpoint truncated"; return MBOTS_E_INVALID; }
    const char *p = static_cast<const char *>(src);
    if (memcmp(p, kMagic, sizeof(kMagic)) != 0) { err = "not a CPU-mode checkpoint"; return MBOTS_E_INVALID; }
    mbots_config c;
    memcpy(&c, p + sizeof(kMagic), sizeof(c));
    // (another agent_capacity is fine when every world of the blob fits this
    // one's: the per-slot arrays are re-laid out world by world, the table's
    // first N rows copied -- SimManager(agent_capacity="auto"))
    if (c.num_worlds != cfg_.num_worlds || c.agent_capacity < 4 || c.agent_capacity > (uint32_t)kMaxCap ||
        c.init_num_agents_per_world != cfg_.init_num_agents_per_world ||
        c.world_offset != cfg_.world_offset || c.flags != cfg_.flags || c.rand_seed != cfg_.rand_seed) {
        err = "checkpoint configuration differs from the manager's";
        return MBOTS_E_INVALID;
    }
    const size_t cap_src = c.agent_capacity;
    // bytes of array v in the blob: per-slot arrays and table columns scale
    // with the capacity, per-world arrays do not
    auto src_bytes = [&](size_t elems, size_t elem_bytes, bool per_slot) {
        return (per_slot ? elems / cap_ * cap_src : elems) * elem_bytes;
    };
    size_t need = sizeof(kMagic) + sizeof(mbots_config) + sizeof(N_) + sizeof(totals_) + sizeof(agent_steps_);
    size_t n_off = 0;
#define X(v) need += src_bytes(v.size(), sizeof(v[0]), true);
    MB_CPU_SLOT_ARRAYS(X)
#undef X
    n_off = need;
#define X(v) need += src_bytes(v.size(), sizeof(v[0]), false);
    MB_CPU_WORLD_ARRAYS(X)
#undef X
    const Table &t0 = T_[0];
#define X(c) need += src_bytes(t0.c.size(), sizeof(t0.c[0]), true);
    MB_CPU_TABLE(X)
#undef X
    if (bytes != need) { err = "checkpoint size mismatch"; return MBOTS_E_INVALID; }
    for (uint32_t w = 0; w < W_; ++w) {   // n_ leads the per-world arrays
        int32_t n;
        memcpy(&n, p + n_off + 4 * (size_t)w, 4);
        if (n < 0 || (size_t)n > cap_) {
            err = "a world of the checkpoint holds " + std::to_string(n) + " agents, more than agent_capacity " +
                  std::to_string(cap_);
            return MBOTS_E_INVALID;
        }
    }
    p += sizeof(kMagic) + sizeof(c);
    auto r = [&](void *d, size_t n) { memcpy(d, p, n); p += n; };
    r(&N_, sizeof(N_));
    r(totals_, sizeof(totals_));
    r(&agent_steps_, sizeof(agent_steps_));
    auto slot = [&](auto &v) {   // [world][cap_src] -> [world][cap_]
        using E = std::remove_reference_t<decltype(v[0])>;
        const size_t keep = std::min(cap_src, (size_t)cap_);
        for (size_t w = 0; w < v.size() / cap_; ++w) memcpy(&v[w * cap_], p + w * cap_src * sizeof(E), keep * sizeof(E));
        p += v.size() / cap_ * cap_src * sizeof(E);
    };
#define X(v) slot(v);
    MB_CPU_SLOT_ARRAYS(X)
#undef X
#define X(v) r(v.data(), v.size() * sizeof(v[0]));
    MB_CPU_WORLD_ARRAYS(X)
#undef X
    tb_ = 0;
    Table &t = T_[0];
    auto col = [&](auto &v) {   // the first N rows live; the rest stale
        using E = std::remove_reference_t<decltype(v[0])>;
        const size_t sb = v.size() / cap_ * cap_src * sizeof(E);
        memcpy(v.data(), p, std::min(sb, v.size() * sizeof(E)));
        p += sb;
    };
#define X(c) col(t.c);
    MB_CPU_TABLE(X)
#undef X
    return MBOTS_OK;
}

}  // namespace cpu
}  // namespace mbots
