// mbots_cpu.hpp -- the CPU execution mode (ExecMode::CPU of the reference's
// Manager, BASELINE config 1: learn/env.py picks it when no GPU is present).
//
// The same world step as the HIP kernels -- identical float expressions (the
// shared host+device helpers of mbots_device.hpp / mbots_ray.hpp), identical
// state layout (SoA [world][slot] agent columns, packed per-chunk food
// records, a double-buffered species-major export table) -- run world-parallel
// on host threads.  Results are bit-identical to the HIP path.  Moves are eager
// (no deferred Prev* columns): the CPU mode is the plumbing configuration.
#pragma once

#include "../../include/mbots.h"
#include "mbots_device.hpp"

#include <cstdint>
#include <string>
#include <vector>

namespace mbots {
namespace cpu {

// one half of the export table (types.hpp:228-252 + the raycast outputs)
struct Table {
    std::vector<int32_t> species, health, action, stats, pspecies, phealth, paction, pstats;
    std::vector<float> pos, sur, reward, hidden, ppos, psur, preward, phidden;
    std::vector<int8_t> sem, psem;
    std::vector<uint8_t> depth, pdepth;
    void resize(size_t rows);
};

class Sim {
public:
    explicit Sim(const mbots_config &cfg);

    void step();
    void shift_observations();
    void write_synthetic_actions(uint32_t seed, uint32_t step, bool write_hidden);
    int export_tensor(int32_t id, mbots_tensor *out);
    void construct_obs(bool prev, float *out, uint64_t out_rows) const;
    void sensor_index(int32_t *out) const;
    uint32_t num_agents() const { return N_; }
    // every table row: N plus the shard ghost's (which follow row N)
    uint32_t num_rows() const { return N_ + (W_ > Wx_ ? (uint32_t)n_[Wx_] : 0u); }
    uint32_t max_population() const
    {
        int32_t m = 0;
        for (int32_t v : n_) m = v > m ? v : m;
        return (uint32_t)m;
    }
    uint32_t world_offset_of(uint32_t w) const { return (uint32_t)world_off_[w]; }
    uint64_t agent_steps() const { return agent_steps_; }
    uint64_t overflow() const;
    Table &table() { return T_[tb_]; }
    // each export row's row in the table before the last step (-1: new), like
    // the HIP path's src_of (slim learner records)
    const int32_t *src_of() const { return src_of_.data(); }
    void world_state(uint32_t w, float *xy_rwrz, int32_t *sp_hp_finder, uint64_t *food,
                     uint32_t *food_rot, int32_t *n_out) const;
    uint64_t checkpoint_bytes() const;
    int save(void *dst, uint64_t bytes, std::string &err) const;
    int load(const void *src, uint64_t bytes, std::string &err);
    const mbots_config &config() const { return cfg_; }

private:
    template <typename F> void for_worlds(F &&fn) const;
    void init_world(uint32_t w);
    void world_step(uint32_t w, const Table &cur);
    void scan();
    void export_world(uint32_t w, const Table &cur, Table &nxt, bool init);
    // agents [lo, hi) of world w (hi < 0: all of them)
    void sensor_world(uint32_t w, Table &nxt, int lo = 0, int hi = -1);
    void sensor_by_agents(Table &nxt);

    mbots_config cfg_;
    uint32_t W_, Wx_, cap_, A_;   // simulated / exported worlds (W_ = Wx_ + the shard ghost)
    unsigned threads_;
    // agent state, [W][cap] (slot order = creation order, survivors compacted)
    std::vector<float> x_, y_, rw_, rz_, sur0_, sur1_;
    std::vector<int32_t> species_, health_, finder_, obsrow_;
    std::vector<uint32_t> stats_;
    // per world
    std::vector<int32_t> n_, cur_food_, scount_, row_base_, world_off_;
    std::vector<uint2> key_;
    std::vector<uint32_t> ctr_, overflow_, food_rot_;
    std::vector<uint64_t> food_;
    std::vector<float> sreward_;
    Table T_[2];
    int tb_ = 0;
    uint32_t N_ = 0;
    uint32_t totals_[5] = {};
    uint64_t agent_steps_ = 0;
    std::vector<int32_t> zeros_rows_, zeros_worlds_, sensor_index_, src_of_;
};

}  // namespace cpu
}  // namespace mbots
