#!/usr/bin/env python3
"""Build an s_memtime-instrumented K1 variant (scratch, never shipped): per-wave
cycles of K1's phases (staging, addFood, actionSystem, healthSync, surroundings,
speciesInfoSync + respawn, compaction, the block's tile atomics), summed into a
device array the variant .so exposes as mbots_dbg_read_stamps /
mbots_dbg_clear_stamps; scripts/k1stamps_probe.py reads it.  Relative shares
only (the stamps add waits of their own).

    python scripts/k1stamps_variant.py && MBOTS_LIB=build_var/libmbots_k1stamps.so python scripts/k1stamps_probe.py
"""
import os, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "madrona-bots_amd/csrc/mbots_kernels.hip")).read()


def rep(s, old, new, count=1):
    assert s.count(old) == count, (s.count(old), old[:70])
    return s.replace(old, new)


T = "__builtin_amdgcn_s_memtime()"
s = rep(src, "constexpr uint32_t kPkgLive = 1u << 8;", """__device__ unsigned long long g_stamps[16];
}
extern "C" int mbots_dbg_read_stamps(unsigned long long *out)
{
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(mbots::g_stamps), sizeof(unsigned long long) * 16);
}
extern "C" int mbots_dbg_clear_stamps()
{
    unsigned long long z[16] = {};
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(mbots::g_stamps), z, sizeof(z));
}
namespace mbots {
constexpr uint32_t kPkgLive = 1u << 8;""")
# kernel: stamp entry / after world_step / end
s = rep(s, """    const uint32_t w = uniform(blockIdx.x * kK1Worlds + wv);
    if (w < S.W) world_step(S, cur, lds[wv], w, lane);""", f"""    const uint32_t w = uniform(blockIdx.x * kK1Worlds + wv);
    unsigned long long ts[9];
    ts[0] = {T};
    for (int q = 1; q < 9; ++q) ts[q] = ts[0];
    if (w < S.W) world_step(S, cur, lds[wv], w, lane, ts);""")
s = rep(s, """            atomicAdd(&tiles[threadIdx.x * nent + tile * kTileBuckets + blockIdx.x % kTileBuckets], v);
        }
    }
}""", f"""            atomicAdd(&tiles[threadIdx.x * nent + tile * kTileBuckets + blockIdx.x % kTileBuckets], v);
        }}
    }}
    const unsigned long long tend = {T};
    if (lane == 0 && w < S.W) {{
        for (int q = 1; q < 8; ++q) atomicAdd(&g_stamps[q - 1], ts[q] - ts[q - 1]);
        atomicAdd(&g_stamps[7], tend - ts[7]);
        atomicAdd(&g_stamps[8], tend - ts[0]);
        atomicAdd(&g_stamps[9], 1ull);
    }}
}}""")
s = rep(s, """__device__ void world_step(SimState &S, const ObsTable &cur, WorldLDS<kCap> &L, uint32_t w,
                           uint32_t lane);""", """__device__ void world_step(SimState &S, const ObsTable &cur, WorldLDS<kCap> &L, uint32_t w,
                           uint32_t lane, unsigned long long *ts);""")
s = rep(s, """__device__ void world_step(SimState &S, const ObsTable &cur, WorldLDS<kCap> &L, uint32_t w,
                           uint32_t lane)
{""", """__device__ void world_step(SimState &S, const ObsTable &cur, WorldLDS<kCap> &L, uint32_t w,
                           uint32_t lane, unsigned long long *ts)
{""")
s = rep(s, """    if (lane == 0) L.consumed = 0;
    wave_sync();
""", f"""    if (lane == 0) L.consumed = 0;
    wave_sync();
    ts[1] = {T};
""")
s = rep(s, """        ctr += k;
    }

    // ---- actionSystem""", f"""        ctr += k;
    }}
    ts[2] = {T};

    // ---- actionSystem""")
s = rep(s, """    wave_sync();

    // ---- healthSync (sim.cpp:505-581) ----""", f"""    wave_sync();
    ts[3] = {T};

    // ---- healthSync (sim.cpp:505-581) ----""")
s = rep(s, """    wave_sync();
    cur_food -= L.consumed;
""", f"""    wave_sync();
    ts[4] = {T};
    cur_food -= L.consumed;
""")
s = rep(s, """    wave_sync();

    // ---- speciesInfoSync (sim.cpp:791-838) ----""", f"""    wave_sync();
    ts[5] = {T};

    // ---- speciesInfoSync (sim.cpp:791-838) ----""")
s = rep(s, """    if (n2 > (int)cap) { ovf += (uint32_t)(n2 - (int)cap); n2 = (int)cap; }
    wave_sync();
""", f"""    if (n2 > (int)cap) {{ ovf += (uint32_t)(n2 - (int)cap); n2 = (int)cap; }}
    wave_sync();
    ts[6] = {T};
""")
s = rep(s, """        S.cur_food[w] = cur_food;
        if (ovf) S.overflow[w] += ovf;
    }
}""", f"""        S.cur_food[w] = cur_food;
        if (ovf) S.overflow[w] += ovf;
    }}
    ts[7] = {T};
}}""")
os.makedirs(os.path.join(ROOT, "build_var"), exist_ok=True)
open("/tmp/mbots_k1stamps.hip", "w").write(s)
subprocess.run(["bash", os.path.join(ROOT, "scripts/build_var.sh"), "k1stamps", "/tmp/mbots_k1stamps.hip"],
               check=True)
