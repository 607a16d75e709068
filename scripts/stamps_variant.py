#!/usr/bin/env python3
"""Build an s_memtime-instrumented sensor variant (scratch, never shipped):
per-wave cycles of staging, P1 (cull), P2 (survivor batches + wide pairs) and
the output pass, summed into a device array that the variant .so exposes as
mbots_dbg_read_stamps / mbots_dbg_clear_stamps; scripts/stamps_probe.py reads
it.  Relative shares only (the stamps add waits of their own).

    python scripts/stamps_variant.py && MBOTS_LIB=build_var/libmbots_stamps.so python scripts/stamps_probe.py
"""
import os, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "madrona-bots_amd/csrc/mbots_kernels.hip")).read()


def rep(s, old, new):
    assert s.count(old) >= 1, old[:70]
    return s.replace(old, new)


s = rep(src, "namespace mbots {\n\nconstexpr int kWorldsPerBlock = 4;", """namespace mbots {
__device__ unsigned long long g_stamps[8];
}
extern "C" int mbots_dbg_read_stamps(unsigned long long *out)
{
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(mbots::g_stamps), sizeof(unsigned long long) * 8);
}
extern "C" int mbots_dbg_clear_stamps()
{
    unsigned long long z[8] = {};
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(mbots::g_stamps), z, sizeof(z));
}
namespace mbots {

constexpr int kWorldsPerBlock = 4;""")
s = rep(s, """template <class LDS>
__device__ __forceinline__ void run_survivors(LDS &L, int nf, int a0, int q0, int cnt)
{
    const int lane = (int)__lane_id();""", """template <class LDS>
__device__ __forceinline__ void run_survivors(LDS &L, int nf, int a0, int q0, int cnt, unsigned long long &p2t)
{
    const unsigned long long t_in = __builtin_amdgcn_s_memtime();
    const int lane = (int)__lane_id();""")
s = rep(s, """        run_wide(L, nf, a0, q0, nw);
        wave_sync();
    }
}""", """        run_wide(L, nf, a0, q0, nw);
        wave_sync();
    }
    p2t += __builtin_amdgcn_s_memtime() - t_in;
}""")
s = rep(s, "run_survivors(L, nf, a0, nq - 64, 64);", "run_survivors(L, nf, a0, nq - 64, 64, p2t);")
s = rep(s, "run_survivors(L, nf, a0, 0, nq);", "run_survivors(L, nf, a0, 0, nq, p2t);")
s = rep(s, """    SensorPrefetch pf;
    sensor_prefetch(S, w, lane, pf);""", """    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long p2t = 0, t_out = 0, t_p1 = 0;
    SensorPrefetch pf;
    sensor_prefetch(S, w, lane, pf);""")
s = rep(s, """    const int nobj = nf + n;
    wave_sync();

    for (int a0 = kChunk0; a0 < n; a0 += kChunkStep) {""", """    const int nobj = nf + n;
    wave_sync();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();

    for (int a0 = kChunk0; a0 < n; a0 += kChunkStep) {
        const unsigned long long tc = __builtin_amdgcn_s_memtime();""")
s = rep(s, """        wave_sync();
        // ---- output: keys vs walls; lane = (agent ci, pixels 4g .. 4g+3) ----""", """        wave_sync();
        const unsigned long long to = __builtin_amdgcn_s_memtime();
        t_p1 += to - tc;
        // ---- output: keys vs walls; lane = (agent ci, pixels 4g .. 4g+3) ----""")
s = rep(s, """            S.finder[base + i] = agent ? (int32_t)(order - kOrderAgent) : -1;
        }
        wave_sync();
    }
    }
}""", """            S.finder[base + i] = agent ? (int32_t)(order - kOrderAgent) : -1;
        }
        wave_sync();
        t_out += __builtin_amdgcn_s_memtime() - to;
    }
    if (lane == 0) {
        atomicAdd(&g_stamps[0], (unsigned long long)(t1 - t0));
        atomicAdd(&g_stamps[1], t_p1 - p2t);
        atomicAdd(&g_stamps[2], p2t);
        atomicAdd(&g_stamps[3], t_out);
        atomicAdd(&g_stamps[4], (unsigned long long)(__builtin_amdgcn_s_memtime() - t0));
        atomicAdd(&g_stamps[5], 1ull);
    }
    }
}""")
os.makedirs(os.path.join(ROOT, "build_var"), exist_ok=True)
open("/tmp/mbots_stamps.hip", "w").write(s)
subprocess.run(["bash", os.path.join(ROOT, "scripts/build_var.sh"), "stamps", "/tmp/mbots_stamps.hip"], check=True)
