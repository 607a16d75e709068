#!/usr/bin/env python3
"""Build a shader-clock probe variant (scratch, never shipped): every wave of
K1, K3a, the sensor, the fused shift and the action writer stores s_memtime
(shader clock ticks) and s_memrealtime (100 MHz) at its start and end, so
(d memtime / d realtime) x 100 MHz is the clock each wave ran at
(MI355X_MICROARCH.md "DVFS give-back", item 6) -- in the overlapped,
unprofiled step.  The variant .so exports mbots_dbg_clock_read; read by
scripts/clockprobe.py.

    python scripts/clockprobe_variant.py && MBOTS_LIB=build_var/libmbots_clockprobe.so python scripts/clockprobe.py
"""
import os, re, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "madrona-bots_amd/csrc/mbots_kernels.hip")).read()
KINDS = ["world_step_kernel", "export_rows_kernel", "sensor_kernel", "shift_move_kernel",
         "synthetic_actions_kernel"]
NW = 1 << 17
s = src.replace("namespace mbots {\n\nconstexpr int kWorldsPerBlock = 4;", """namespace mbots {
__device__ unsigned long long g_ck[5][4][%d];   // [kind][t0 real, t1 real, t0 clk, t1 clk][wave]
struct ClockWave {
    int k;
    unsigned long long r0, c0;
    __device__ static unsigned idx()
    {
        return ((blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    }
    __device__ explicit ClockWave(int k_) : k(k_)
    {
        r0 = __builtin_amdgcn_s_memrealtime();
        c0 = __builtin_amdgcn_s_memtime();
    }
    __device__ ~ClockWave()
    {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime();
        const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63u) == 0 && idx() < %du) {
            g_ck[k][0][idx()] = r0; g_ck[k][1][idx()] = r1;
            g_ck[k][2][idx()] = c0; g_ck[k][3][idx()] = c1;
        }
    }
};
}
extern "C" int mbots_dbg_clock_read(unsigned long long *out)
{
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(mbots::g_ck), sizeof(mbots::g_ck));
}
namespace mbots {

constexpr int kWorldsPerBlock = 4;""" % (NW, NW), 1)
assert s != src
for k, name in enumerate(KINDS):
    pat = re.compile(r"(void %s\([^)]*\)\s*\{)" % name, re.S)
    s, n = pat.subn(lambda m: m.group(1) + "\n    ClockWave _clk(%d);" % k, s, count=1)
    assert n == 1, name
os.makedirs(os.path.join(ROOT, "build_var"), exist_ok=True)
open("/tmp/k_clockprobe.hip", "w").write(s)
subprocess.check_call(["bash", os.path.join(ROOT, "scripts/build_var.sh"), "clockprobe", "/tmp/k_clockprobe.hip"])
print("built build_var/libmbots_clockprobe.so")
