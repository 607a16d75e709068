#!/usr/bin/env python3
"""Build a kernel-timeline probe variant (scratch, never shipped): every wave of
K1, K2, K3a, the sensor, the fused shift and the action writer stores its
start / end s_memrealtime (100 MHz, chip-wide) into a per-kernel array indexed
by its wave, so after a run the arrays hold the last launch of each kernel --
the unprofiled step's kernel spans and the gaps between them.  The variant .so
exports mbots_dbg_probe_read; scripts/tlprobe.py reads it.

    python scripts/tlprobe_variant.py && MBOTS_LIB=build_var/libmbots_tlprobe.so python scripts/tlprobe.py
"""
import os, re, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "madrona-bots_amd/csrc/mbots_kernels.hip")).read()
KINDS = ["world_step_kernel", "scan_kernel", "export_rows_kernel", "sensor_kernel",
         "shift_move_kernel", "synthetic_actions_kernel"]
NW = 1 << 17

s = src.replace("namespace mbots {\n\nconstexpr int kWorldsPerBlock = 4;", """namespace mbots {
__device__ unsigned long long g_pt0[6][%d], g_pt1[6][%d];
struct ProbeWave {   // stamps stored at once: nothing stays live across the kernel
    int k;
    __device__ static unsigned idx()
    {
        return ((blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    }
    __device__ explicit ProbeWave(int k_) : k(k_)
    {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63u) == 0 && idx() < %du) g_pt0[k][idx()] = t;
    }
    __device__ ~ProbeWave()
    {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63u) == 0 && idx() < %du) g_pt1[k][idx()] = t;
    }
};
}
extern "C" int mbots_dbg_probe_read(unsigned long long *t0, unsigned long long *t1)
{
    int rc = (int)hipMemcpyFromSymbol(t0, HIP_SYMBOL(mbots::g_pt0), sizeof(mbots::g_pt0));
    if (rc == 0) rc = (int)hipMemcpyFromSymbol(t1, HIP_SYMBOL(mbots::g_pt1), sizeof(mbots::g_pt1));
    return rc;
}
namespace mbots {

constexpr int kWorldsPerBlock = 4;""" % (NW, NW, NW, NW), 1)
assert s != src
# a ProbeWave at the top of each probed kernel body (its destructor runs on every return)
for k, name in enumerate(KINDS):
    pat = re.compile(r"(void %s\([^)]*\)\s*\{)" % name, re.S)
    s, n = pat.subn(lambda m: m.group(1) + "\n    ProbeWave _probe(%d);" % k, s, count=1)
    assert n == 1, name
d = os.path.join(ROOT, "build_var")
os.makedirs(d, exist_ok=True)
open("/tmp/k_tlprobe.hip", "w").write(s)
subprocess.check_call(["bash", os.path.join(ROOT, "scripts/build_var.sh"), "tlprobe", "/tmp/k_tlprobe.hip"])
print("built build_var/libmbots_tlprobe.so")
