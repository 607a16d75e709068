"""CPU: the C ABI from a C99 host (tests/c_host/host.c, built here with gcc
-std=c99 -pedantic -Werror against include/mbots.h and libmbots.so) gives the
same exported bytes as the same calls through madrona_bots (MBOTS_EXEC_CPU)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "madrona-bots_amd", "madrona_bots")

IDS = ("action", "reward", "position", "prev_position", "health", "surrounding", "semantic",
       "prev_semantic", "stats", "species_count")


def _fnv1a(chunks):
    h = 1469598103934665603
    for b in chunks:
        for x in b:
            h ^= x
            h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def _views(m):
    get = {"action": lambda: m.action_tensor(False), "reward": lambda: m.reward_tensor(False),
           "position": lambda: m.position_tensor(False), "prev_position": lambda: m.position_tensor(True),
           "health": lambda: m.health_tensor(False), "surrounding": lambda: m.surrounding_tensor(False),
           "semantic": lambda: m.semantic_tensor(False), "prev_semantic": lambda: m.semantic_tensor(True),
           "stats": lambda: m.stats_tensor(False), "species_count": lambda: m.species_count_tensor()}
    return [np.ascontiguousarray(get[k]().to_torch().numpy()).tobytes() for k in IDS]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no C compiler")
def test_c_host_matches_python_surface(tmp_path):
    exe = tmp_path / "host"
    subprocess.run(["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-O1",
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "c_host", "host.c"),
                    "-L", LIBDIR, "-lmbots", "-Wl,-rpath," + LIBDIR, "-o", str(exe)], check=True)
    W, T = 16, 6
    out = subprocess.run([str(exe), str(W), str(T)], check=True, capture_output=True, text=True).stdout.split()
    import madrona_bots as mb
    m = mb.SimManager(0, W, 69, 32, exec_mode="cpu")
    for t in range(T):
        m.write_synthetic_actions(1234, t, True)
        m.step()
        if t + 1 < T:
            m.shift_observations()
    assert out[:2] == ["agents", str(m.num_agents())]
    assert int(out[3], 16) == _fnv1a(_views(m))


@pytest.mark.gpu
@pytest.mark.parametrize("W", [16, 4100])
def test_c_host_hip_equals_cpu(tmp_path, W):
    """The same C host on MBOTS_EXEC_HIP (device views copied out with
    hipMemcpy) prints the CPU mode's digest: K1-finder mode at 16 worlds, the
    joined schedule with its value waits at 4100."""
    exe = tmp_path / "host_hip"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-O1", "-D__HIP_PLATFORM_AMD__", "-DMBOTS_HOST_HIP",
                    "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                    os.path.join(ROOT, "tests", "c_host", "host.c"),
                    "-L", LIBDIR, "-lmbots", "-L", "/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath," + LIBDIR + ":/opt/rocm/lib", "-o", str(exe)], check=True)
    run = lambda mode: subprocess.run([str(exe), str(W), "8", mode], check=True, capture_output=True,
                                      text=True, timeout=120).stdout.split()
    cpu, hip = run("cpu"), run("hip")
    assert hip == cpu, (hip, cpu)
