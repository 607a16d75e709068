"""TEST INFRASTRUCTURE ONLY: ctypes view of the C oracle (oracle/liborc.so).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
parity checker / CPU baseline.  The product package (madrona-bots_amd/) never
imports this module.  Parity status: see mbots_oracle.h ("parity unpinned" for
the Madrona-internal RNG/math/sensor; restated from cited reference lines
otherwise).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

NUM_SPECIES = 4
HIDDEN = 16
SENSOR = 32

COL_SPECIES, COL_POS, COL_HEALTH, COL_SURROUND, COL_REWARD, COL_ACTION, \
    COL_STATS, COL_HIDDEN, COL_SEMANTIC, COL_DEPTH = range(10)

_COL_SPEC = {
    COL_SPECIES: (np.int32, 1),
    COL_POS: (np.float32, 2),
    COL_HEALTH: (np.int32, 1),
    COL_SURROUND: (np.float32, 2),
    COL_REWARD: (np.float32, 1),
    COL_ACTION: (np.int32, 6),
    COL_STATS: (np.int32, 4),
    COL_HIDDEN: (np.float32, HIDDEN),
    COL_SEMANTIC: (np.int8, SENSOR),
    COL_DEPTH: (np.uint8, SENSOR),
}


class _Cfg(ctypes.Structure):
    _fields_ = [("num_worlds", ctypes.c_uint32), ("world_offset", ctypes.c_uint32),
                ("rand_seed", ctypes.c_uint32), ("init_agents", ctypes.c_uint32),
                ("cap", ctypes.c_uint32), ("reward_fixed", ctypes.c_uint32),
                ("num_threads", ctypes.c_uint32)]


def build():
    """Compile liborc.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liborc.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32
        L.orc_create.restype = vp
        L.orc_create.argtypes = [ctypes.POINTER(_Cfg)]
        L.orc_destroy.argtypes = [vp]
        L.orc_step.argtypes = [vp]
        L.orc_shift_observations.argtypes = [vp]
        L.orc_num_agents.restype = u32
        L.orc_num_agents.argtypes = [vp]
        L.orc_column.restype = vp
        L.orc_column.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        L.orc_species_count.restype = vp
        L.orc_species_count.argtypes = [vp]
        L.orc_world_counts.argtypes = [vp, vp, vp]
        L.orc_write_synthetic_actions.argtypes = [vp, u32, u32, ctypes.c_int]
        L.orc_sensor_index.argtypes = [vp, vp]
        L.orc_overflow.restype = u32
        L.orc_overflow.argtypes = [vp]
        L.orc_world_state.argtypes = [vp, u32, vp, vp, vp, vp, vp, vp]
        L.orc_world_food.restype = i32
        L.orc_world_food.argtypes = [vp, u32, vp]
        L.orc_threefry2x32.argtypes = [vp, vp, vp]
        L.orc_sample_uniform.restype = ctypes.c_float
        L.orc_sample_uniform.argtypes = [u32]
        L.orc_sample_i32.restype = i32
        L.orc_sample_i32.argtypes = [u32, i32, i32]
        f32 = ctypes.c_float
        L.orc_probe_box.argtypes = [f32, f32, f32, f32, f32, f32, u32, vp, vp]
        L.orc_probe_agent.argtypes = [f32, f32, f32, f32, f32, f32, vp, vp]
        L.orc_probe_walls.argtypes = [f32, f32, f32, f32, vp, vp]
        L.orc_action_hash.restype = u32
        L.orc_action_hash.argtypes = [u32, u32, u32, u32]
        _LIB = L
    return _LIB


def threefry2x32(key, ctr):
    k = (ctypes.c_uint32 * 2)(*key)
    c = (ctypes.c_uint32 * 2)(*ctr)
    o = (ctypes.c_uint32 * 2)()
    lib().orc_threefry2x32(k, c, o)
    return int(o[0]), int(o[1])


def probe_box(agent, heading, centre, rot):
    """Rays of one agent against one food box: (hit[33] bool, z[33] f32)."""
    hit = np.zeros(33, np.uint8)
    z = np.zeros(33, np.float32)
    lib().orc_probe_box(float(agent[0]), float(agent[1]), float(heading[0]), float(heading[1]),
                        float(centre[0]), float(centre[1]), int(rot), hit.ctypes.data,
                        z.ctypes.data)
    return hit.astype(bool), z


def probe_agent(agent, heading, centre):
    """Rays of one agent against another agent's disc: (hit[33] bool, z[33] f32)."""
    hit = np.zeros(33, np.uint8)
    z = np.zeros(33, np.float32)
    lib().orc_probe_agent(float(agent[0]), float(agent[1]), float(heading[0]), float(heading[1]),
                          float(centre[0]), float(centre[1]), hit.ctypes.data, z.ctypes.data)
    return hit.astype(bool), z


def probe_walls(agent, heading):
    """Rays of a lone agent against the walls: (sem[33] int8: 5 wall / -1 miss,
    depth[33] uint8), the finder ray last."""
    sem = np.zeros(33, np.int8)
    dep = np.zeros(33, np.uint8)
    lib().orc_probe_walls(float(agent[0]), float(agent[1]), float(heading[0]), float(heading[1]),
                          sem.ctypes.data, dep.ctypes.data)
    return sem, dep


class OracleSim:
    """CPU restatement with the SimManager-shaped surface (numpy arrays)."""

    def __init__(self, num_worlds, rand_seed, init_num_agents_per_world, cap=128,
                 world_offset=0, reward_fixed=False, num_threads=1):
        self.num_worlds = int(num_worlds)
        self.cap = int(cap)
        cfg = _Cfg(num_worlds, world_offset, rand_seed, init_num_agents_per_world, cap,
                   1 if reward_fixed else 0, num_threads)
        self._destroy = lib().orc_destroy
        self._h = lib().orc_create(ctypes.byref(cfg))
        if not self._h:
            raise MemoryError("orc_create failed")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._destroy(h)   # (held by the object: module globals are gone at interpreter exit)
            self._h = None

    def step(self):
        lib().orc_step(self._h)

    def shift_observations(self):
        lib().orc_shift_observations(self._h)

    def num_agents(self):
        return int(lib().orc_num_agents(self._h))

    def column(self, col, is_prev=False):
        dt, k = _COL_SPEC[col]
        n = self.num_agents()
        ptr = lib().orc_column(self._h, col, 1 if is_prev else 0)
        nbytes = n * k * np.dtype(dt).itemsize
        buf = (ctypes.c_char * max(nbytes, 1)).from_address(ptr)
        return np.frombuffer(buf, dtype=dt, count=n * k).reshape(n, k)

    def species_count(self):
        ptr = lib().orc_species_count(self._h)
        buf = (ctypes.c_int32 * (self.num_worlds * 4)).from_address(ptr)
        return np.frombuffer(buf, dtype=np.int32).reshape(self.num_worlds, 4)

    def world_counts(self):
        c = np.zeros(self.num_worlds, np.int32)
        o = np.zeros(self.num_worlds, np.int32)
        lib().orc_world_counts(self._h, c.ctypes.data, o.ctypes.data)
        return c, o

    def sensor_index(self):
        out = np.zeros(self.num_agents(), np.int32)
        lib().orc_sensor_index(self._h, out.ctypes.data)
        return out

    def write_synthetic_actions(self, seed, step, write_hidden=False):
        lib().orc_write_synthetic_actions(self._h, seed, step, 1 if write_hidden else 0)

    def overflow(self):
        return int(lib().orc_overflow(self._h))

    def world_state(self, w):
        xy = np.zeros((self.cap, 2), np.float32)
        rot = np.zeros((self.cap, 2), np.float32)
        sp = np.zeros(self.cap, np.int32)
        hp = np.zeros(self.cap, np.int32)
        fd = np.zeros(self.cap, np.int32)
        n = ctypes.c_int32()
        lib().orc_world_state(self._h, w, xy.ctypes.data, rot.ctypes.data, sp.ctypes.data,
                              hp.ctypes.data, fd.ctypes.data, ctypes.byref(n))
        k = n.value
        food = np.zeros((240, 4), np.int32)
        nf = int(lib().orc_world_food(self._h, w, food.ctypes.data))
        return dict(xy=xy[:k], rot=rot[:k], species=sp[:k], health=hp[:k], finder=fd[:k],
                    food=food[:nf].copy())

    def snapshot(self, include_prev=True):
        """Copy of every exported column (dict name -> array)."""
        names = ["species", "pos", "health", "surround", "reward", "action", "stats",
                 "hidden", "semantic", "depth"]
        out = {}
        for i, nm in enumerate(names):
            out[nm] = self.column(i).copy()
            if include_prev:
                out["prev_" + nm] = self.column(i, True).copy()
        out["species_count"] = self.species_count().copy()
        return out
