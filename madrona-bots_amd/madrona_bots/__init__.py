"""madrona_bots -- MI355X-native drop-in for the reference's Python module.

Mirrors the nanobind surface of src/entry/entry.cpp:16-45:

    SimManager(gpu_id, num_worlds, rand_seed, init_num_agents_per_world)
        .step()  .shift_observations()
        .depth_tensor(is_prev)  .semantic_tensor(is_prev)  .reward_tensor(is_prev)
        .species_count_tensor() .position_tensor(is_prev)  .health_tensor(is_prev)
        .surrounding_tensor(is_prev)  .action_tensor(is_prev)
        .stats_tensor(is_prev)  .hidden_state_tensor(is_prev)

Each accessor returns a ``Tensor`` whose ``to_torch()`` is a zero-copy torch
view of memory owned by the manager (madrona::py::Tensor, mgr.cpp:70-76).
The simulation runs in libmbots.so: hand-written gfx950 kernels
(``exec_mode="hip"``, the default) or, for ``exec_mode="cpu"``
(madrona::ExecMode::CPU; learn/env.py:12-15 picks it without a GPU), the same
world step on host threads with bit-identical results and host tensor views.
Importing without the built library raises ImportError; a HIP-mode manager
without a GPU raises RuntimeError (no silent fallback).
"""
import ctypes
import os
import types
import warnings

import torch  # loads the HIP runtime libmbots.so links against (same soname)

__all__ = ["SimManager", "ScriptBotsViewer", "Tensor", "madrona", "ExportID", "ExecMode", "unpack_rollout",
           "unpack_learner", "rebuild_learner", "CapacityWarning", "CapacityError", "MAX_CAPACITY",
           "CAPACITY_CLASSES"]

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libmbots.so")

if not os.path.exists(_LIB_PATH):
    raise ImportError(
        f"madrona_bots: {_LIB_PATH} is missing; build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")


class _Config(ctypes.Structure):
    _fields_ = [("gpu_id", ctypes.c_int32), ("num_worlds", ctypes.c_uint32),
                ("rand_seed", ctypes.c_uint32), ("init_num_agents_per_world", ctypes.c_uint32),
                ("sensor_size", ctypes.c_uint32), ("world_offset", ctypes.c_uint32),
                ("agent_capacity", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("exec_mode", ctypes.c_int32)]


class _LearnerOut(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in
                ("obs", "prev_obs", "reward", "stats", "action", "hidden", "prev_hidden")]


class _CTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("dtype", ctypes.c_int32), ("device", ctypes.c_int32),
                ("dims", ctypes.c_int64 * 2)]


def _load():
    L = ctypes.CDLL(_LIB_PATH)
    vp, i32, u32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32
    P = ctypes.POINTER
    sig = {
        "mbots_create": [P(_Config), P(vp)],
        "mbots_destroy": [vp],
        "mbots_step": [vp, vp],
        "mbots_shift_observations": [vp, vp],
        "mbots_num_agents": [vp, P(u32)],
        "mbots_construct_obs": [vp, i32, vp, ctypes.c_uint64, vp],
        "mbots_checkpoint_size": [vp, P(ctypes.c_uint64)],
        "mbots_save_checkpoint": [vp, vp, ctypes.c_uint64],
        "mbots_load_checkpoint": [vp, vp, ctypes.c_uint64],
        "mbots_world_state": [vp, u32, vp, vp, vp, vp, P(i32)],
        "mbots_export": [vp, i32, P(_CTensor)],
        "mbots_export_on": [vp, i32, vp, P(_CTensor)],
        "mbots_set_action": [vp, u32, P(i32)],
        "mbots_agent_offset_for_world": [vp, u32, P(u32)],
        "mbots_write_synthetic_actions": [vp, u32, u32, i32, vp],
        "mbots_join": [vp, vp],
        "mbots_record_sensor_done": [vp, vp],
        "mbots_rollout_record_bytes": [vp, P(u32)],
        "mbots_pack_rollout": [vp, vp, ctypes.c_uint64, vp],
        "mbots_unpack_rollout": [vp, ctypes.c_uint64, i32, i32, vp, vp, vp, vp],
        "mbots_learner_record_bytes": [vp, P(u32)],
        "mbots_pack_learner": [vp, vp, ctypes.c_uint64, vp],
        "mbots_unpack_learner": [vp, ctypes.c_uint64, i32, i32, P(_LearnerOut), vp],
        "mbots_pack_learner_slim": [vp, vp, ctypes.c_uint64, vp],
        "mbots_unpack_learner_slim": [vp, ctypes.c_uint64, i32, i32, P(_LearnerOut), vp, vp],
        "mbots_rebuild_learner": [vp, ctypes.c_uint64, vp, vp, u32, vp, vp, vp, ctypes.c_uint64, vp, vp, vp,
                                  i32, vp],
        "mbots_write_actions": [vp, vp, vp, ctypes.c_uint64, vp],
        "mbots_num_rows": [vp, P(u32)],
        "mbots_agent_steps": [vp, P(ctypes.c_uint64)],
        "mbots_overflow": [vp, P(ctypes.c_uint64)],
        "mbots_enable_kernel_timing": [vp, i32],
        "mbots_kernel_times": [vp, P(ctypes.c_double), P(ctypes.c_uint64)],
        "mbots_schedule_info": [vp, P(u32)],
        "mbots_max_population": [vp, P(u32)],
    }
    for name, args in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    L.mbots_last_error.restype = ctypes.c_char_p
    L.mbots_last_error.argtypes = []
    return L


_lib = _load()


def _check(rc):
    if rc != 0:
        msg = _lib.mbots_last_error().decode(errors="replace")
        raise (CapacityError if rc == _E_CAPACITY else RuntimeError)(f"madrona_bots: {msg} (status {rc})")


_W_CAPACITY, _E_CAPACITY = 1, -5   # include/mbots.h MBOTS_W_CAPACITY / MBOTS_E_CAPACITY
MAX_CAPACITY = 4096                # MBOTS_MAX_CAPACITY
CAPACITY_CLASSES = (128, 256, 512, 1024, 2048, 4096)   # the kernels' slot classes


def _capacity_class(need):
    """The smallest kernel capacity class holding `need` agents (the largest
    class when none does)."""
    for c in CAPACITY_CLASSES:
        if need <= c:
            return c
    return MAX_CAPACITY


class CapacityWarning(RuntimeWarning):
    """Births or respawns were dropped because a world reached agent_capacity:
    the reference's worlds have no cap (sim.cpp:561-564, :830-834), so the run
    now differs from the reference's (MBOTS_W_CAPACITY)."""


class CapacityError(RuntimeError):
    """CapacityWarning under strict_capacity=True (MBOTS_E_CAPACITY); the step ran."""


class ExportID:
    """enum class ExportID (src/sim/sim.hpp:18-55) + build extensions."""
    Reset, Action, PrevAction, HiddenState, PrevHiddenState, Reward, PrevReward, Done, \
        Position, PrevPosition, Health, PrevHealth, Surrounding, PrevSurrounding, \
        SensorSemantic, SensorDepth, PrevSensorSemantic, PrevSensorDepth, Stats, PrevStats, \
        SensorIndex, SpeciesCount = range(22)
    Species, PrevSpecies = 32, 33


_DTYPES = {0: (torch.uint8, "|u1"), 1: (torch.int8, "|i1"), 2: (torch.int32, "<i4"),
           3: (torch.float32, "<f4")}
_DTYPE_CODE = {v[0]: k for k, v in _DTYPES.items()}


def _raw_stream(device):
    """hipStream_t of torch's current stream on `device` (no Stream object)."""
    return torch._C._cuda_getCurrentRawStream(device)

FLAG_REWARD_FIXED = 0x1
FLAG_FIX_DEPTH_ALIAS = 0x2
FLAG_SHARD_GHOST = 0x4
FLAG_STRICT_CAPACITY = 0x8


class ExecMode:
    """madrona::ExecMode (MBOTS_EXEC_*)."""
    CUDA = HIP = 0
    CPU = 1


def _exec_mode(v):
    if isinstance(v, str):
        v = {"hip": ExecMode.HIP, "cuda": ExecMode.HIP, "gpu": ExecMode.HIP,
             "cpu": ExecMode.CPU}.get(v.lower())
        if v is None:
            raise ValueError("exec_mode must be 'hip' or 'cpu'")
    v = int(v)
    if v not in (ExecMode.HIP, ExecMode.CPU):
        raise ValueError(f"unknown exec_mode {v}")
    return v


OBS_DIM = 69   # learn/env.py:19
# TK_* indices of mbots_kernel_times
KERNELS = ("world_step", "scan", "export", "sensor", "shift", "actions", "move", "obs")


class _Handle:
    """One manager's library handle (mbots_create / mbots_destroy).  Every
    exported view holds it -- a torch view's storage holds the Tensor whose
    array interface it was built from, and that Tensor holds this -- so a view
    outlives the SimManager that produced it.  The manager's view
    cache holds views, which hold this handle and never the manager, so there
    is no reference cycle: the device memory is freed by reference counting
    once the manager and every view of it are gone."""
    __slots__ = ("h",)

    def __init__(self, h):
        self.h = h

    def __del__(self):
        h = self.h
        if h and _lib is not None:   # module globals may be gone at interpreter exit
            _lib.mbots_destroy(h)
            self.h = None


class Tensor:
    """Non-owning device tensor view (madrona::py::Tensor)."""

    def __init__(self, keep, ct, column=False, mgr=None):
        self._keep = keep            # the manager's _Handle: keeps its memory alive
        self._mgr = mgr              # the manager (its view cache), for table columns
        self._column = column        # a table column: W x cap row slots behind it
        self._ptr = int(ct.data or 0)
        self._torch_dtype, self._typestr = _DTYPES[ct.dtype]
        self._device = int(ct.device)
        self.shape = (int(ct.dims[0]), int(ct.dims[1]))

    def devicePtr(self):
        return self._ptr

    @property
    def dtype(self):
        return self._torch_dtype

    @property
    def __cuda_array_interface__(self):
        return {"shape": self.shape, "typestr": self._typestr, "data": (self._ptr, False),
                "version": 3, "strides": None, "stream": None}

    def to_torch(self):
        """Zero-copy torch view on cuda:<gpu_id> (host memory in CPU mode)."""
        if self._device < 0:
            return self._host_view()
        dev = torch.device("cuda", self._device)
        if self.shape[0] == 0:
            return torch.empty(self.shape, dtype=self._torch_dtype, device=dev)
        # one torch view per column allocation, sliced to the current row count:
        # the learner reads ~10 views per step and is host-bound at small world
        # counts (scripts/refhost.py); building a view from the array interface
        # every time is most of an accessor's host cost
        # (a view taken before an agent_capacity="auto" growth belongs to the
        # manager's previous storage: no cached view of the current one)
        base = self._mgr._view_cache(self) if (self._column and self._mgr is not None
                                                and self._keep is self._mgr._hd) else None
        if base is not None:
            return base[:self.shape[0]]
        t = torch.as_tensor(self, device=dev)
        if t.data_ptr() != self._ptr:
            raise RuntimeError("madrona_bots: to_torch() produced a copy, expected a view")
        return t

    def _host_view(self):
        import numpy as np
        npdt = {torch.uint8: np.uint8, torch.int8: np.int8, torch.int32: np.int32,
                torch.float32: np.float32}[self._torch_dtype]
        n = self.shape[0] * self.shape[1]
        if n == 0:
            return torch.empty(self.shape, dtype=self._torch_dtype)
        buf = (ctypes.c_char * (n * np.dtype(npdt).itemsize)).from_address(self._ptr)
        buf._keep = self._keep       # the view (numpy base -> buffer) keeps the manager's memory
        t = torch.from_numpy(np.frombuffer(buf, dtype=npdt, count=n).reshape(self.shape))
        if t.data_ptr() != self._ptr:
            raise RuntimeError("madrona_bots: to_torch() produced a copy, expected a view")
        return t


def unpack_rollout(records, with_depth=None):
    """Learner side of the config-5 gather: uint8 [N, 64 | 96] rollout records
    (SimManager.pack_rollout, gathered from every rank) -> {"obs": float32
    [N, 69] (construct_obs, bit-identical), "reward": float32 [N, 1],
    "stats": int32 [N, 4]} on the records' device (mbots_unpack_rollout)."""
    if records.dtype != torch.uint8 or records.dim() != 2 or records.shape[1] not in (64, 96):
        raise ValueError("records must be uint8 [N, 64] or [N, 96]")
    depth = records.shape[1] == 96 if with_depth is None else bool(with_depth)
    if depth != (records.shape[1] == 96):
        raise ValueError("with_depth does not match the record width")
    rec = records.contiguous()
    n = rec.shape[0]
    dev = rec.device
    obs = torch.empty((n, OBS_DIM), dtype=torch.float32, device=dev)
    rew = torch.empty((n, 1), dtype=torch.float32, device=dev)
    st = torch.empty((n, 4), dtype=torch.int32, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else None)
    _check(_lib.mbots_unpack_rollout(ctypes.c_void_p(rec.data_ptr()), n, 1 if depth else 0,
                                     dev.index if dev.type == "cuda" else -1,
                                     ctypes.c_void_p(obs.data_ptr()), ctypes.c_void_p(rew.data_ptr()),
                                     ctypes.c_void_p(st.data_ptr()), stream))
    return {"obs": obs, "reward": rew, "stats": st}


LEARNER_BYTES, LEARNER_BYTES_DEPTH = 272, 336
LEARNER_SLIM_BYTES, LEARNER_SLIM_BYTES_DEPTH = 128, 192
_LEARNER_KEYS = ("obs", "prev_obs", "reward", "stats", "action", "hidden", "prev_hidden")
_SLIM_KEYS = ("obs", "prev_obs", "reward", "stats", "src")


def unpack_learner(records, with_depth=None, keys=None):
    """Learner side of the config-5 round trip: uint8 [N, 272 | 336] learner
    records (SimManager.pack_learner, gathered from every rank) -> the columns
    learn/training_loop.py reads after step(): "obs" / "prev_obs" float32
    [N, 69] (construct_obs of the current / previous columns, bit-identical),
    "reward" [N, 1], "stats" int32 [N, 4], "action" int32 [N, 6], "hidden" /
    "prev_hidden" float32 [N, 16] (mbots_unpack_learner), on the records'
    device; `keys` selects the outputs.  Slim records (uint8 [N, 128 | 192],
    SimManager.pack_learner(slim=True)) give "obs", "prev_obs", "reward",
    "stats" and "src" int32 [N] -- each row's index in the table before the
    step, -1 for a newborn (mbots_unpack_learner_slim; harness/gather.py
    rebuilds action / hidden / prev_hidden from it)."""
    widths = (LEARNER_BYTES, LEARNER_BYTES_DEPTH, LEARNER_SLIM_BYTES, LEARNER_SLIM_BYTES_DEPTH)
    if records.dtype != torch.uint8 or records.dim() != 2 or records.shape[1] not in widths:
        raise ValueError(f"records must be uint8 [N, w], w in {widths}")
    slim = records.shape[1] in (LEARNER_SLIM_BYTES, LEARNER_SLIM_BYTES_DEPTH)
    wide = LEARNER_SLIM_BYTES_DEPTH if slim else LEARNER_BYTES_DEPTH
    depth = records.shape[1] == wide if with_depth is None else bool(with_depth)
    if depth != (records.shape[1] == wide):
        raise ValueError("with_depth does not match the record width")
    keys = (_SLIM_KEYS if slim else _LEARNER_KEYS) if keys is None else tuple(keys)
    allowed = _SLIM_KEYS if slim else _LEARNER_KEYS
    if any(k not in allowed for k in keys):
        raise ValueError(f"keys must be among {allowed}")
    rec = records.contiguous()
    n, dev = rec.shape[0], rec.device
    shapes = {"obs": ((n, OBS_DIM), torch.float32), "prev_obs": ((n, OBS_DIM), torch.float32),
              "reward": ((n, 1), torch.float32), "stats": ((n, 4), torch.int32),
              "action": ((n, 6), torch.int32), "hidden": ((n, 16), torch.float32),
              "prev_hidden": ((n, 16), torch.float32), "src": ((n,), torch.int32)}
    out = {k: torch.empty(shapes[k][0], dtype=shapes[k][1], device=dev) for k in keys}
    lo = _LearnerOut(**{k: (out[k].data_ptr() if k in out else None) for k in _LEARNER_KEYS})
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else None)
    devi = dev.index if dev.type == "cuda" else -1
    if slim:
        src = ctypes.c_void_p(out["src"].data_ptr() if "src" in out else None)
        _check(_lib.mbots_unpack_learner_slim(ctypes.c_void_p(rec.data_ptr()), n, 1 if depth else 0, devi,
                                              ctypes.byref(lo), src, stream))
    else:
        _check(_lib.mbots_unpack_learner(ctypes.c_void_p(rec.data_ptr()), n, 1 if depth else 0, devi,
                                         ctypes.byref(lo), stream))
    return out


def rebuild_learner(src, cur_counts, last_counts, last_action, last_memory, last_hidden):
    """The learner rank's rebuild from slim records (mbots_rebuild_learner):
    src int32 [N] (unpack_learner of slim records, in the reassembled global
    order), cur_counts / last_counts int64 [ranks, 4] species rows per rank of
    the gathered and of the last table, last_action int32 [M, 6] /
    last_memory f32 [M, 16] (the learner's writes after the last step) and
    last_hidden f32 [M, 16] (that step's HiddenState), all on one device (or
    the host) -> {"action" [N, 6], "hidden" [N, 16], "prev_hidden" [N, 16]}:
    the manager's Action, HiddenState and PrevHiddenState, bit-identical."""
    dev = src.device
    n = src.shape[0]
    cc = torch.as_tensor(cur_counts, dtype=torch.int64).cpu().contiguous()
    lc = torch.as_tensor(last_counts, dtype=torch.int64).cpu().contiguous()
    if cc.dim() != 2 or cc.shape[1] != 4 or lc.shape != cc.shape:
        raise ValueError("cur_counts / last_counts must be int64 [ranks, 4] of the same ranks")
    la = last_action.to(device=dev, dtype=torch.int32).contiguous()
    lm = last_memory.to(device=dev, dtype=torch.float32).contiguous()
    lh = last_hidden.to(device=dev, dtype=torch.float32).contiguous()
    s = src.to(torch.int32).contiguous()
    out = {"action": torch.empty((n, 6), dtype=torch.int32, device=dev),
           "hidden": torch.empty((n, 16), dtype=torch.float32, device=dev),
           "prev_hidden": torch.empty((n, 16), dtype=torch.float32, device=dev)}
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else None)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731
    _check(_lib.mbots_rebuild_learner(ptr(s), n, ptr(cc), ptr(lc), cc.shape[0], ptr(la), ptr(lm), ptr(lh),
                                      la.shape[0], ptr(out["action"]), ptr(out["hidden"]), ptr(out["prev_hidden"]),
                                      dev.index if dev.type == "cuda" else -1, stream))
    return out


madrona = types.ModuleType("madrona_bots.madrona")
madrona.ExecMode = ExecMode
madrona.Tensor = Tensor


class SimManager:
    """Manager (src/entry/mgr.hpp:10-68) with the nanobind constructor
    signature (entry.cpp:17-28).  Keyword-only extensions: exec_mode ("hip" /
    "cpu" or ExecMode.*: the Manager's ExecMode), agent_capacity
    (per-world slot cap), world_offset (global index of this shard's first
    world), reward_fixed (rewards[speciesID-1] instead of the reference's
    off-by-one), fix_depth_alias (depth_tensor returns real depth,
    SURVEY B.1), shard_ghost (also step world world_offset + num_worlds, never
    exported, so a shard's faithful B.3 rewards equal one device's; its agents
    act on the write_synthetic_actions stream), strict_capacity (a world that
    reaches agent_capacity -- at most MAX_CAPACITY = 4096 slots -- and drops a
    birth or respawn makes step() raise CapacityError instead of warning with
    CapacityWarning: the reference has no cap).

    agent_capacity="auto" grows the worlds' capacity instead of dropping
    agents: before each step() the manager reads the largest world population
    n (mbots_max_population: a wait for the last step's row counts, not for
    its sensor) and, when the step could overflow -- a step adds at
    most n births (one per agent, sim.cpp:561-564) and A respawns
    (:830-834) -- moves its state into the next capacity class (128, 256, 512,
    1024) through a checkpoint, so the run stays the reference's (bitwise equal
    to a manager that never drops) up to 1024 agents per world.  Views fetched
    before a growth keep the old storage alive but no longer follow the
    manager: take them after step(), as learn/training_loop.py:43-50 does."""

    def __init__(self, gpu_id, num_worlds, rand_seed, init_num_agents_per_world, *,
                 exec_mode="hip", agent_capacity=128, world_offset=0, reward_fixed=False,
                 fix_depth_alias=False, shard_ghost=False, strict_capacity=False):
        self.exec_mode = _exec_mode(exec_mode)
        self.gpu_id = int(gpu_id)
        self.num_worlds = int(num_worlds)
        self._auto_cap = isinstance(agent_capacity, str)
        if self._auto_cap:
            if agent_capacity != "auto":
                raise ValueError('agent_capacity must be an int or "auto"')
            if shard_ghost:
                raise ValueError('agent_capacity="auto" does not combine with shard_ghost')
            agent_capacity = _capacity_class(3 * int(init_num_agents_per_world))
        self.agent_capacity = int(agent_capacity)
        flags = (FLAG_REWARD_FIXED if reward_fixed else 0) | \
                (FLAG_FIX_DEPTH_ALIAS if fix_depth_alias else 0) | \
                (FLAG_SHARD_GHOST if shard_ghost else 0) | \
                (FLAG_STRICT_CAPACITY if strict_capacity else 0)
        self._cfg = (self.gpu_id, self.num_worlds, int(rand_seed) & 0xFFFFFFFF,
                     int(init_num_agents_per_world), 32, int(world_offset), flags, self.exec_mode)
        self._ghost = bool(shard_ghost)
        self._fix_depth = bool(fix_depth_alias)
        self._ktiming = False
        self._open(self.agent_capacity)

    def _open(self, cap):
        """Create the native manager at capacity `cap` (and reset the caches
        that belong to one)."""
        g, W, seed, A, sensor, off, flags, mode = self._cfg
        cfg = _Config(g, W, seed, A, sensor, off, int(cap), flags, mode)
        h = ctypes.c_void_p()
        _check(_lib.mbots_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._hd = _Handle(h)        # destroyed when the manager and all its views are gone
        self._h = h
        self.agent_capacity = int(cap)
        # row slots of every table column (the shard ghost is one more world)
        self._cap_rows = (self.num_worlds + (1 if self._ghost else 0)) * self.agent_capacity
        self._views = {}

    def _grow_if_needed(self):
        """agent_capacity="auto": the next capacity class before a step that
        could overflow this one (at most 2 n + A agents after it)."""
        if self.agent_capacity >= MAX_CAPACITY:
            return
        # (waits for the last step's row counts only, not for its sensor or the
        # caller's chain: the device stays fed while the host runs one step ahead)
        v = ctypes.c_uint32()
        _check(_lib.mbots_max_population(self._h, ctypes.byref(v)))
        need = 2 * int(v.value) + self._cfg[3]
        if need <= self.agent_capacity:
            return
        blob = self.save_checkpoint()
        old = (self._hd, self._h, self.agent_capacity, self._cap_rows, self._views)
        self._open(_capacity_class(need))   # (raises with the manager unchanged)
        try:
            _check(_lib.mbots_load_checkpoint(self._h, ctypes.c_void_p(blob.ctypes.data), blob.size))
        except BaseException:
            # keep running in the old class rather than on a fresh world
            self._hd, self._h, self.agent_capacity, self._cap_rows, self._views = old
            raise
        if self._ktiming:
            self.enable_kernel_timing(True)
        del old                      # (freed now unless a view still holds it)

    def _stream(self):
        if self.exec_mode == ExecMode.CPU:
            return ctypes.c_void_p(None)
        return ctypes.c_void_p(_raw_stream(self.gpu_id))

    def _view_cache(self, tensor):
        """Torch view of the whole allocation behind `tensor` (every row slot
        the manager reserved for that column), created once; None for exports
        that are not table columns."""
        rows, cols = tensor.shape
        cap_rows = self._cap_rows
        if rows > cap_rows:
            return None
        key = (tensor._ptr, tensor._torch_dtype, cols)
        base = self._views.get(key)
        if base is None:
            # (owned by the handle, not the manager: no cycle through the cache)
            full = Tensor(self._hd, _CTensor(tensor._ptr, _DTYPE_CODE[tensor._torch_dtype], tensor._device,
                                             (ctypes.c_int64 * 2)(cap_rows, cols)))
            base = torch.as_tensor(full, device=torch.device("cuda", tensor._device))
            if base.data_ptr() != tensor._ptr:
                raise RuntimeError("madrona_bots: to_torch() produced a copy, expected a view")
            self._views[key] = base
        return base

    @property
    def device(self):
        """torch device of the exported views."""
        if self.exec_mode == ExecMode.CPU:
            return torch.device("cpu")
        return torch.device("cuda", self.gpu_id)

    # -- graphs -------------------------------------------------------------
    def step(self):
        if self._auto_cap:
            self._grow_if_needed()
        rc = _lib.mbots_step(self._h, self._stream())
        if rc == _W_CAPACITY:   # the step ran; agents were dropped at the cap (reported late by a few steps)
            warnings.warn(f"madrona_bots: {_lib.mbots_last_error().decode(errors='replace')}",
                          CapacityWarning, stacklevel=2)
        elif rc:
            _check(rc)

    def shift_observations(self):
        _check(_lib.mbots_shift_observations(self._h, self._stream()))

    # -- exports ------------------------------------------------------------
    def _export(self, eid):
        # stream-ordered on torch's current stream: the view's deferred copies
        # and joins are enqueued there, after everything the manager enqueued
        # on whatever stream its previous call used (mbots_export_on)
        ct = _CTensor()
        _check(_lib.mbots_export_on(self._h, eid, self._stream(), ctypes.byref(ct)))
        return Tensor(self._hd, ct, column=eid not in (ExportID.SpeciesCount, ExportID.Reset), mgr=self)

    def depth_tensor(self, is_prev=False):
        return self._export(ExportID.PrevSensorDepth if is_prev else ExportID.SensorDepth)

    def semantic_tensor(self, is_prev=False):
        return self._export(ExportID.PrevSensorSemantic if is_prev else ExportID.SensorSemantic)

    def reward_tensor(self, is_prev=False):
        return self._export(ExportID.PrevReward if is_prev else ExportID.Reward)

    def species_count_tensor(self):
        return self._export(ExportID.SpeciesCount)

    def position_tensor(self, is_prev=False):
        return self._export(ExportID.PrevPosition if is_prev else ExportID.Position)

    def health_tensor(self, is_prev=False):
        return self._export(ExportID.PrevHealth if is_prev else ExportID.Health)

    def surrounding_tensor(self, is_prev=False):
        return self._export(ExportID.PrevSurrounding if is_prev else ExportID.Surrounding)

    def action_tensor(self, is_prev=False):
        return self._export(ExportID.PrevAction if is_prev else ExportID.Action)

    def stats_tensor(self, is_prev=False):
        return self._export(ExportID.PrevStats if is_prev else ExportID.Stats)

    def hidden_state_tensor(self, is_prev=False):
        return self._export(ExportID.PrevHiddenState if is_prev else ExportID.HiddenState)

    # C++-only accessors of the reference (mgr.hpp:38, :54-62) + extensions
    def sensor_index_tensor(self):
        return self._export(ExportID.SensorIndex)

    def done_tensor(self):
        return self._export(ExportID.Done)

    def species_tensor(self, is_prev=False):
        return self._export(ExportID.PrevSpecies if is_prev else ExportID.Species)

    def set_action(self, agent_idx, forward, backward, rotate_left, rotate_right, shoot, breed):
        a = (ctypes.c_int32 * 6)(forward, backward, rotate_left, rotate_right, shoot, breed)
        _check(_lib.mbots_set_action(self._h, int(agent_idx), a))

    def agent_offset_for_world(self, world_idx):
        v = ctypes.c_uint32()
        _check(_lib.mbots_agent_offset_for_world(self._h, int(world_idx), ctypes.byref(v)))
        return v.value

    # -- build utilities ------------------------------------------------------
    def num_agents(self):
        v = ctypes.c_uint32()
        _check(_lib.mbots_num_agents(self._h, ctypes.byref(v)))
        return v.value

    def construct_obs(self, is_prev=False, out=None):
        """learn/util.py construct_obs over all N rows (every species, species-
        major) in one fused kernel: float32 [N, 69] = depth | health | position |
        semantic | surrounding, bit-identical to the torch.cat of the views.
        Slice [start:end] per species with species_count_tensor()."""
        import torch
        n = self.num_agents()
        if out is None:
            out = torch.empty((n, OBS_DIM), dtype=torch.float32, device=self.device)
        if out.dtype != torch.float32 or out.device != self.device or not out.is_contiguous() \
                or out.dim() != 2 or out.shape[1] != OBS_DIM or out.shape[0] < n:
            raise ValueError(f"out must be a contiguous float32 [>= {n}, {OBS_DIM}] tensor on "
                             f"{self.device}")
        _check(_lib.mbots_construct_obs(self._h, 1 if is_prev else 0,
                                        ctypes.c_void_p(out.data_ptr()), out.shape[0],
                                        self._stream()))
        return out[:n]

    def rollout_record_bytes(self):
        """Bytes per rollout record (include/mbots.h: 64, or 96 with real depth)."""
        v = ctypes.c_uint32()
        _check(_lib.mbots_rollout_record_bytes(self._h, ctypes.byref(v)))
        return v.value

    def pack_rollout(self, out=None):
        """The raw columns the learner reads after step() (semantic, health,
        position, surrounding, reward, stats; depth when fixed) as one uint8
        [N, rollout_record_bytes()] record per export row -- the payload of the
        config-5 gather to the learner rank; unpack_rollout()
        rebuilds construct_obs rows from it.  `out` may hold more rows (padding)."""
        import torch
        n = self.num_agents()
        rb = self.rollout_record_bytes()
        if out is None:
            out = torch.empty((n, rb), dtype=torch.uint8, device=self.device)
        if out.dtype != torch.uint8 or out.device != self.device or not out.is_contiguous() \
                or out.dim() != 2 or out.shape[1] != rb or out.shape[0] < n:
            raise ValueError(f"out must be a contiguous uint8 [>= {n}, {rb}] tensor on {self.device}")
        _check(_lib.mbots_pack_rollout(self._h, ctypes.c_void_p(out.data_ptr()), out.shape[0],
                                       self._stream()))
        return out[:n]

    def num_rows(self):
        """Every table row: num_agents() plus the shard ghost's rows (which
        follow row N; see write_actions)."""
        v = ctypes.c_uint32()
        _check(_lib.mbots_num_rows(self._h, ctypes.byref(v)))
        return v.value

    def learner_record_bytes(self, slim=False):
        """Bytes per learner record (include/mbots.h: 272, or 336 with real
        depth; slim records 128 / 192)."""
        if slim:
            return LEARNER_SLIM_BYTES_DEPTH if self._fix_depth else LEARNER_SLIM_BYTES
        v = ctypes.c_uint32()
        _check(_lib.mbots_learner_record_bytes(self._h, ctypes.byref(v)))
        return v.value

    def pack_learner(self, out=None, slim=False):
        """Everything the reference training loop reads after step() --
        current and previous observation columns, reward, stats, Action,
        HiddenState, PrevHiddenState (learn/training_loop.py:43-93) -- as one
        uint8 [N, learner_record_bytes()] record per export row: the payload of
        the config-5 gather (harness/gather.py); unpack_learner() rebuilds the
        learner's tensors.  `out` may hold more rows (padding).  slim=True:
        the 128-B records without Action / HiddenState / PrevHiddenState but
        with each row's provenance (include/mbots.h MBOTS_LEARNER_SLIM_BYTES),
        for a learner that rebuilds those from its own writes."""
        n = self.num_agents()
        rb = self.learner_record_bytes(slim)
        if out is None:
            out = torch.empty((n, rb), dtype=torch.uint8, device=self.device)
        if out.dtype != torch.uint8 or out.device != self.device or not out.is_contiguous() \
                or out.dim() != 2 or out.shape[1] != rb or out.shape[0] < n:
            raise ValueError(f"out must be a contiguous uint8 [>= {n}, {rb}] tensor on {self.device}")
        fn = _lib.mbots_pack_learner_slim if slim else _lib.mbots_pack_learner
        _check(fn(self._h, ctypes.c_void_p(out.data_ptr()), out.shape[0], self._stream()))
        return out[:n]

    def write_actions(self, actions=None, memory=None):
        """The learner's writes for every row at once (training_loop.py:136-137:
        action_tensor[...] = one_hot; memory_tensor[...] = new_memory):
        int32 [R, 6] actions and/or float32 [R, 16] memory, R = num_agents() or
        num_rows() (the latter also drives the shard ghost's agents, which then
        act exactly as the next rank's first world does) -- mbots_write_actions."""
        def arg(t, cols, dtype):
            if t is None:
                return None, None
            if t.dtype != dtype or t.dim() != 2 or t.shape[1] != cols or t.device != self.device:
                raise ValueError(f"expected {dtype} [rows, {cols}] on {self.device}")
            t = t.contiguous()
            return t, t.shape[0]
        a, ra = arg(actions, 6, torch.int32)
        m, rm = arg(memory, 16, torch.float32)
        rows = ra if ra is not None else rm
        if rows is None:
            return
        if ra is not None and rm is not None and ra != rm:
            raise ValueError("actions and memory must have the same rows")
        _check(_lib.mbots_write_actions(self._h, ctypes.c_void_p(a.data_ptr() if a is not None else None),
                                        ctypes.c_void_p(m.data_ptr() if m is not None else None), rows,
                                        self._stream()))

    def save_checkpoint(self, path=None):
        """Live simulator state as bytes (and to `path` if given); see
        load_checkpoint.  Not in the reference."""
        import numpy as np
        n = ctypes.c_uint64()
        _check(_lib.mbots_checkpoint_size(self._h, ctypes.byref(n)))
        buf = np.empty(n.value, dtype=np.uint8)
        _check(_lib.mbots_save_checkpoint(self._h, ctypes.c_void_p(buf.ctypes.data), n.value))
        if path is not None:
            buf.tofile(path)
        return buf

    def load_checkpoint(self, src):
        """Restore a checkpoint (bytes/array or a file path) saved by a manager
        of the same configuration; the next step continues bit-exactly."""
        import numpy as np
        buf = np.fromfile(src, dtype=np.uint8) if isinstance(src, (str, os.PathLike)) \
            else np.ascontiguousarray(np.frombuffer(src, dtype=np.uint8))
        _check(_lib.mbots_load_checkpoint(self._h, ctypes.c_void_p(buf.ctypes.data), buf.size))

    def world_state(self, world_idx):
        """Debug dump of one world (replacing the viewer's
        state readback): live agents' position, rotation (w, z), species,
        health, finder slot, and the live food packages (chunk, x, y, rotation as
        a 22-bit quarter-turn fraction),
        as numpy arrays (save with numpy.savez)."""
        import numpy as np
        cap = self.agent_capacity
        xyr = np.zeros((cap, 4), np.float32)
        shf = np.zeros((cap, 3), np.int32)
        food = np.zeros(48, np.uint64)
        rot = np.zeros((5, 48), np.uint32)
        n = ctypes.c_int32()
        _check(_lib.mbots_world_state(self._h, int(world_idx), ctypes.c_void_p(xyr.ctypes.data),
                                      ctypes.c_void_p(shf.ctypes.data),
                                      ctypes.c_void_p(food.ctypes.data),
                                      ctypes.c_void_p(rot.ctypes.data), ctypes.byref(n)))
        k = n.value
        pk = []
        for c, rec in enumerate(food.tolist()):
            for q in range(5):
                if (rec >> (40 + q)) & 1:
                    xy = (rec >> (8 * q)) & 0xFF
                    pk.append((c, (c % 8) * 16 + (xy & 15), (c // 8) * 16 + (xy >> 4),
                               int(rot[q, c])))
        return {"position": xyr[:k, :2].copy(), "rotation_wz": xyr[:k, 2:].copy(),
                "species": shf[:k, 0].copy(), "health": shf[:k, 1].copy(),
                "finder": shf[:k, 2].copy(),
                "food": np.array(pk, np.int32).reshape(-1, 4)}

    def dump_worlds(self, path, worlds):
        """Write world_state() of each world in `worlds` to one .npz
        (keys "w<idx>/<field>") for offline inspection -- the build's
        replacement for the reference viewer's readback (src/gfx)."""
        import numpy as np
        arrays = {}
        for w in worlds:
            for k, v in self.world_state(w).items():
                arrays[f"w{int(w)}/{k}"] = v
        np.savez(path, **arrays)
        return sorted(arrays)

    def join(self):
        """Make torch's current stream wait for the manager's outstanding
        sensor work (mbots_join): ends a sequence of steps captured into a
        HIP graph (torch.cuda.graph) with no unjoined work."""
        _check(_lib.mbots_join(self._h, self._stream()))

    def record_sensor_done(self, event):
        """Record a timing-enabled torch.cuda.Event on the manager's internal
        stream after the last step's sensor (mbots_record_sensor_done): a
        benchmark timing point that adds no wait to any stream."""
        if not event.cuda_event:   # torch creates its events on first record
            event.record()
        _check(_lib.mbots_record_sensor_done(self._h, ctypes.c_void_p(event.cuda_event)))

    def write_synthetic_actions(self, seed, step, write_hidden=False):
        _check(_lib.mbots_write_synthetic_actions(self._h, int(seed) & 0xFFFFFFFF,
                                                  int(step) & 0xFFFFFFFF,
                                                  1 if write_hidden else 0, self._stream()))

    def agent_steps(self):
        v = ctypes.c_uint64()
        _check(_lib.mbots_agent_steps(self._h, ctypes.byref(v)))
        return v.value

    def overflow(self):
        v = ctypes.c_uint64()
        _check(_lib.mbots_overflow(self._h, ctypes.byref(v)))
        return v.value

    def enable_kernel_timing(self, enable=True):
        self._ktiming = bool(enable)
        _check(_lib.mbots_enable_kernel_timing(self._h, 1 if enable else 0))

    def schedule_info(self):
        """The step schedule in use (mbots_schedule_info): {"k1_finder",
        "fork_by_value", "join_by_value", "swap", "mixed_classes": bool,
        "epoch", "epoch_wraps", "steps": int}."""
        v = (ctypes.c_uint32 * 4)()
        _check(_lib.mbots_schedule_info(self._h, v))
        f = v[0]
        return {"k1_finder": bool(f & 1), "fork_by_value": bool(f & 2), "join_by_value": bool(f & 4),
                "swap": bool(f & 8), "mixed_classes": bool(f & 16), "epoch": int(v[1]),
                "epoch_wraps": int(v[2]), "steps": int(v[3])}

    def kernel_times(self):
        """{kernel: (total_ms, launches)} since enable_kernel_timing()."""
        ms = (ctypes.c_double * len(KERNELS))()
        n = (ctypes.c_uint64 * len(KERNELS))()
        _check(_lib.mbots_kernel_times(self._h, ms, n))
        return {k: (ms[i], n[i]) for i, k in enumerate(KERNELS)}


class ScriptBotsViewer:
    """The reference module's second class (src/entry/entry.cpp:47-80): a
    windowed viewer around a Manager (src/gfx, Vulkan) whose ``loop(num_epochs,
    step_fn, carry)`` calls ``step_fn(epoch, carry)`` once per rendered frame
    and whose ``get_sim_mgr()`` returns the manager.  The viewer is out of this
    build's scope, so the name exists
    for the reference's imports -- ``from madrona_bots import SimManager,
    ScriptBotsViewer`` (learn/training_loop.py:8, learn/env_app.py:2,
    learn/app.py:1) -- and constructing it raises.  Headless training takes the
    training loop's other branch (``TrainLoopManager`` over ``SimManager``,
    training_loop.py:15-26, :172-173); ``SimManager.world_state`` /
    ``dump_worlds`` replace the viewer's readback for offline inspection."""

    def __init__(self, gpu_id, num_worlds, rand_seed, init_num_agents_per_world, window_width,
                 window_height):
        raise NotImplementedError(
            "madrona_bots: ScriptBotsViewer (the reference's Vulkan viewer, src/gfx) is not part of this "
            "build; run headless with SimManager (learn/training_loop.py without --enable_viewer) and "
            "inspect worlds with SimManager.world_state() / dump_worlds()")
