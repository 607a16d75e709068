"""GPU parity: HIP product vs the CPU oracle, bitwise on every exported column.

The oracle (oracle/mbots_oracle.c) restates src/sim/sim.cpp; both sides run the
same seeds and the identity-keyed synthetic action stream, so
integer columns must be bit-exact and float columns bit-exact too (the float
tolerance the north star allows, 1e-5, is not needed: both sides round
identically with -ffp-contract=off)."""
import numpy as np
import pytest
import torch

import pyoracle
from simpair import compare

pytestmark = pytest.mark.gpu


def _pair(W, seed=69, A=32, steps=12, cap=128, reward_fixed=False, depth_fixed=False,
          write_hidden=True, world_offset=0):
    import madrona_bots as mb
    mgr = mb.SimManager(0, W, seed, A, agent_capacity=cap, reward_fixed=reward_fixed,
                        fix_depth_alias=depth_fixed, world_offset=world_offset)
    orc = pyoracle.OracleSim(W, seed, A, cap=cap, reward_fixed=reward_fixed,
                             world_offset=world_offset, num_threads=8)
    errs = compare(mgr, orc, "init", depth_fixed=depth_fixed)
    assert not errs, errs[:5]
    for t in range(steps):
        mgr.write_synthetic_actions(1234, t, write_hidden)
        orc.write_synthetic_actions(1234, t, write_hidden)
        mgr.step()
        orc.step()
        errs = compare(mgr, orc, f"step {t}", depth_fixed=depth_fixed)
        assert not errs, errs[:5]
        mgr.shift_observations()
        orc.shift_observations()
        errs = compare(mgr, orc, f"shift {t}", depth_fixed=depth_fixed)
        assert not errs, errs[:5]
    return mgr, orc


def test_parity_small():
    _pair(4, steps=24)


def test_parity_64_worlds():
    _pair(64, steps=40)


def test_parity_reward_fixed_and_depth():
    _pair(32, steps=16, reward_fixed=True, depth_fixed=True)


def test_parity_seed_and_offset():
    _pair(48, seed=7, steps=16, world_offset=1000)


@pytest.mark.parametrize("cap,depth_fixed", [(128, True), (256, False)])
def test_parity_population_order(cap, depth_fixed):
    """A whole number of 1024-world scan tiles: the sensor renders the worlds
    in K2's per-tile descending-population order (S.sorder) -- in both capacity
    classes and with the depth bytes -- and every column still equals the
    oracle's."""
    _pair(2048, steps=4, cap=cap, depth_fixed=depth_fixed)


@pytest.mark.parametrize("cap,A,depth_fixed,shift", [(256, 96, True, False), (256, 96, False, True),
                                                     (128, 32, True, True)])
def test_k1_finder_step_only_prev_sensor(cap, A, depth_fixed, shift):
    """in K1-finder mode (<= 2048 worlds) the next K1 waits
    only for the sensor before the last one, while the sensor reads K1's
    old-row column (obsrow_out) to move the previous sensor rows into its own
    rows -- so that column is double-buffered by step parity.  Steps back to
    back with no read in between (the bench's loop: actions, step, optionally
    the shift) at 2048 worlds, where the sensor's waves take more than one
    residency round (256 slots and the depth bytes lower its occupancy) and,
    with 96 agents per world, takes several times the next K1's time, so that
    K1 runs while the sensor's last blocks are still to start; after each
    burst every column, the prev sensor's semantic and depth included, equals
    the oracle's."""
    import madrona_bots as mb
    W = 2048
    mgr = mb.SimManager(0, W, 69, A, agent_capacity=cap, fix_depth_alias=depth_fixed)
    orc = pyoracle.OracleSim(W, 69, A, cap=cap, num_threads=16)
    t = 0
    for burst in range(2):
        for _ in range(5):
            mgr.write_synthetic_actions(1234, t, True)
            orc.write_synthetic_actions(1234, t, True)
            mgr.step()
            orc.step()
            if shift:
                mgr.shift_observations()
                orc.shift_observations()
            t += 1
        errs = compare(mgr, orc, f"burst {burst}", depth_fixed=depth_fixed)
        assert not errs, errs[:5]


def test_parity_small_population():
    # A=4 -> one agent per species; respawn path exercised constantly
    _pair(64, A=4, steps=30, cap=16)


def test_parity_4096_worlds():
    _pair(4096, steps=6)


@pytest.mark.parametrize("shifts", [0, 1, 2])
def test_parity_lazy_shift_unobserved(shifts):
    """shift_observations() leaves six Prev* columns as views of the current
    ones; the next step moves them from there.  A step defers moving
    PrevAction / PrevHiddenState (a shift overwrites them); with no shift the
    next step moves them first.  Compare only every 5th step, so most steps run
    on those paths without an accessor materialising the copies."""
    import madrona_bots as mb
    W = 64
    mgr = mb.SimManager(0, W, 69, 32)
    orc = pyoracle.OracleSim(W, 69, 32, num_threads=8)
    for t in range(15):
        mgr.write_synthetic_actions(1234, t, True)
        orc.write_synthetic_actions(1234, t, True)
        mgr.step()
        orc.step()
        if t % 5 == 4:
            errs = compare(mgr, orc, f"step {t}")
            assert not errs, errs[:5]
        for _ in range(shifts):
            mgr.shift_observations()
            orc.shift_observations()
    errs = compare(mgr, orc, "end")
    assert not errs, errs[:5]


# ---------------------------------------------------------------------------
# golden fixtures (tests/golden, generated by the oracle) through the HIP path
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["oracle_w4_a32_s69", "oracle_w8_a4_s7_fixed"])
def test_hip_matches_golden_fixture(name):
    import madrona_bots as mb
    from golden_util import load_fixture, table_digests
    meta, arrays = load_fixture(name)
    mgr = mb.SimManager(0, meta["worlds"], meta["seed"], meta["agents"],
                        agent_capacity=meta["cap"], reward_fixed=meta["reward_fixed"])
    acc = {"species": "species_tensor", "pos": "position_tensor", "health": "health_tensor",
           "surround": "surrounding_tensor", "reward": "reward_tensor",
           "action": "action_tensor", "stats": "stats_tensor",
           "hidden": "hidden_state_tensor", "semantic": "semantic_tensor"}

    def get(nm, prev):
        if nm == "depth":   # not exported without fix_depth_alias: reuse the oracle's
            return np.zeros(0)
        a = getattr(mgr, acc[nm])(prev).to_torch().cpu().numpy()
        if nm == "health":
            a = a.view(np.int32)
        return a

    def digests():
        d = table_digests(get, mgr.species_count_tensor().to_torch().cpu().numpy())
        return d

    log = [["init", mgr.num_agents(), digests()]]
    for t in range(meta["steps"]):
        mgr.write_synthetic_actions(meta["action_seed"], t, meta["write_hidden"])
        mgr.step()
        log.append([f"step{t}", mgr.num_agents(), digests()])
        mgr.shift_observations()
        log.append([f"shift{t}", mgr.num_agents(), digests()])
    for (tag, n, dg), (tag2, n2, dg2) in zip(meta["log"], log):
        assert tag == tag2 and n == n2, (tag, n, n2)
        bad = [k for k in dg if "depth" not in k and dg[k] != dg2[k]]
        assert not bad, f"{name} {tag}: columns differ from golden: {bad}"
    for nm in ("species", "pos", "reward", "semantic"):
        assert np.array_equal(get(nm, False), arrays[nm])


# ---------------------------------------------------------------------------
# BASELINE sizes: size-independent properties
# ---------------------------------------------------------------------------
def _checksum(mgr):
    h = 0
    for nm in ("position_tensor", "health_tensor", "reward_tensor", "semantic_tensor",
               "action_tensor", "hidden_state_tensor", "stats_tensor"):
        for prev in (False, True):
            t = getattr(mgr, nm)(prev).to_torch()
            h = (h * 1000003 + int(t.view(torch.uint8).to(torch.int64).sum())) % (1 << 61)
    return h


@pytest.mark.parametrize("W", [65536])
def test_large_invariants_and_determinism(W):
    import madrona_bots as mb
    sums = []
    for rep in range(2):
        m = mb.SimManager(0, W, 69, 32)
        for t in range(20):
            m.write_synthetic_actions(1234, t, True)
            m.step()
            N = m.num_agents()
            sc = m.species_count_tensor().to_torch()
            assert int(sc.sum()) == N and tuple(sc.shape) == (W, 4)
            sp = m.species_tensor(False).to_torch()
            assert bool((sp[1:] >= sp[:-1]).all())                  # species-major rows
            assert torch.equal(torch.bincount(sp.ravel().long(), minlength=5)[1:].cpu(),
                               sc.sum(0).cpu().long())
            sem = m.semantic_tensor(False).to_torch()
            assert int(sem.min()) >= -1 and int(sem.max()) <= 6 and not bool((sem == 0).any())   # -1: a miss
            assert bool((m.health_tensor(False).to_torch().view(torch.int32) > 0).all())
            m.shift_observations()
            for nm in ("position_tensor", "health_tensor", "surrounding_tensor",
                       "reward_tensor", "action_tensor", "hidden_state_tensor"):
                assert torch.equal(getattr(m, nm)(True).to_torch(), getattr(m, nm)(False).to_torch())
            st, pst = m.stats_tensor(False).to_torch(), m.stats_tensor(True).to_torch()
            assert torch.equal(pst[:, 1], st[:, 0])                 # sim.cpp:1034
        assert m.overflow() == 0
        sums.append(_checksum(m))
        del m
    assert sums[0] == sums[1]                                       # bitwise deterministic


@pytest.mark.parametrize("reward_fixed", [True, False])
def test_two_shards_equal_one_on_device(reward_fixed):
    # faithful B.3 rewards across the shard boundary: shard 0 steps a ghost of
    # shard 1's first world (shard_ghost), the last shard none
    import madrona_bots as mb
    W = 2048

    def run(m):
        for t in range(10):
            m.write_synthetic_actions(1234, t, True)
            m.step()
            m.shift_observations()
    full = mb.SimManager(0, W, 69, 32, reward_fixed=reward_fixed)
    run(full)
    shards = [mb.SimManager(0, W // 2, 69, 32, reward_fixed=reward_fixed, world_offset=r * (W // 2),
                            shard_ghost=(not reward_fixed) and r == 0)
              for r in range(2)]
    for s in shards:
        run(s)
    fsc = full.species_count_tensor().to_torch().cpu().numpy()
    ssc = [s.species_count_tensor().to_torch().cpu().numpy() for s in shards]
    assert np.array_equal(fsc, np.concatenate(ssc))
    assert full.num_agents() == sum(s.num_agents() for s in shards)
    for nm in ("position_tensor", "health_tensor", "reward_tensor", "semantic_tensor",
               "hidden_state_tensor", "action_tensor", "stats_tensor"):
        for prev in (False, True):
            f = getattr(full, nm)(prev).to_torch().cpu().numpy()
            parts = [getattr(s, nm)(prev).to_torch().cpu().numpy() for s in shards]
            # species-major per shard: species s of the full table = shard0's ++ shard1's
            fo, so = 0, [0, 0]
            for sp in range(4):
                cnt = [int(x[:, sp].sum()) for x in ssc]
                want = np.concatenate([parts[k][so[k]:so[k] + cnt[k]] for k in range(2)])
                assert np.array_equal(f[fo:fo + sum(cnt)], want), (nm, prev, sp)
                fo += sum(cnt)
                so = [so[k] + cnt[k] for k in range(2)]


@pytest.mark.parametrize("W", [1, 5, 1023, 1025])
def test_parity_edge_world_counts(W):
    # single world, a ragged 4-world block, one world short of / past a
    # 1024-world scan tile
    _pair(W, steps=6)


def test_parity_capacity_overflow():
    # agent_capacity == initial population: every birth and respawn beyond the
    # slot capacity is dropped and counted identically on both sides
    mgr, orc = _pair(48, A=32, cap=32, steps=10)
    assert mgr.overflow() == orc.overflow()
    assert mgr.overflow() > 0


def test_parity_large_population_two_passes():
    # > 64 agents per world: every per-world loop takes its second 64-lane pass
    mgr, orc = _pair(16, A=100, cap=128, steps=6)
    assert mgr.num_agents() > 16 * 64


def test_action_written_between_step_and_shift():
    """Action / HiddenState stay in the other table half after a step until an
    accessor, a write or the shift needs them: a write through a view taken
    between step() and shift_observations() must be what the shift copies."""
    import madrona_bots as mb
    m = mb.SimManager(0, 32, 69, 32)
    for t in range(3):
        m.write_synthetic_actions(1234, t)
        m.step()
        a = m.action_tensor(False).to_torch()
        h = m.hidden_state_tensor(False).to_torch()
        pat = torch.arange(a.numel(), device=a.device, dtype=torch.int32).reshape(a.shape) % 7 + t
        hp = torch.full_like(h, float(t) + 0.25)
        a.copy_(pat)
        h.copy_(hp)
        m.shift_observations()
        assert torch.equal(m.action_tensor(True).to_torch(), pat)
        assert torch.equal(m.hidden_state_tensor(True).to_torch(), hp)
        assert torch.equal(m.action_tensor(False).to_torch(), pat)


def _obs_rows_oracle(orc, prev, fixd):
    """learn/util.py construct_obs rows from the oracle's columns (depth as
    uint8 -- the semantic buffer unless fixed, B.1 --, health's int32 bits as
    f32, B.2, position, semantic as int8, surrounding)."""
    sem = orc.column(pyoracle.COL_SEMANTIC, prev)
    dep = orc.column(pyoracle.COL_DEPTH, prev) if fixd else sem.view(np.uint8)
    hp = np.ascontiguousarray(orc.column(pyoracle.COL_HEALTH, prev)).view(np.float32)
    return np.concatenate([dep.astype(np.float32), hp, orc.column(pyoracle.COL_POS, prev),
                           sem.astype(np.float32), orc.column(pyoracle.COL_SURROUND, prev)], axis=1)


@pytest.mark.parametrize("seed", list(range(1, 13)))
def test_random_call_sequences(seed, W=None):
    """Random interleavings of step / shift / action writes / single-column
    reads / fused learner rows (construct_obs, current or previous) /
    checkpoint hand-overs against the oracle.  Each read materialises one
    lazily shifted or deferred column at a different point of the step cycle,
    and construct_obs(prev) gathers the still-deferred Prev columns itself; a
    checkpoint saved at any point of the cycle continues in a fresh manager of
    a random capacity class (128 / 256 / 512 / 1024: the cross-capacity load
    agent_capacity="auto" grows through).
    Small world counts run in K1-finder mode (no wait for the last sensor),
    4100 worlds on the joined schedule with its value waits.  A full
    comparison follows every few operations and at the end."""
    from simpair import COLUMNS, bits, gpu_column
    import madrona_bots as mb
    rng = np.random.default_rng(seed)
    caps = np.random.default_rng(seed + 1000)   # (its own stream: the op sequences stay the seeds')
    W = W or (4100 if seed % 4 == 0 else 20 + seed)
    fixd = bool(seed % 2)
    mgr = mb.SimManager(0, W, 69, 32, fix_depth_alias=fixd)
    orc = pyoracle.OracleSim(W, 69, 32, num_threads=8)
    t = 0
    for it in range(48):
        op = int(rng.integers(0, 8))
        if op == 7:
            if rng.integers(0, 2):   # (half the draws: a checkpoint is a rare call)
                blob = mgr.save_checkpoint()
                cap = int(caps.choice(mb.CAPACITY_CLASSES))
                mgr = mb.SimManager(0, W, 69, 32, fix_depth_alias=fixd, agent_capacity=cap)
                mgr.load_checkpoint(blob)
            continue
        if op in (0, 1):
            wh = bool(rng.integers(0, 2))
            mgr.write_synthetic_actions(1234, t, wh)
            orc.write_synthetic_actions(1234, t, wh)
            mgr.step()
            orc.step()
            t += 1
        elif op == 2:
            mgr.shift_observations()
            orc.shift_observations()
        elif op == 3:
            wh = bool(rng.integers(0, 2))
            mgr.write_synthetic_actions(4321, t, wh)
            orc.write_synthetic_actions(4321, t, wh)
        elif op == 4:
            name, cid = COLUMNS[int(rng.integers(len(COLUMNS)))]
            prev = bool(rng.integers(0, 2))
            g, o = gpu_column(mgr, name, prev), orc.column(cid, prev)
            assert g.shape == o.shape and np.array_equal(bits(g), bits(o)), (it, name, prev)
        elif op == 6:
            prev = bool(rng.integers(0, 2))
            g = mgr.construct_obs(prev).cpu().numpy()
            o = _obs_rows_oracle(orc, prev, fixd)
            assert g.shape == o.shape and np.array_equal(bits(g), bits(o)), (it, "construct_obs", prev)
        elif it % 4 == 0:
            errs = compare(mgr, orc, f"op {it}", depth_fixed=fixd)
            assert not errs, errs[:5]
    errs = compare(mgr, orc, "end", depth_fixed=fixd)
    assert not errs, errs[:5]


@pytest.mark.parametrize("seed", [101, 102])
def test_random_call_sequences_swapped_schedule(seed):
    """The random call sequences at 16400 worlds, on the swapped schedule
    (K1 / K2 / the sensor on the internal stream: the default above 8192
    worlds) with the lazy prev-sensor move."""
    test_random_call_sequences(seed, W=16400)


@pytest.mark.parametrize("ops", ["hss" + "wss" * 9, "hsswss" + "ss" * 4 + "wsw", "sss" + "hss" * 6,
                                 "hsS" + "wsS" * 5 + "ws"])
def test_aliased_current_action_hidden(ops):
    """After a fused shift the current Action / HiddenState columns are views
    of their Prev columns (DESIGN.md "Aliased current Action / HiddenState"):
    K1 reads the actions through that view when nothing wrote them, the next
    step's moves gather an unwritten HiddenState from the Prev column, and a
    second shift keeps them equal.  Ops: w = action write without hidden,
    h = with hidden, s = step or shift (alternating), S = shift again; the
    tables are compared only at the end, so no accessor copies the views out
    on the way."""
    import madrona_bots as mb
    W = 40
    mgr = mb.SimManager(0, W, 69, 32)
    orc = pyoracle.OracleSim(W, 69, 32, num_threads=8)
    t, stepped = 0, False
    for op in ops:
        if op in "wh":
            mgr.write_synthetic_actions(1234, t, op == "h")
            orc.write_synthetic_actions(1234, t, op == "h")
        elif op == "s" and not stepped:
            mgr.step(); orc.step(); t += 1
            stepped = True
        else:
            mgr.shift_observations(); orc.shift_observations()
            stepped = False
    errs = compare(mgr, orc, "end")
    assert not errs, errs[:5]


def test_reference_loop_pattern_prefetch():
    """learn/training_loop.py's order -- step, the action / memory views, reward,
    construct_obs(cur), construct_obs(prev), PrevHiddenState, shift, the
    learner's writes -- makes the manager prefetch the deferred moves at the
    next step (DESIGN.md "Prefetch"); every column still equals the oracle's,
    also when the pattern stops (no reads: back to the lazy path)."""
    import madrona_bots as mb
    W = 96
    mgr = mb.SimManager(0, W, 69, 32)
    orc = pyoracle.OracleSim(W, 69, 32, num_threads=8)
    for t in range(14):
        mgr.write_synthetic_actions(1234, t, True)
        orc.write_synthetic_actions(1234, t, True)
        mgr.step()
        orc.step()
        if t < 9 or t == 12:
            mgr.action_tensor(False).to_torch()
            mgr.hidden_state_tensor(False).to_torch()
            mgr.reward_tensor(False).to_torch().clone()
            mgr.construct_obs(False)
            mgr.construct_obs(True)
            mgr.hidden_state_tensor(True).to_torch()
        mgr.shift_observations()
        orc.shift_observations()
        errs = compare(mgr, orc, f"shift {t}")
        assert not errs, errs[:5]


def _breed_heavy(n, step):
    """breed 1/2, forward 1/4, rotate 1/4, no shooting: the population grows
    until the slot capacity binds (makeAgent has no cap)"""
    g = torch.Generator().manual_seed(1000 + step)
    r = torch.randint(0, 8, (n,), generator=g)
    a = torch.zeros((n, 6), dtype=torch.int32)
    a[r < 4, 5] = 1
    a[(r >= 4) & (r < 6), 0] = 1
    a[r == 6, 2] = 1
    a[r == 7, 3] = 1
    return a


@pytest.mark.parametrize("cap,W,steps", [(256, 48, 45), (128, 48, 45), (512, 16, 70), (1024, 8, 110),
                                         (2048, 4, 190),
                                         pytest.param(4096, 2, 255, marks=pytest.mark.timeout(600))])
def test_capacity_classes_breed_heavy(cap, W, steps):
    """Worlds filling each kernel capacity class under a breed-heavy stream --
    128 and 256 slots (two / four 64-slot groups in K1 and the sensor), 512,
    1024, 2048 and 4096 (4 / 2 / 1 / 1 worlds per K1 block, one wave per world
    in the sensor, 64-bit depth keys): every column and the dropped-birth count
    equal the oracle's after every step."""
    import madrona_bots as mb
    mgr = mb.SimManager(0, W, 69, 32, agent_capacity=cap)
    orc = pyoracle.OracleSim(W, 69, 32, cap=cap, num_threads=16)
    peak = 0
    for t in range(steps):
        n = mgr.num_agents()
        a = _breed_heavy(n, t)
        mgr.action_tensor(False).to_torch().copy_(a.to("cuda"))
        orc.column(pyoracle.COL_ACTION)[:] = a.numpy()
        mgr.step()
        orc.step()
        errs = compare(mgr, orc, f"step {t}")
        assert not errs, errs[:5]
        mgr.shift_observations()
        orc.shift_observations()
        peak = max(peak, int(mgr.species_count_tensor().to_torch().sum(1).max()))
    assert mgr.overflow() == orc.overflow() > 0
    assert peak == cap


@pytest.mark.parametrize("W,steps", [(8, 80), (2100, 30)])
def test_auto_capacity_grows_without_drops(W, steps):
    """agent_capacity="auto" on the device: the breed-heavy stream grows the
    worlds through the capacity classes (cross-capacity checkpoint hand-overs
    before each step that could overflow) and every column stays bitwise equal
    to an oracle that never drops (cap 1024), after every step."""
    import madrona_bots as mb
    mgr = mb.SimManager(0, W, 69, 32, agent_capacity="auto")
    orc = pyoracle.OracleSim(W, 69, 32, cap=1024, num_threads=16)
    seen = {mgr.agent_capacity}
    for t in range(steps):
        n = mgr.num_agents()
        a = _breed_heavy(n, t)
        mgr.action_tensor(False).to_torch().copy_(a.to("cuda"))
        orc.column(pyoracle.COL_ACTION)[:] = a.numpy()
        mgr.step()
        orc.step()
        seen.add(mgr.agent_capacity)
        errs = compare(mgr, orc, f"step {t} cap {mgr.agent_capacity}")
        assert not errs, errs[:5]
        mgr.shift_observations()
        orc.shift_observations()
    assert {128, 256} <= seen
    assert mgr.overflow() == orc.overflow() == 0


def test_max_population_matches_species_counts():
    """mbots_max_population (K2's per-tile maxima in the pinned mirror; after a
    checkpoint load, until the next K2, read from the device) equals the
    largest world of species_count after every step, on the plain and the
    swapped schedule."""
    import ctypes
    import madrona_bots as mb

    def maxpop(m):
        v = ctypes.c_uint32()
        mb._check(mb._lib.mbots_max_population(m._h, ctypes.byref(v)))
        return int(v.value)

    for W in (3000, 16400):
        m = mb.SimManager(0, W, 69, 32)
        for t in range(12):
            a = _breed_heavy(m.num_agents(), t).to("cuda")
            m.action_tensor(False).to_torch().copy_(a)
            m.step()
            assert maxpop(m) == int(m.species_count_tensor().to_torch().sum(1).max()), (W, t)
            m.shift_observations()
        blob = m.save_checkpoint()
        b = mb.SimManager(0, W, 69, 32)
        b.load_checkpoint(blob)
        assert maxpop(b) == maxpop(m)


def test_checkpoint_across_capacities_gpu():
    """A device checkpoint restores into managers of other capacity classes
    (per-slot columns re-laid out world by world) and the runs continue
    bitwise equal; a world that does not fit is refused."""
    import madrona_bots as mb
    a = mb.SimManager(0, 4100, 69, 32)
    for t in range(6):
        a.write_synthetic_actions(1234, t, True)
        a.step()
        a.shift_observations()
    blob = a.save_checkpoint()
    others = [mb.SimManager(0, 4100, 69, 32, agent_capacity=c) for c in (256, 1024)]
    for b in others:
        b.load_checkpoint(blob.tobytes())
    for t in range(6, 10):
        for m in [a] + others:
            m.write_synthetic_actions(1234, t, True)
            m.step()
            m.shift_observations()
    for b in others:
        for name in ("position_tensor", "reward_tensor", "semantic_tensor", "hidden_state_tensor",
                     "action_tensor", "stats_tensor"):
            for prev in (False, True):
                assert torch.equal(getattr(a, name)(prev).to_torch(), getattr(b, name)(prev).to_torch()), \
                    (b.agent_capacity, name, prev)
    with pytest.raises(RuntimeError, match="more than agent_capacity|row count out of range"):
        mb.SimManager(0, 4100, 69, 32, agent_capacity=32).load_checkpoint(blob.tobytes())


@pytest.mark.parametrize("cap,W,steps", [(512, 4100, 24), (256, 16400, 16), (1024, 3000, 20), (2048, 2100, 16),
                                         (4096, 2100, 16)])
def test_mixed_classes_equal_single_class(cap, W, steps, monkeypatch):
    """Mixed capacity classes (the 128-slot K1 and sensor for every world that
    fits them, the class kernels for the worlds K2 lists) against the same
    manager running every world in the class kernels (MBOTS_MIXED=0), under the
    breed-heavy stream that makes some worlds outgrow 128 slots while others do
    not: every column bitwise equal after every step and shift (the
    single-class path is the oracle-checked one above); 16400 worlds take the
    swapped schedule and K2's population order, 4100 the split sensor."""
    import madrona_bots as mb
    monkeypatch.setenv("MBOTS_MIXED", "0")
    ref = mb.SimManager(0, W, 69, 32, agent_capacity=cap)
    monkeypatch.delenv("MBOTS_MIXED")
    mgr = mb.SimManager(0, W, 69, 32, agent_capacity=cap)
    assert mgr.schedule_info()["mixed_classes"] and not ref.schedule_info()["mixed_classes"]
    from simpair import COLUMNS, bits, gpu_column
    big = 0
    for t in range(steps):
        a = _breed_heavy(mgr.num_agents(), t).to("cuda")
        for m in (mgr, ref):
            m.action_tensor(False).to_torch().copy_(a)
            m.step()
        n = mgr.species_count_tensor().to_torch().sum(1)
        k = int((2 * n + 32 > 128).sum())   # worlds the next K1 runs in the class kernel
        big = max(big, k if k < W else 0)
        for where in ("step", "shift"):
            assert mgr.num_agents() == ref.num_agents(), (t, where)
            for name, _ in COLUMNS + [("depth_tensor", None)]:
                for prev in (False, True):
                    g, r = gpu_column(mgr, name, prev), gpu_column(ref, name, prev)
                    assert np.array_equal(bits(g), bits(r)), (t, where, name, prev)
            if where == "step":
                for m in (mgr, ref):
                    m.shift_observations()
    assert mgr.overflow() == ref.overflow()
    assert big > 0   # both kinds of world were on the device at once


@pytest.mark.parametrize("cap,W", [(512, 4100), (1024, 8192)])
def test_large_capacity_classes_bench_stream(cap, W):
    """The 512 / 1024-slot classes at world counts past the split sensor and
    the K1 finder mode (4100: no population order; 8192: K2's population order
    and the value-wait fork / join) on the bench's synthetic stream, against
    the oracle after every step and shift."""
    import madrona_bots as mb
    mgr = mb.SimManager(0, W, 69, 32, agent_capacity=cap)
    orc = pyoracle.OracleSim(W, 69, 32, cap=cap, num_threads=16)
    for t in range(6):
        for s in (mgr, orc):
            s.write_synthetic_actions(1234, t, True)
            s.step()
        errs = compare(mgr, orc, f"step {t}")
        assert not errs, errs[:5]
        mgr.shift_observations()
        orc.shift_observations()
        errs = compare(mgr, orc, f"shift {t}")
        assert not errs, errs[:5]


@pytest.mark.parametrize("W,cap", [(64, 128), (1024, 128), (4100, 128), (4100, 512)])
def test_graph_capture_replays_match_oracle(W, cap):
    """Steps recorded into a HIP graph (torch.cuda.graph; the fork / join
    events become capturable records, mbots_join ends the capture) and replayed
    equal the same call sequence run eagerly on the oracle, bitwise.  A replay
    repeats the captured action-stream step numbers; the oracle mirrors that.
    (cap 512: the mixed capacity classes' K2 lists and class kernels inside
    the graph.)"""
    import madrona_bots as mb
    mgr = mb.SimManager(0, W, 69, 32, agent_capacity=cap)
    orc = pyoracle.OracleSim(W, 69, 32, cap=cap, num_threads=8)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for t in range(3):
            mgr.write_synthetic_actions(1234, t)
            orc.write_synthetic_actions(1234, t)
            mgr.step(); orc.step()
            mgr.shift_observations(); orc.shift_observations()
        mgr.write_synthetic_actions(1234, 3)
        orc.write_synthetic_actions(1234, 3)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):   # records, runs nothing
            mgr.step(); mgr.shift_observations(); mgr.write_synthetic_actions(1234, 4)
            mgr.step(); mgr.shift_observations(); mgr.write_synthetic_actions(1234, 5)
            mgr.join()
    # replays and reads on torch's default stream, not the recording stream:
    # the accessors run their deferred copies on the reader's stream, after
    # what the manager enqueued (mbots_export_on)
    for _ in range(3):
        g.replay()
        for t in (4, 5):
            orc.step(); orc.shift_observations(); orc.write_synthetic_actions(1234, t)
    errs = compare(mgr, orc, f"graph W={W}")
    assert not errs, errs[:5]


VIEW_NAMES = ("species_tensor", "position_tensor", "health_tensor", "surrounding_tensor", "reward_tensor",
              "action_tensor", "stats_tensor", "hidden_state_tensor", "semantic_tensor")


@pytest.mark.parametrize("W", [1024, 4100])
def test_views_read_on_another_stream(W):
    """Steps on stream A, every view (current and Prev*) read and copied on
    stream B without any host synchronisation in between: B's reads are
    ordered after A's step and after the deferred copies the accessors
    enqueue (mbots_export_on), bitwise against the oracle after every step
    and every shift (the reference's synchronous step makes its views valid on
    any stream, mgr.cpp:51-63)."""
    import madrona_bots as mb
    from simpair import COLUMNS, bits
    mgr = mb.SimManager(0, W, 69, 32)
    orc = pyoracle.OracleSim(W, 69, 32, num_threads=8)
    a, b = torch.cuda.Stream(), torch.cuda.Stream()

    def read_on_b(where):
        with torch.cuda.stream(b):
            got = {(nm, p): getattr(mgr, nm)(p).to_torch().clone() for nm in VIEW_NAMES for p in (False, True)}
            got[("depth_tensor", False)] = mgr.depth_tensor(False).to_torch().clone()
        b.synchronize()
        errs = []
        for nm, cid in COLUMNS:
            for p in (False, True):
                g, o = got[(nm, p)].cpu().numpy(), orc.column(cid, p)
                if g.shape != o.shape or not np.array_equal(bits(g), bits(o)):
                    errs.append(f"{where}: {nm}(prev={p})")
        if not np.array_equal(got[("depth_tensor", False)].cpu().numpy(),
                              orc.column(pyoracle.COL_SEMANTIC).view(np.uint8)):
            errs.append(f"{where}: depth_tensor")
        return errs

    errs = []
    for t in range(5):
        with torch.cuda.stream(a):
            mgr.write_synthetic_actions(1234, t, True)
            mgr.step()
        orc.write_synthetic_actions(1234, t, True)
        orc.step()
        errs += read_on_b(f"step {t}")
        with torch.cuda.stream(a):
            mgr.shift_observations()
        orc.shift_observations()
        errs += read_on_b(f"shift {t}")
    assert not errs, errs[:5]


def test_graph_capture_rejects_host_reads_and_odd_step_counts():
    """under stream capture a host-side agent count would be baked
    into every replay, so accessors that need it fail loudly; and a captured
    sequence must hold an even number of steps (the table halves alternate),
    which mbots_join checks."""
    import madrona_bots as mb
    mgr = mb.SimManager(0, 64, 69, 32)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        mgr.write_synthetic_actions(1234, 0)
        mgr.step(); mgr.shift_observations(); mgr.write_synthetic_actions(1234, 1)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            mgr.step(); mgr.shift_observations(); mgr.write_synthetic_actions(1234, 2)
            with pytest.raises(RuntimeError, match="even number of steps"):
                mgr.join()
            with pytest.raises(RuntimeError, match="captured into a graph"):
                mgr.num_agents()
            mgr.step(); mgr.shift_observations(); mgr.write_synthetic_actions(1234, 3)
            mgr.join()
    g.replay()
    torch.cuda.synchronize()
    assert mgr.num_agents() > 0
    # a capture that ends without join() and holds an odd number of steps --
    # possible from C, where mbots_pack_rollout into a preallocated buffer also
    # joins the sensor -- is reported by the next step
    import ctypes
    buf = torch.empty((4096, mgr.rollout_record_bytes()), dtype=torch.uint8, device="cuda")
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        torch.cuda.synchronize()
        with torch.cuda.graph(g2, stream=s):
            mgr.step(); mgr.shift_observations()
            assert mb._lib.mbots_pack_rollout(mgr._h, ctypes.c_void_p(buf.data_ptr()), buf.shape[0],
                                              ctypes.c_void_p(s.cuda_stream)) == 0
    with pytest.raises(RuntimeError, match="odd number of steps"):
        mgr.step()
    # ... and from then on by every entry point, since the host's table
    # halves no longer follow the device (accessors and writers
    # used to read or write the wrong half silently)
    with pytest.raises(RuntimeError, match="odd number of steps"):
        mgr.num_agents()
    with pytest.raises(RuntimeError, match="odd number of steps"):
        mgr.position_tensor()
    with pytest.raises(RuntimeError, match="odd number of steps"):
        mgr.write_synthetic_actions(1234, 9)
    with pytest.raises(RuntimeError, match="odd number of steps"):
        mgr.save_checkpoint()


@pytest.mark.parametrize("fix_depth", [False, True])
def test_agents_driven_into_the_walls(fix_depth):
    """Every agent walks forward into the +x wall, turns about and walks into
    the -x wall, so the population piles up against the walls: near points inside the wall boxes
    and beyond them (semantic -1), agents on the boundary itself (not strictly
    inside the inner rectangle) -- the sensor's wall fix-up on most agents.
    Actions are written through the action views of both sides; the whole
    table is compared with the oracle every 10 steps."""
    import madrona_bots as mb
    W = 32
    mgr = mb.SimManager(0, W, 69, 32, fix_depth_alias=fix_depth)
    orc = pyoracle.OracleSim(W, 69, 32, num_threads=8)
    saw_miss = saw_wall = False
    # forward to the +x wall, turn about (31 x 0.1 rad), forward to the -x
    # wall: near points inside the +x wall box, then beyond the -x one
    for t in range(260):
        k = 2 if 100 <= t < 131 else 0   # rotate left / forward (sim.cpp:419-502)
        a = mgr.action_tensor(False).to_torch()
        a.zero_()
        a[:, k] = 1
        o = orc.column(pyoracle.COL_ACTION)
        o[:] = 0
        o[:, k] = 1
        mgr.step()
        orc.step()
        mgr.shift_observations()
        orc.shift_observations()
        if t % 10 == 9:
            errs = compare(mgr, orc, f"step {t}", depth_fixed=fix_depth)
            assert not errs, errs[:5]
            sem = mgr.semantic_tensor(False).to_torch().cpu()
            saw_miss |= bool((sem == -1).any())
            saw_wall |= bool((sem == 5).any())
    x = mgr.position_tensor(False).to_torch().cpu()
    edge = (x[:, 0] <= 0.2) | (x[:, 0] >= 127.0) | (x[:, 1] <= 0.2) | (x[:, 1] >= 95.0)
    assert edge.float().mean() > 0.2, "the agents should be at the walls by now"
    assert saw_miss and saw_wall
