"""CPU: known-answer tests of the oracle (oracle/mbots_oracle.c), hand-derived
from the cited reference formulas, plus independent numpy restatements of the
small systems.  No GPU needed."""
import numpy as np
import pytest

import pyoracle as po


def f32(x):
    return np.float32(x)


# ---------------------------------------------------------------------------
# RNG: Threefry-2x32-20 known-answer vectors published with Random123
# (kat_vectors: "threefry2x32 20 <ctr0> <ctr1> <key0> <key1> <out0> <out1>")
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("ctr,key,out", [
    ((0x00000000, 0x00000000), (0x00000000, 0x00000000), (0x6b200159, 0x99ba4efe)),
    ((0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff), (0x1cb996fc, 0xbb002be7)),
    ((0x243f6a88, 0x85a308d3), (0x13198a2e, 0x03707344), (0xc4923a9c, 0x483df7a0)),
])
def test_threefry_kat(ctr, key, out):
    assert po.threefry2x32(key, ctr) == out


def test_samplers():
    L = po.lib()
    assert L.orc_sample_uniform(0) == 0.0
    assert L.orc_sample_uniform(0xFFFFFFFF) == f32(16777215 / 16777216)
    for bits in (0, 1, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF, 12345678):
        v = L.orc_sample_i32(bits, 0, 10)
        assert 0 <= v < 10 and v == (bits * 10) >> 32
        assert 1 <= L.orc_sample_i32(bits, 1, 3) < 3


def _rows_by_species(sim):
    """A=4, one agent per species, no deaths: row r holds species r+1."""
    sp = sim.column(po.COL_SPECIES).ravel()
    assert list(sp) == [1, 2, 3, 4]


# ---------------------------------------------------------------------------
# actionSystem (sim.cpp:419-502)
# ---------------------------------------------------------------------------
def test_forward_step_moves_plus_one_x():
    sim = po.OracleSim(1, 69, 4, cap=16)
    _rows_by_species(sim)
    p0 = sim.column(po.COL_POS).copy()
    act = sim.column(po.COL_ACTION)
    act[:] = 0
    act[:, 0] = 1                       # forward
    sim.step()
    _rows_by_species(sim)
    p1 = sim.column(po.COL_POS)
    # identity rotation: view_dir = (1 - 2*0, 2*0*1) = (1, 0) exactly
    exp_x = np.minimum(f32(127.0), np.maximum(f32(0.0), p0[:, 0] + f32(1.0)))
    assert np.array_equal(p1[:, 0], exp_x)
    assert np.array_equal(p1[:, 1], p0[:, 1])


def test_rotate_left_ten_times_then_forward():
    sim = po.OracleSim(1, 3, 4, cap=16)
    act = sim.column(po.COL_ACTION)
    for _ in range(10):
        act = sim.column(po.COL_ACTION)
        act[:] = 0
        act[:, 2] = 1                   # rotateLeft: rot *= angleAxis(0.1, z)
        sim.step()
    p0 = sim.column(po.COL_POS).copy()
    act = sim.column(po.COL_ACTION)
    act[:] = 0
    act[:, 0] = 1
    sim.step()
    d = sim.column(po.COL_POS) - p0
    want = np.array([np.cos(1.0), np.sin(1.0)])
    for k in range(4):
        x, y = p0[k]
        if 2 < x < 125 and 2 < y < 93:          # not clamped by the walls
            assert np.allclose(d[k], want, atol=1e-5), (d[k], want)


# ---------------------------------------------------------------------------
# speciesInfoSync (sim.cpp:791-838) + rewardSystem setting 8 (sim.cpp:942-956)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("fixed", [False, True])
def test_reward_no_events(fixed):
    sim = po.OracleSim(1, 69, 4, cap=16, reward_fixed=fixed)
    act = sim.column(po.COL_ACTION)
    act[:] = 0
    sim.step()
    _rows_by_species(sim)
    assert not sim.column(po.COL_STATS).any()
    assert list(sim.column(po.COL_HEALTH).ravel()) == [100] * 4
    # rewards[i] = count/A + avg/100 - 2 = 1/4 + 1 - 2 = -0.75
    sr = f32(f32(f32(1.0) / f32(4.0)) + f32(f32(100.0) / f32(100.0))) - f32(2.0)
    r_own = f32(f32(sr + f32(f32(100.0) / f32(100.0))) - f32(0.5))
    rew = sim.column(po.COL_REWARD).ravel()
    if fixed:
        assert list(rew) == [r_own] * 4
    else:
        # faithful rewards[speciesID]: species 1..3 read rewards[1..3] (= -0.75),
        # species 4 reads past the array -> 0 for the table's last world (B.3)
        r4 = f32(f32(f32(0.0) + f32(1.0)) - f32(0.5))
        assert list(rew) == [r_own, r_own, r_own, r4]


def test_respawn_refills_species():
    # A = 4: any species that drops below A/4 = 1 is respawned in the same step
    sim = po.OracleSim(16, 5, 4, cap=16)
    for t in range(40):
        sim.write_synthetic_actions(99, t)
        sim.step()
        assert (sim.species_count() >= 1).all()


# ---------------------------------------------------------------------------
# updateSurroundingObservation (sim.cpp:583-654): numpy float32 restatement
# ---------------------------------------------------------------------------
def _chunk_index(cx, cy):
    x, y = int(cx), int(cy)
    if x < 0 or y < 0 or x >= 8 or y >= 6:
        return -1
    return x + y * 8


def test_surrounding_matches_numpy_restatement():
    W = 4
    sim = po.OracleSim(W, 69, 32, cap=128)
    p0 = sim.column(po.COL_POS).copy()
    act = sim.column(po.COL_ACTION)
    act[:] = 0          # no actions: the only motion is the clamp to [0, Lx-1] x [0, Ly-1]
    sim.step()
    assert sim.num_agents() == W * 32        # nobody born or died: rows are stable
    pos = sim.column(po.COL_POS)
    sur = sim.column(po.COL_SURROUND)
    # clamp (sim.cpp:485-486) and the speed heuristic (u32)(2 |dpos|) (sim.cpp:488-501)
    assert np.array_equal(pos[:, 0], np.minimum(f32(127), np.maximum(f32(0), p0[:, 0])))
    assert np.array_equal(pos[:, 1], np.minimum(f32(95), np.maximum(f32(0), p0[:, 1])))
    d = pos - p0
    speed = (np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) * f32(2)).astype(np.uint32)
    # export rows are ordered (species, world, slot): rebuild per-world row lists
    sc = sim.species_count()
    row = 0
    rows_of = {w: [] for w in range(W)}
    for s in range(4):
        for w in range(W):
            rows_of[w] += list(range(row, row + sc[w, s]))
            row += sc[w, s]
    for w in range(W):
        rr = rows_of[w]
        n_ag = np.zeros(48, np.uint32)
        t_sp = np.zeros(48, np.uint32)
        for r in rr:
            c = _chunk_index(np.floor(pos[r, 0] / f32(16)), np.floor(pos[r, 1] / f32(16)))
            n_ag[c] += 1
            t_sp[c] += speed[r]
        for r in rr:
            cpx = pos[r, 0] - f32(8.0)
            cpy = pos[r, 1] - f32(8.0)
            chx, chy = cpx / f32(16), cpy / f32(16)
            x0, y0, x1, y1 = np.floor(chx), np.floor(chy), np.ceil(chx), np.ceil(chy)
            idx = [_chunk_index(x0, y0), _chunk_index(x1, y0), _chunk_index(x0, y1),
                   _chunk_index(x1, y1)]
            xi, yi = chx - x0, chy - y0
            for col, cnt in ((0, n_ag), (1, t_sp)):
                n = [f32(cnt[i]) if i >= 0 else f32(0) for i in idx]
                nx0 = xi * n[1] + (f32(1) - xi) * n[0]
                nx1 = xi * n[3] + (f32(1) - xi) * n[2]
                want = yi * nx1 + (f32(1) - yi) * nx0
                assert sur[r, col] == want, (w, r, col, sur[r, col], want)


def test_surround_at_chunk_centroid_is_that_count():
    # at a chunk centroid (8 + 16 i, 8 + 16 j) the interpolants are 0 and the
    # presence heuristic is exactly that chunk's agent count
    chx = (f32(8 + 16 * 3) - f32(8)) / f32(16)
    assert chx - np.floor(chx) == 0.0


# ---------------------------------------------------------------------------
# Export invariants and shift_observations (sim.cpp:1002-1048)
# ---------------------------------------------------------------------------
def test_export_invariants_and_shift():
    sim = po.OracleSim(32, 11, 32, cap=128)
    for t in range(30):
        sim.write_synthetic_actions(1234, t, True)
        sim.step()
        N = sim.num_agents()
        sc = sim.species_count()
        assert sc.sum() == N
        sp = sim.column(po.COL_SPECIES).ravel()
        assert (np.diff(sp) >= 0).all()             # species-major rows
        assert list(np.bincount(sp, minlength=5)[1:]) == list(sc.sum(0))
        assert (sim.column(po.COL_HEALTH) > 0).all()
        sem = sim.column(po.COL_SEMANTIC)
        assert set(np.unique(sem).tolist()) <= {-1, 1, 2, 3, 4, 5, 6}   # -1: a miss
        sim.shift_observations()
        for c in (po.COL_SPECIES, po.COL_POS, po.COL_HEALTH, po.COL_SURROUND, po.COL_REWARD,
                  po.COL_ACTION, po.COL_HIDDEN):
            assert np.array_equal(sim.column(c), sim.column(c, True))
        st, pst = sim.column(po.COL_STATS), sim.column(po.COL_STATS, True)
        assert np.array_equal(pst[:, [0, 2, 3]], st[:, [0, 2, 3]])
        assert np.array_equal(pst[:, 1], st[:, 0])  # hitEnemy <- hitFriendly (sim.cpp:1034)
    assert sim.overflow() == 0


def test_prev_sensor_is_last_steps_sensor():
    sim = po.OracleSim(1, 69, 4, cap=16)
    act = sim.column(po.COL_ACTION)
    act[:] = 0
    sim.step()
    sem0 = sim.column(po.COL_SEMANTIC).copy()
    act = sim.column(po.COL_ACTION)
    act[:] = 0
    act[:, 2] = 1
    sim.step()
    _rows_by_species(sim)
    assert np.array_equal(sim.column(po.COL_SEMANTIC, True), sem0)


def test_health_export_is_int_bits():
    # health_tensor views int32 health as float32 (types.hpp:119-124, mgr.cpp:329-346)
    h = np.array([100], np.int32).view(np.float32)[0]
    assert h == np.float32(1.4e-43)


# ---- food boxes (the +-1 cube of sim.cpp:332-341, rotated) ----
FWD = list(range(24))


def _hit_pixels(hit):
    return [k for k in range(33) if hit[k]]


def test_food_box_axis_aligned_ahead():
    # box centre 10 ahead, rotation 0: spans Y in [-1, 1] from X = 9, so the
    # line Y = u X meets it iff |u| <= 1/9: pixels 11, 12 (u = -+1/24) + finder
    hit, z = po.probe_box((20.0, 20.0), (1.0, 0.0), (30.0, 20.0), 0)
    assert _hit_pixels(hit) == [11, 12, 32]
    assert z[11] == z[12] == z[32] == 9.0          # nearest face at view depth 9


def test_food_box_diagonal_is_wider_and_nearer():
    # a quarter-turn fraction 1/2 (45 degrees): corners at sqrt 2 on the
    # diagonals, |u| <= sqrt(2)/10 = 0.141 covers pixels 10..13 (u = -+0.125)
    hit, z = po.probe_box((20.0, 20.0), (1.0, 0.0), (30.0, 20.0), 1 << 21)
    assert _hit_pixels(hit) == [10, 11, 12, 13, 32]
    assert abs(float(z[10]) - (10.0 - 2.0 ** 0.5)) < 1e-3
    # rotation by a full quarter turn is the same square as rotation 0
    hit_q, z_q = po.probe_box((20.0, 20.0), (1.0, 0.0), (30.0, 20.0), (1 << 22) - 1)
    assert _hit_pixels(hit_q) == [11, 12, 32]


def test_food_box_behind_uses_backward_camera():
    # backward pixels 24..31 at u = (2k+1)/8 - 1: only the 45-degree box reaches
    # |u| = 0.125 (pixels 27, 28); no forward pixel, no finder
    hit, _ = po.probe_box((50.0, 20.0), (1.0, 0.0), (40.0, 20.0), 0)
    assert _hit_pixels(hit) == []
    hit, z = po.probe_box((50.0, 20.0), (1.0, 0.0), (40.0, 20.0), 1 << 21)
    assert _hit_pixels(hit) == [27, 28]
    assert abs(float(z[27]) - (10.0 - 2.0 ** 0.5)) < 1e-3


def test_food_box_containing_the_agent_near_sphere():
    # the agent at the centre of an axis-aligned box, heading +x: ray (1, u)
    # leaves the box at X = 1, t = sqrt(1 + u^2), seen iff t >= 1.1 (nearSphere,
    # mgr.cpp:133): |u| >= 0.458 -> forward pixels 0..6, 17..23, backward
    # u = +-7/8, +-5/8 (24, 25, 30, 31); the finder (t = 1) sees nothing of it
    hit, z = po.probe_box((20.0, 20.0), (1.0, 0.0), (20.0, 20.0), 0)
    assert _hit_pixels(hit) == list(range(7)) + list(range(17, 26)) + [30, 31]
    assert (z[hit] == 0.0).all()


# ---- the near sphere and the agent disc -------------------
R_AGENT, NEAR = 0.92, 1.1


def _dirs(heading):
    """World directions of the 33 rays (float64): 24 forward, 8 backward, finder."""
    hx, hy = heading
    out = []
    for k in range(33):
        u = (2 * k - 23) / 24 if k < 24 else ((2 * (k - 24) - 7) / 8 if k < 32 else 0.0)
        sg = -1.0 if 24 <= k < 32 else 1.0
        out.append((sg * (hx + u * hy), sg * (hy - u * hx)))
    return np.array(out)


def _ref_disc(agent, heading, centre, R=R_AGENT):
    """Independent float64 restatement: ray k sees the disc iff it leaves it at
    distance >= 1.1; returns (hit[33], margin[33]) -- margin: how far the ray
    is from either decision boundary (tangency, t_exit = 1.1)."""
    d = _dirs(heading)
    d /= np.linalg.norm(d, axis=1)[:, None]
    v = np.array(centre, np.float64) - np.array(agent, np.float64)
    tm = d @ v
    dist2 = v @ v - tm * tm
    half = np.sqrt(np.maximum(R * R - dist2, 0.0))
    hit = (dist2 <= R * R) & (tm + half >= NEAR)
    margin = np.minimum(np.abs(R * R - dist2), np.where(dist2 <= R * R, np.abs(tm + half - NEAR), 1.0))
    return hit, margin


def _ref_box(agent, heading, centre, rot22):
    """float64 slab restatement for a food square (rotation = quarter-turn
    fraction * pi/2): hit iff the ray's parameter interval in the square is
    non-empty and it exits at distance >= 1.1."""
    w = rot22 * (np.pi / 2) / 4194304.0
    a1 = np.array([np.cos(w), np.sin(w)])
    a2 = np.array([-np.sin(w), np.cos(w)])
    d = _dirs(heading)
    d /= np.linalg.norm(d, axis=1)[:, None]
    o = np.array(agent, np.float64) - np.array(centre, np.float64)
    lo = np.full(33, -np.inf)
    hi = np.full(33, np.inf)
    for ax in (a1, a2):
        b = d @ ax
        m = o @ ax
        with np.errstate(divide="ignore", invalid="ignore"):
            t1, t2 = (-1.0 - m) / b, (1.0 - m) / b
        lo = np.maximum(lo, np.where(b != 0, np.minimum(t1, t2), np.where(abs(m) <= 1, -np.inf, np.inf)))
        hi = np.minimum(hi, np.where(b != 0, np.maximum(t1, t2), np.where(abs(m) <= 1, np.inf, -np.inf)))
    hit = (lo <= hi) & (hi >= NEAR)
    margin = np.minimum(np.abs(hi - lo), np.abs(hi - NEAR))
    return hit, margin


def test_disc_at_1_5_ahead():
    # centre 1.5 ahead: the line reaches the 0.92 disc for |u| <= 0.777 (pixels
    # 3..20) and every such ray leaves it beyond 1.1; depth f - R = 0.58
    hit, z = po.probe_agent((30.0, 30.0), (1.0, 0.0), (31.5, 30.0))
    assert _hit_pixels(hit) == list(range(3, 21)) + [32]
    assert (np.abs(z[hit] - 0.58) < 1e-3).all()
    ref, _ = _ref_disc((30.0, 30.0), (1.0, 0.0), (31.5, 30.0))
    assert np.array_equal(hit, ref)


def test_disc_at_0_9_ahead_overlapping_bodies():
    # centre 0.9 ahead: the camera lies inside the other agent's disc; rays see
    # its far side where it reaches past the near sphere (the finder does:
    # its near point (1.1, 0) is 0.2 from the centre); depth clamps at 0
    hit, z = po.probe_agent((30.0, 30.0), (1.0, 0.0), (30.9, 30.0))
    ref, margin = _ref_disc((30.0, 30.0), (1.0, 0.0), (30.9, 30.0))
    assert margin.min() > 1e-4
    assert np.array_equal(hit, ref)
    assert hit[32] and hit[:24].any() and not hit[24:32].any()
    assert (z[hit] == 0.0).all()


def test_disc_inside_the_near_sphere_is_invisible():
    # 0.1 + 0.92 < 1.1: the whole disc lies inside the near sphere
    for c in ((30.1, 30.0), (30.0, 30.05), (29.9, 30.0)):
        hit, _ = po.probe_agent((30.0, 30.0), (1.0, 0.0), c)
        assert not hit.any(), c


def test_disc_behind_is_seen_by_backward_pixels():
    hit, z = po.probe_agent((30.0, 30.0), (0.0, 1.0), (30.0, 28.5))
    ref, _ = _ref_disc((30.0, 30.0), (0.0, 1.0), (30.0, 28.5))
    assert np.array_equal(hit, ref)
    assert _hit_pixels(hit) == list(range(25, 31))      # |u| <= 0.777: not +-7/8
    assert (np.abs(z[hit] - 0.58) < 1e-3).all()


def test_disc_and_box_predicates_match_float64_restatement():
    """2000 random (agent, heading, object) configurations within 4 units:
    every ray not within 1e-4 of a decision boundary agrees with the float64
    geometry (discs of radius 0.92, rotated unit squares, near sphere 1.1)."""
    rng = np.random.default_rng(7)
    checked = 0
    for t in range(2000):
        a = rng.uniform(10, 60, 2).astype(np.float32)
        th = rng.uniform(0, 2 * np.pi)
        h = (np.float32(np.cos(th)), np.float32(np.sin(th)))
        c = (a + rng.uniform(-4, 4, 2)).astype(np.float32)
        if t % 2:
            hit, _ = po.probe_agent(a, h, c)
            ref, margin = _ref_disc(a.astype(np.float64), np.array(h, np.float64), c.astype(np.float64))
        else:
            rot = int(rng.integers(0, 1 << 22))
            hit, _ = po.probe_box(a, h, c, rot)
            ref, margin = _ref_box(a.astype(np.float64), np.array(h, np.float64), c.astype(np.float64), rot)
        ok = margin > 1e-4
        assert np.array_equal(hit[ok], ref[ok]), (t, a, h, c)
        checked += int(ok.sum())
    assert checked > 60000


def test_walls_near_sphere_classes():
    # agent 0.5 from the left wall looking at it: every forward near point lies
    # beyond the wall box (x < -0.2): a miss (semantic -1, depth 255); the
    # backward pixels see the right wall's inner face 127.3 away
    sem, dep = po.probe_walls((0.5, 50.0), (-1.0, 0.0))
    assert (sem[:24] == -1).all() and sem[32] == -1 and (dep[:24] == 255).all()
    assert (sem[24:32] == 5).all() and dep[27] == dep[28] == 127
    # 1.0 from it: the central near points fall inside the wall box (the wall,
    # depth s0 = 1.1 / |(1, u)| -> byte 1), the outer ones still in the arena
    # (the wall's face 0.8 ahead along the heading -> byte 0)
    sem, dep = po.probe_walls((1.0, 50.0), (-1.0, 0.0))
    assert (sem[:24] == 5).all() and sem[32] == 5
    assert dep[11] == dep[12] == dep[32] == 1 and dep[0] == dep[23] == 0
    # the arena's middle: every ray ends on a wall
    sem, dep = po.probe_walls((64.0, 48.0), (1.0, 0.0))
    assert (sem == 5).all() and dep[11] == 63 and dep[27] == 63


def test_food_box_rotation_follows_heading_frame():
    # heading +y: a box 10 ahead along +y behaves like the +x case
    hit, z = po.probe_box((20.0, 20.0), (0.0, 1.0), (20.0, 30.0), 0)
    assert _hit_pixels(hit) == [11, 12, 32] and z[11] == 9.0
