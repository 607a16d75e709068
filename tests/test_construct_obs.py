"""Fused learner observation rows (SimManager.construct_obs, the HIP
construct_obs kernel) against learn/util.py:14-29's torch.cat of the exported
views (madrona-bots_amd/harness/rollout.py construct_obs), bit for bit."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd", "harness"))

import rollout  # noqa: E402


def _bits(t):
    return t.contiguous().view(torch.int32)


@pytest.mark.gpu
@pytest.mark.parametrize("fix_depth", [False, True])
def test_fused_obs_equals_torch_cat(fix_depth):
    import madrona_bots as mb
    sim = mb.SimManager(0, 512, 69, 32, fix_depth_alias=fix_depth)
    sim.write_synthetic_actions(1234, 0)
    for t in range(6):
        sim.step()
        for prev in (False, True):
            fused = sim.construct_obs(prev)
            assert fused.shape == (sim.num_agents(), rollout.OBS_DIM)
            for s, e in rollout.species_offsets(sim):
                ref = rollout.construct_obs(sim, s, e, prev=prev)
                assert torch.equal(_bits(fused[s:e]), _bits(ref)), (t, prev, s, e)
        sim.shift_observations()
        # after the (lazy) shift: Prev rows read through the current columns
        fused = sim.construct_obs(True)
        for s, e in rollout.species_offsets(sim):
            ref = rollout.construct_obs(sim, s, e, prev=True)
            assert torch.equal(_bits(fused[s:e]), _bits(ref)), (t, "shifted", s, e)
        sim.write_synthetic_actions(1234, t + 1)


@pytest.mark.gpu
def test_fused_obs_out_buffer():
    import madrona_bots as mb
    sim = mb.SimManager(0, 64, 7, 16)
    sim.step()
    n = sim.num_agents()
    buf = torch.full((n + 5, rollout.OBS_DIM), -7.0, device="cuda")
    out = sim.construct_obs(False, out=buf)
    assert out.data_ptr() == buf.data_ptr() and out.shape[0] == n
    assert torch.all(buf[n:] == -7.0)
    with pytest.raises(ValueError):
        sim.construct_obs(False, out=torch.empty((n - 1, rollout.OBS_DIM), device="cuda"))


@pytest.mark.gpu
def test_prev_obs_gathers_the_deferred_move():
    """construct_obs(True) right after step(), with no Prev* view read in
    between (the reference loop's pattern, training_loop.py:86): the six Prev*
    columns are still the step's deferred move, so the kernel gathers health /
    position / surrounding from the other half along src_of (newborn rows
    zero).  Compared bit for bit with the CPU mode, which moves eagerly, every
    step; a breed-heavy action stream makes newborn rows."""
    import madrona_bots as mb
    hip = mb.SimManager(0, 256, 69, 32)
    cpu = mb.SimManager(0, 256, 69, 32, exec_mode="cpu")
    for m in (hip, cpu):
        m.write_synthetic_actions(1234, 0, True)
    for t in range(10):
        for m in (hip, cpu):
            m.step()
        assert hip.num_agents() == cpu.num_agents()
        for prev in (True, False):
            a = hip.construct_obs(prev).cpu()
            b = cpu.construct_obs(prev)
            assert torch.equal(_bits(a), _bits(b)), (t, prev)
        for m in (hip, cpu):
            m.shift_observations()
            m.write_synthetic_actions(1234, t + 1, True)
    # and the columns a later accessor materialises agree as well
    hip.step(); cpu.step()
    a = hip.construct_obs(True).cpu()
    assert torch.equal(_bits(a), _bits(cpu.construct_obs(True)))
    for k in ("position_tensor", "health_tensor", "surrounding_tensor"):
        x = getattr(hip, k)(True).to_torch().cpu()
        y = getattr(cpu, k)(True).to_torch()
        assert torch.equal(x.contiguous().view(torch.int32), y.contiguous().view(torch.int32)), k
