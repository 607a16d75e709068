"""GPU: tensor views, shapes/dtypes of the reference accessors (mgr.cpp:199-422)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_tensor_shapes_and_zero_copy():
    import madrona_bots as mb
    m = mb.SimManager(0, 16, 69, 32)
    m.step()
    N = m.num_agents()
    W = 16
    expect = {
        "depth_tensor": (torch.uint8, 32), "semantic_tensor": (torch.int8, 32),
        "reward_tensor": (torch.float32, 1), "position_tensor": (torch.float32, 2),
        "health_tensor": (torch.float32, 1), "surrounding_tensor": (torch.float32, 2),
        "action_tensor": (torch.int32, 6), "stats_tensor": (torch.int32, 4),
        "hidden_state_tensor": (torch.float32, 16),
    }
    for name, (dt, k) in expect.items():
        for prev in (False, True):
            t = getattr(m, name)(prev).to_torch()
            assert t.dtype == dt and tuple(t.shape) == (N, k), (name, t.dtype, t.shape)
            assert t.device.type == "cuda"
    sc = m.species_count_tensor().to_torch()
    assert tuple(sc.shape) == (W, 4) and sc.dtype == torch.int32
    assert int(sc.sum()) == N
    # zero-copy: writing through the view changes what the next view sees
    a = m.action_tensor(False).to_torch()
    a.zero_()
    a[0, 2] = 1
    torch.cuda.synchronize()
    assert int(m.action_tensor(False).to_torch()[0, 2]) == 1
    # health is int32 bits seen as float32
    h = m.health_tensor(False).to_torch().view(torch.int32)
    assert int(h.max()) <= 200 and int(h.min()) > 0


def test_set_action_and_offsets():
    import madrona_bots as mb
    m = mb.SimManager(0, 8, 69, 32)
    m.step()
    m.set_action(3, 1, 0, 0, 0, 0, 1)
    a = m.action_tensor(False).to_torch().cpu().numpy()
    assert list(a[3]) == [1, 0, 0, 0, 0, 1]
    offs = [m.agent_offset_for_world(w) for w in range(8)]
    assert offs[0] == 0 and all(b >= a for a, b in zip(offs, offs[1:]))
    si = m.sensor_index_tensor().to_torch().cpu().numpy().ravel()
    assert sorted(si.tolist()) == list(range(m.num_agents()))


@pytest.mark.parametrize("worlds", [8, 1100])
def test_offsets_and_sensor_index_match_oracle(worlds):
    """agentOffsetForWorld (mgr.cpp:274-277) and sensorIndexTensor
    (mgr.cpp:241-249) against the oracle's world counts and slot -> row map,
    after several steps (deaths, births and respawns move both)."""
    import madrona_bots as mb
    import pyoracle
    m = mb.SimManager(0, worlds, 69, 32)
    o = pyoracle.OracleSim(worlds, 69, 32, num_threads=8)
    for t in range(6):
        m.write_synthetic_actions(1234, t, True)
        o.write_synthetic_actions(1234, t, True)
        m.step(); o.step()
        m.shift_observations(); o.shift_observations()
        counts, offsets = o.world_counts()
        got = np.array([m.agent_offset_for_world(w) for w in range(worlds)])
        assert np.array_equal(got, offsets), t
        si = m.sensor_index_tensor().to_torch().cpu().numpy().ravel()
        assert np.array_equal(si, o.sensor_index()), t
        assert int(counts.sum()) == m.num_agents()
