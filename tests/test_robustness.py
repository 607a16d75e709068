"""Robustness of the host surface:

* views outlive the SimManager that produced them (every torch view holds the
  manager's library handle; no reference cycle through the view cache);
* a world that reaches agent_capacity warns (CapacityWarning) or, with
  strict_capacity=True, raises (CapacityError): the reference's worlds have no
  cap (sim.cpp:561-564, :830-834), so the run silently diverged before;
* the step's value waits stay off under serialised kernel dispatch
  (AMD_SERIALIZE_KERNEL, one of include/mbots.h MBOTS_SERIALISING_ENV), where
  the runtime's polling kernel could otherwise be dispatched before its
  producer and never finish ("Small world counts")."""
import gc
import os
import subprocess
import sys
import warnings

import numpy as np
import pytest
import torch

import pyoracle
from simpair import compare

HERE = os.path.dirname(os.path.abspath(__file__))


def _breed_all(mgr):
    """Every agent breeds (and walks): a same-species target in its finder
    slot then makes a child, so a world fills its slots within a few steps."""
    n = mgr.num_agents()
    a = torch.zeros((n, 6), dtype=torch.int32, device=mgr.device)
    a[:, 5] = 1
    a[::3, 0] = 1
    mgr.write_actions(a)


def _drive_to_cap(mgr, steps=12):
    """Steps a breed-only stream; returns the warnings step() raised."""
    with warnings.catch_warnings(record=True) as got:
        warnings.simplefilter("always")
        for _ in range(steps):
            _breed_all(mgr)
            mgr.step()
            mgr.num_agents()      # the host sees the step's row counts (and the drops)
            mgr.shift_observations()
        mgr.step()                # reported by the step after the counts that show the drops
    return [w for w in got if issubclass(w.category, Warning)]


def _capacity(exec_mode):
    import madrona_bots as mb
    mgr = mb.SimManager(0, 16, 69, 32, exec_mode=exec_mode, agent_capacity=32)
    got = _drive_to_cap(mgr)
    assert mgr.overflow() > 0
    caps = [w for w in got if issubclass(w.category, mb.CapacityWarning)]
    assert caps, [str(w.message) for w in got]
    assert "agent_capacity 32" in str(caps[0].message)
    assert all(not issubclass(w.category, mb.CapacityWarning) or "dropped" in str(w.message) for w in got)
    # strict: the same stream raises (the step still ran)
    strict = mb.SimManager(0, 16, 69, 32, exec_mode=exec_mode, agent_capacity=32, strict_capacity=True)
    with pytest.raises(mb.CapacityError, match="dropped at agent_capacity"):
        _drive_to_cap(strict)
    # a population below the cap never reports
    calm = mb.SimManager(0, 16, 69, 32, exec_mode=exec_mode, agent_capacity=128)
    with warnings.catch_warnings():
        warnings.simplefilter("error", mb.CapacityWarning)
        for t in range(5):
            calm.write_synthetic_actions(1234, t)
            calm.step()
            calm.shift_observations()
    assert calm.overflow() == 0


def _views_outlive(exec_mode):
    import madrona_bots as mb

    def make():
        m = mb.SimManager(0, 32, 69, 32, exec_mode=exec_mode)
        for t in range(3):
            m.write_synthetic_actions(1234, t, True)
            m.step()
            m.shift_observations()
        return m

    # views taken from a manager nobody else references
    pos = make().position_tensor().to_torch()
    hid = make().hidden_state_tensor(True).to_torch()[:, :4]   # a view of a view
    gc.collect()
    junk = [make() for _ in range(2)]   # reuse whatever a freed manager would have released
    ref = make()
    assert torch.equal(pos.cpu(), ref.position_tensor().to_torch().cpu())
    assert torch.equal(hid.cpu(), ref.hidden_state_tensor(True).to_torch()[:, :4].cpu())
    del junk
    # the manager itself is freed by reference counting (no cycle through the view cache)
    import weakref
    m = make()
    m.position_tensor().to_torch()
    r = weakref.ref(m)
    del m
    assert r() is None


def test_views_outlive_manager_cpu():
    _views_outlive("cpu")


def test_capacity_warning_and_strict_cpu():
    _capacity("cpu")


@pytest.mark.gpu
def test_views_outlive_manager_gpu():
    _views_outlive("hip")


@pytest.mark.gpu
def test_capacity_warning_and_strict_gpu():
    _capacity("hip")


@pytest.mark.gpu
@pytest.mark.gpu_first   # conftest runs it before any test touches the GPU in this process
def test_value_waits_off_under_serialised_dispatch():
    """A fresh child Python under AMD_SERIALIZE_KERNEL=3 steps 4096 worlds
    (value-wait size) and matches the oracle, within 120 s."""
    env = dict(os.environ, AMD_SERIALIZE_KERNEL="3")
    env.pop("MBOTS_VALUE_FORK", None)
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "serialised_child.py"), "4096", "10"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "OK" in p.stdout, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])


def test_schedule_info_cpu():
    import madrona_bots as mb
    m = mb.SimManager(0, 8, 69, 32, exec_mode="cpu")
    for _ in range(3):
        m.step()
    info = m.schedule_info()
    assert info["steps"] == 3 and not any(info[k] for k in ("k1_finder", "fork_by_value", "swap"))


@pytest.mark.gpu
def test_value_wait_epoch_wrap(monkeypatch):
    """the value waits' epochs restart from 0 at 0x7FFFFFF0
    (drain the device, clear both signal words, synchronise, count on from 1).
    MBOTS_EPOCH_START starts a 4096-world manager (fork and join by value) a
    few epochs short of the restart; 20 steps of the bench's loop with no host
    read in between -- so the host runs ahead and every step takes the value
    waits -- cross it, and the tables equal the oracle's, then again after
    more steps."""
    import madrona_bots as mb
    W = 4096
    monkeypatch.setenv("MBOTS_EPOCH_START", str(0x7FFFFFF0 - 6))
    mgr = mb.SimManager(0, W, 69, 32)
    monkeypatch.delenv("MBOTS_EPOCH_START")
    info = mgr.schedule_info()
    assert info["fork_by_value"] and info["join_by_value"] and info["epoch"] == 0x7FFFFFF0 - 6
    orc = pyoracle.OracleSim(W, 69, 32, num_threads=8)
    t = 0
    for burst in (20, 5):
        # a spin kernel first, so the host enqueues the whole burst while the
        # device is still busy: every step sees the last sensor unfinished
        torch.cuda._sleep(20_000_000)
        for k in range(burst):
            mgr.write_synthetic_actions(1234, t + k, True)
            mgr.step()
            mgr.shift_observations()
        for k in range(burst):
            orc.write_synthetic_actions(1234, t + k, True)
            orc.step()
            orc.shift_observations()
        t += burst
        errs = compare(mgr, orc, f"after {t} steps")
        assert not errs, errs[:5]
    info = mgr.schedule_info()
    assert info["epoch_wraps"] == 1 and 0 < info["epoch"] < 64, info


@pytest.mark.gpu
def test_capture_guard_refuses_other_stream_without_poisoning():
    """a call on another stream while a capture of the manager's
    steps is still recording (an odd count so far) is refused on its own; the
    capture then ends with an even count and the manager keeps working.  A
    capture that ENDS with an odd count still poisons the manager
    (tests/test_parity_gpu.py)."""
    import madrona_bots as mb
    W = 64
    mgr = mb.SimManager(0, W, 69, 32)
    orc = pyoracle.OracleSim(W, 69, 32, num_threads=8)
    s, other = torch.cuda.Stream(), torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        mgr.write_synthetic_actions(1234, 0)
        orc.write_synthetic_actions(1234, 0)
        mgr.step(); orc.step()
        mgr.shift_observations(); orc.shift_observations()
        mgr.write_synthetic_actions(1234, 1)
        orc.write_synthetic_actions(1234, 1)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
            mgr.step(); mgr.shift_observations(); mgr.write_synthetic_actions(1234, 2)
            with torch.cuda.stream(other):
                with pytest.raises(RuntimeError, match="still recording"):
                    mgr.write_synthetic_actions(1234, 9)
            mgr.step(); mgr.shift_observations(); mgr.write_synthetic_actions(1234, 3)
            mgr.join()
    g.replay()
    for t in (2, 3):
        orc.step(); orc.shift_observations(); orc.write_synthetic_actions(1234, t)
    errs = compare(mgr, orc, "after the capture")
    assert not errs, errs[:5]
