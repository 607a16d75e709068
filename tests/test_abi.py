"""CPU: the C-ABI libraries load and export every symbol their headers declare
(no compute calls -- there is no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "madrona-bots_amd", "madrona_bots", "libmbots.so")


def declared(header):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mbots_[a-z_]+|orc_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_the_reference_surface():
    names = declared(os.path.join(ROOT, "include", "mbots.h"))
    for fn in ("mbots_create", "mbots_destroy", "mbots_step", "mbots_shift_observations",
               "mbots_num_agents", "mbots_export", "mbots_set_action",
               "mbots_agent_offset_for_world", "mbots_last_error"):
        assert fn in names


def test_libmbots_exports_all_declared_symbols():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared(os.path.join(ROOT, "include", "mbots.h"))
               if not hasattr(lib, n)]
    assert not missing, missing


def test_liborc_exports_all_declared_symbols():
    import pyoracle
    lib = pyoracle.lib()
    missing = [n for n in declared(os.path.join(ROOT, "oracle", "mbots_oracle.h"))
               if not hasattr(lib, n)]
    assert not missing, missing


def test_python_module_imports_and_fails_loudly_without_gpu():
    import torch
    import madrona_bots as mb
    assert hasattr(mb, "SimManager") and hasattr(mb.madrona, "Tensor")
    for m in ("step", "shift_observations", "depth_tensor", "semantic_tensor",
              "reward_tensor", "species_count_tensor", "position_tensor", "health_tensor",
              "surrounding_tensor", "action_tensor", "stats_tensor", "hidden_state_tensor"):
        assert callable(getattr(mb.SimManager, m))
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError, match="madrona_bots"):
            mb.SimManager(0, 4, 69, 32)
    # the library reports invalid configs before touching the device
    with pytest.raises(RuntimeError):
        mb.SimManager(0, 0, 69, 32)
