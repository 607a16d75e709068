"""Helpers that drive the HIP product (madrona_bots) and the CPU oracle
(oracle/pyoracle.py, test infrastructure) through the same call sequence and
compare every exported column."""
import numpy as np

import pyoracle

# (accessor name, oracle column id, view dtype for bitwise compare)
COLUMNS = [
    ("species_tensor", pyoracle.COL_SPECIES),
    ("position_tensor", pyoracle.COL_POS),
    ("health_tensor", pyoracle.COL_HEALTH),
    ("surrounding_tensor", pyoracle.COL_SURROUND),
    ("reward_tensor", pyoracle.COL_REWARD),
    ("action_tensor", pyoracle.COL_ACTION),
    ("stats_tensor", pyoracle.COL_STATS),
    ("hidden_state_tensor", pyoracle.COL_HIDDEN),
    ("semantic_tensor", pyoracle.COL_SEMANTIC),
]


def gpu_column(mgr, name, is_prev):
    t = getattr(mgr, name)(is_prev).to_torch()
    return t.cpu().numpy()


def bits(a):
    a = np.ascontiguousarray(a)
    if a.dtype.itemsize == 4:
        return a.view(np.uint32)
    return a.view(np.uint8)


def compare(mgr, orc, where, prev_too=True, depth_fixed=False):
    """Bitwise comparison of every exported column; returns list of errors."""
    errs = []
    n_g, n_o = mgr.num_agents(), orc.num_agents()
    if n_g != n_o:
        return [f"{where}: num_agents gpu={n_g} oracle={n_o}"]
    sc_g = mgr.species_count_tensor().to_torch().cpu().numpy()
    if not np.array_equal(sc_g, orc.species_count()):
        errs.append(f"{where}: species_count differs")
    cols = list(COLUMNS)
    for name, cid in cols:
        for is_prev in ((False, True) if prev_too else (False,)):
            g = gpu_column(mgr, name, is_prev)
            o = orc.column(cid, is_prev)
            if g.shape != o.shape:
                errs.append(f"{where}: {name}(prev={is_prev}) shape {g.shape} vs {o.shape}")
                continue
            gb, ob = bits(g), bits(o)
            bad = np.nonzero((gb != ob).reshape(len(gb), -1).any(axis=1))[0]
            if len(bad):
                r = bad[0]
                errs.append(f"{where}: {name}(prev={is_prev}) {len(bad)} rows differ; "
                            f"first row {r}: gpu={g[r]} oracle={o[r]}")
    # depth_tensor: the reference exports the semantic buffer (B.1)
    dg = gpu_column(mgr, "depth_tensor", False)
    if depth_fixed:
        do = orc.column(pyoracle.COL_DEPTH)
    else:
        do = orc.column(pyoracle.COL_SEMANTIC).view(np.uint8)
    if not np.array_equal(dg, do):
        errs.append(f"{where}: depth_tensor differs")
    if depth_fixed and prev_too:   # (aliased, the prev depth is the prev semantic above)
        if not np.array_equal(gpu_column(mgr, "depth_tensor", True), orc.column(pyoracle.COL_DEPTH, True)):
            errs.append(f"{where}: depth_tensor(prev=True) differs")
    return errs
