"""Debug: run a few steps of a small world count under a finder-check build
(MBOTS_LIB, -DMB_FINDER_CHECK) with kernels serialised, so K1's printf lists
every camera whose computed finder slot differs from the last sensor's."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import _variant  # noqa
import torch
import madrona_bots as mb
m = mb.SimManager(0, int(sys.argv[1]), 69, 32)
for t in range(int(sys.argv[2])):
    m.write_synthetic_actions(1234, t)
    m.step()
    m.shift_observations()
    torch.cuda.synchronize()
print("done", m.num_agents(), flush=True)
