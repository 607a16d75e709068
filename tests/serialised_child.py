"""Child process of tests/test_robustness.py::test_value_waits_off_under_serialised_dispatch
(not a test module): run the bench's loop at 4096 worlds -- where the step's
hops are hipStreamWaitValue32 waits unless the environment serialises kernel
dispatch (include/mbots.h, "Environment") -- under the environment the parent
set, and compare every column with the oracle after the last step."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "madrona-bots_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import madrona_bots as mb  # noqa: E402
import pyoracle  # noqa: E402
from simpair import compare  # noqa: E402


def main():
    W, steps = int(sys.argv[1]), int(sys.argv[2])
    mgr = mb.SimManager(0, W, 69, 32)
    orc = pyoracle.OracleSim(W, 69, 32, num_threads=8)
    for t in range(steps):
        for m in (mgr, orc):
            m.write_synthetic_actions(1234, t)
            m.step()
            m.shift_observations()
        print(f"step {t}", flush=True)
    errs = compare(mgr, orc, f"after {steps} steps")
    if errs:
        print("MISMATCH", errs[:5], flush=True)
        sys.exit(1)
    print("OK", mgr.num_agents(), flush=True)


if __name__ == "__main__":
    main()
