import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "madrona-bots_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "gpu_first: run before every other test (it starts a child "
                                       "process, so this process must not have touched the GPU yet)")


def pytest_collection_modifyitems(config, items):
    first = [it for it in items if it.get_closest_marker("gpu_first")]
    if first:
        items[:] = first + [it for it in items if not it.get_closest_marker("gpu_first")]
