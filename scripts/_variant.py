"""A/B loading for the measurement scripts (never the product, which only
loads the libmbots.so next to its own __init__.py): with MBOTS_LIB set,
`import _variant` imports madrona_bots from a scratch copy of the package whose
libmbots.so is that library, so everything the script (or the program
scripts/run_variant.py runs) does with madrona_bots uses it."""
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load():
    lib = os.environ.get("MBOTS_LIB")
    if not lib:
        return
    lib = os.path.abspath(lib)
    if not os.path.exists(lib):
        sys.exit(f"_variant: MBOTS_LIB={lib} does not exist")
    d = tempfile.mkdtemp(prefix="mbvar_")
    pkg = os.path.join(d, "madrona_bots")
    os.makedirs(pkg)
    shutil.copy(os.path.join(ROOT, "madrona-bots_amd", "madrona_bots", "__init__.py"), pkg)
    os.symlink(lib, os.path.join(pkg, "libmbots.so"))
    sys.path.insert(0, d)
    import madrona_bots
    if not madrona_bots.__file__.startswith(d):
        sys.exit("_variant: madrona_bots was imported before the variant")


_load()
