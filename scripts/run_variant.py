#!/usr/bin/env python3
"""Run a Python program with madrona_bots loading the library MBOTS_LIB names
(scripts/_variant.py), in this process (no exec: safe under rocprofv3):

    MBOTS_LIB=build_var/libmbots_x.so python scripts/run_variant.py bench.py --steps 50"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _variant  # noqa: E402,F401

if __name__ == "__main__":
    if sys.argv[1] == "-m":   # run_variant.py -m pytest ...
        mod = sys.argv[2]
        sys.argv = [mod] + sys.argv[3:]
        runpy.run_module(mod, run_name="__main__", alter_sys=True)
    else:
        prog = sys.argv[1]
        sys.argv = sys.argv[1:]
        runpy.run_path(prog, run_name="__main__")
