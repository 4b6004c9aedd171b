"""Diagnostic only: run bench.py against a given build of libgymchess.so (A/B of two builds on
one box without touching the in-tree library).

    python tools/ab_lib.py <path/to/libgymchess.so> [bench.py args...]
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
sys.path.insert(0, ROOT)
from gym_chess_amd import _lib  # noqa: E402

_lib.load(os.path.abspath(sys.argv[1]))
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
