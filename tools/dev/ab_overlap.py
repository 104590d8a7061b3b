"""A/B: bench.py with the block backward's weight-gradient halves overlapped (side stream) or serial.
    python tools/ab_overlap.py {0|1} [bench args]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "graph-physics_amd")]
flag = sys.argv.pop(1) == "1"
from graphphysics.models import _engine  # noqa: E402

_engine.OVERLAP_WGRAD = flag
import bench  # noqa: E402

bench.main()
