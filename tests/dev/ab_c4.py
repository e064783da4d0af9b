"""Diagnostic A/B of engine builds on the C4 scenario-group bench (GPU box; timing only):
    python tests/dev/ab_c4.py libks_engine_X.so"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib  # noqa: E402

_lib.LIB_PATH = lib_path(sys.argv[1])
import bench  # noqa: E402

sys.argv = sys.argv[:1] + ["--config", "c4", "--steps", "2", "--warmup", "1"]
bench.main()
