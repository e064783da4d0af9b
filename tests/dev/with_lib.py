"""Dev tool (not a test): run pytest with a diagnostic engine build (build/diag/, tests/dev/devlib.py)
in place of the product library — e.g. a regression test against the pre-fix code:
    python tests/dev/with_lib.py libks_engine_oldballot.so tests/test_engine_gpu_c5.py -k overflow"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from devlib import lib_path  # noqa: E402
from kubesim_amd import _lib  # noqa: E402

_lib.LIB_PATH = lib_path(sys.argv[1])
import pytest  # noqa: E402

sys.exit(pytest.main(sys.argv[2:]))
