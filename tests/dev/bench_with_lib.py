"""Dev tool (not a test): bench.py on an A/B engine build in build/diag/ (tests/dev/devlib.py) —
e.g. a build of an earlier commit's sources, saved before a change:
    python tests/dev/bench_with_lib.py libks_engine_base.so --no-c4 --no-c5 ...
The provenance check is skipped (the build is of other sources by design)."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from devlib import lib_path  # noqa: E402
from kubesim_amd import _lib  # noqa: E402

_lib.LIB_PATH = lib_path(sys.argv[1])
_lib.source_hash = lambda: None
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
sys.path.insert(0, ROOT)
runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")
