"""Dev tools (not tests): where diagnostic engine builds live.  `make -C kubernetes-simulator_amd/csrc
<stamps|chunkdiag|variant|abl>` writes them to build/diag/ (git-ignored, outside the package);
the product library stays kubernetes-simulator_amd/kubesim_amd/libks_engine.so."""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DIAG = os.path.join(ROOT, "build", "diag")


def lib_path(name: str) -> str:
    if name == "libks_engine.so":
        return os.path.join(ROOT, "kubernetes-simulator_amd", "kubesim_amd", name)
    return os.path.join(DIAG, name)
