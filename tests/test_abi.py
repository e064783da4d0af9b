"""The C-ABI library loads on a GPU-less host and exports exactly what include/ks_engine.h
declares; configuration validation needs no device."""
import ctypes as C
import os
import re

from kubesim_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = ""
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if h.endswith(".h"):
            src += open(os.path.join(ROOT, "include", h)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"typedef[^;]*;", "", src)  # callback types are not entry points
    return sorted(set(re.findall(r"\b(ks_[a-z_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert _declared() == sorted(_lib.EXPORTED_SYMBOLS + _lib.RUN_SYMBOLS)


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    R = _lib.load_run()  # include/ks_kubesim.h: the C++ Run loop over the C-ABI
    for sym in _lib.EXPORTED_SYMBOLS:
        assert hasattr(L, sym), sym
    for sym in _lib.RUN_SYMBOLS:
        assert hasattr(R, sym), sym


def test_retired_resolver_flags_rejected_without_device():
    """Bits 16, 32 and 128 were the pair, sweep and sequential resolvers (removed in round 4)."""
    L = _lib.load()
    for bit in (16, 32, 128, 1024):
        cfg = _lib.KsConfig()
        cfg.abi_version = _lib.KS_ABI_VERSION
        cfg.tick_seconds = 10
        cfg.engine_flags = bit
        h = C.c_void_p()
        assert L.ks_create(C.byref(cfg), C.byref(h)) == _lib.KS_EINVAL


def test_bad_configs_rejected_without_device():
    L = _lib.load()
    def create(**kw):
        cfg = _lib.KsConfig()
        cfg.abi_version = _lib.KS_ABI_VERSION
        cfg.tick_seconds = 10
        cfg.n_scorers = 1
        cfg.scorers[0].kind, cfg.scorers[0].weight, cfg.scorers[0].value = 0, 1, 1
        for k, v in kw.items():
            setattr(cfg, k, v)
        h = C.c_void_p()
        return L.ks_create(C.byref(cfg), C.byref(h))
    assert create(abi_version=99) == _lib.KS_EINVAL
    assert create(tick_seconds=0) == _lib.KS_EINVAL
    assert create(filter_mode=7) == _lib.KS_EINVAL
    assert create(filters=8) == _lib.KS_EINVAL
    assert create(n_scorers=9) == _lib.KS_EINVAL
    assert create(batch_pods=100000) == _lib.KS_EINVAL


def test_engine_refuses_without_library(monkeypatch, tmp_path):
    import importlib
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    import pytest
    with pytest.raises(ImportError):
        _lib.load()
    importlib.reload(_lib)


def test_node_mix_matches_documented_formula():
    """ks_node_mix is a pure function (no device): the digest's node weight as the header
    spells it out."""
    from kubesim_amd import _lib
    from usage_digest import node_mix
    L = _lib.load()
    for nd in (0, 1, 2, 63, 50_000, (1 << 24) - 1):
        assert L.ks_node_mix(nd) == node_mix(nd)


def test_library_built_from_these_sources():
    """Provenance: both libraries carry the hash of the sources they were built
    from (csrc/Makefile HASHED), and it is the hash of the sources in this tree — _lib.load()
    refuses any other library, so a GPU record cannot come from a stale binary."""
    want = _lib.source_hash()
    assert want is not None and len(want) == 16
    assert _lib.load().ks_build_id().decode() == want
    assert _lib.load_run().ks_run_build_id().decode() == want
