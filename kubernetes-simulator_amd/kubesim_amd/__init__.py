"""kubesim_amd — MI355X-native scheduling engine for kubesim (host side).

The product is the C-ABI library ``libks_engine.so`` (include/ks_engine.h) built from
``kubernetes-simulator_amd/csrc``; this package is its Python host binding plus the
placement-independent host ingest (trace generation, dictionary encoding).
"""
from . import tracegen, encode  # noqa: F401

__all__ = ["tracegen", "encode", "engine"]
