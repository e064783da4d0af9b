"""ctypes binding of the C-ABI in include/ks_engine.h (libks_engine.so, built in-tree).

There is no fallback: if the HIP library is missing or fails to load, importing the engine
raises.  The CPU oracle under oracle/ is test infrastructure and is never used here.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libks_engine.so")
RUN_LIB_PATH = os.path.join(HERE, "libks_kubesim.so")

KS_OK, KS_EINVAL, KS_ENOTFOUND, KS_EDEVICE, KS_ENOMEM, KS_ERANGE = 0, 1, 2, 3, 4, 5
KS_FILTER_REFERENCE_LITERAL, KS_FILTER_FEEDS_SCORE = 0, 1
KS_FILTER_FIT, KS_FILTER_TAINT, KS_FILTER_SELECTOR = 1, 2, 4
KS_SCORER_CONST, KS_SCORER_LEAST_REQUESTED, KS_SCORER_BALANCED = 0, 1, 2
KS_POD_OK, KS_POD_OVER_CAPACITY = 0, 1
KS_PODFLAG_BAD_KEY, KS_PODFLAG_BAD_SPEC = 1, 2
KS_ABI_VERSION = 2
KS_ENGINE_FORCE_WIDE = 1
KS_ENGINE_NO_TINY = 2
KS_ENGINE_NO_MICRO = 4
KS_ENGINE_ONE_POD_RESOLVER = 8
KS_ENGINE_CHUNK_RESOLVER = 64
KS_ENGINE_NO_OVERLAP = 256
KS_ENGINE_PRUNED_LISTS = 512
KS_SELFTEST_LR_MICRO = 0

STATUS_NAMES = {KS_OK: "OK", KS_EINVAL: "InvalidArgument", KS_ENOTFOUND: "NotFound",
                KS_EDEVICE: "DeviceError", KS_ENOMEM: "OutOfMemory", KS_ERANGE: "OutOfDomain"}

# every symbol include/*.h declares
EXPORTED_SYMBOLS = ("ks_create", "ks_destroy", "ks_load_nodes", "ks_submit_pods", "ks_step",
                    "ks_filter", "ks_score", "ks_usage", "ks_current_tick", "ks_tick_seconds", "ks_queued_pods",
                    "ks_last_error", "ks_last_step_stats", "ks_last_step_kernels", "ks_set_profiling", "ks_debug_counters", "ks_debug_invariants", "ks_debug_window", "ks_debug_watch", "ks_build_id", "ks_selftest",
                    "ks_comm_unique_id", "ks_shard", "ks_shard_host", "ks_group_create", "ks_group_destroy",
                    "ks_group_add", "ks_group_size", "ks_group_step", "ks_pod_status",
                    "ks_usage_at", "ks_usage_digest", "ks_node_mix", "ks_pod_lookup", "ks_node_pods",
                    "ks_shard_layout", "ks_merge_candidates",
                    # include/ks_ingest.h
                    "ks_parse_quantity", "ks_parse_simspec", "ks_cluster_parse", "ks_cluster_free",
                    "ks_cluster_nodes", "ks_cluster_tick", "ks_cluster_start_clock", "ks_cluster_arrays",
                    "ks_cluster_node_name", "ks_cluster_tolerations", "ks_cluster_selector",
                    "ks_cluster_parse_ex", "ks_cluster_note_pod", "ks_cluster_seal")
KS_CLUSTER_DEFER_MASKS = 1
KS_COMM_ID_BYTES = 128
# include/ks_kubesim.h (libks_kubesim.so)
RUN_SYMBOLS = ("ks_run", "ks_trace_submit", "ks_local_exchange_create", "ks_local_exchange_destroy",
               "ks_local_allgather", "ks_local_exchange_abort", "ks_run_build_id")


class KsScorer(C.Structure):
    _fields_ = [("kind", C.c_int32), ("weight", C.c_int32), ("value", C.c_int32)]


class KsConfig(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("tick_seconds", C.c_int32), ("filter_mode", C.c_int32),
                ("filters", C.c_uint32), ("n_scorers", C.c_int32), ("scorers", KsScorer * 8),
                ("device", C.c_int32), ("batch_pods", C.c_int32), ("engine_flags", C.c_uint32),
                ("reserved", C.c_int32 * 7)]


class KsBind(C.Structure):
    _fields_ = [("pod", C.c_int64), ("node", C.c_int32), ("status", C.c_int32), ("tick", C.c_int64)]


class KsPodInfo(C.Structure):
    _fields_ = [("phase", C.c_int32), ("node", C.c_int32), ("start_tick", C.c_int64),
                ("total_seconds", C.c_int32), ("pad", C.c_int32)]


KS_PHASE_PENDING, KS_PHASE_RUNNING, KS_PHASE_SUCCEEDED, KS_PHASE_FAILED = 0, 1, 2, 3


class KsStepStats(C.Structure):
    _fields_ = [("step_ms", C.c_double), ("scan_ms", C.c_double), ("resolve_ms", C.c_double),
                ("launches", C.c_int64), ("pods", C.c_int64), ("other_ms", C.c_double)]


class KsKernelStats(C.Structure):
    _fields_ = [("prep_ms", C.c_double), ("scan_ms", C.c_double), ("merge_ms", C.c_double),
                ("resolve_ms", C.c_double), ("fused_ms", C.c_double), ("part_ms", C.c_double),
                ("xchg_ms", C.c_double), ("prep_n", C.c_int64), ("scan_n", C.c_int64), ("merge_n", C.c_int64),
                ("resolve_n", C.c_int64), ("fused_n", C.c_int64), ("xchg_n", C.c_int64),
                ("side_scan_ms", C.c_double), ("side_part_ms", C.c_double), ("side_xchg_ms", C.c_double),
                ("wait_ms", C.c_double), ("side_n", C.c_int64),
                ("usage_ms", C.c_double), ("usage_n", C.c_int64), ("usage_pods", C.c_int64)]


class KsPods(C.Structure):
    _fields_ = [("m", C.c_int64), ("arrival", C.c_void_p), ("req", C.c_void_p), ("keymask", C.c_void_p),
                ("tol", C.c_void_p), ("sel", C.c_void_p), ("phase_off", C.c_void_p), ("phase_sec", C.c_void_p),
                ("phase_use", C.c_void_p), ("flags", C.c_void_p), ("key_id", C.c_void_p)]


class KsTraceSubmitter(C.Structure):
    _fields_ = [("trace", KsPods), ("next", C.c_int64), ("tick_seconds", C.c_int64)]


_lib = None
_run_lib = None
CSRC = os.path.join(os.path.dirname(HERE), "csrc")


def source_hash():
    """The provenance hash the Makefile embeds (ks_build_id): SHA-256 of the files its HASHED list
    names, in that order, first 16 hex digits; None when the sources are not beside the package."""
    import hashlib
    mk = os.path.join(CSRC, "Makefile")
    if not os.path.exists(mk):
        return None
    with open(mk) as f:
        line = next((x for x in f if x.startswith("HASHED =")), None)
    if line is None:
        return None
    h = hashlib.sha256()
    for name in line.split("=", 1)[1].split():
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _check_build(path, got):
    want = source_hash()
    got = got.decode() if got else ""
    if want is not None and got != want:
        raise ImportError(f"{path} was built from other sources (build id {got!r}, sources {want!r}): "
                          "run __graft_entry__.build()")


def load_run():
    """Load libks_kubesim.so (KubeSim.Run in C++ over the C-ABI, include/ks_kubesim.h)."""
    global _run_lib
    if _run_lib is not None:
        return _run_lib
    load()
    if not os.path.exists(RUN_LIB_PATH):
        raise ImportError(f"{RUN_LIB_PATH} is missing: run __graft_entry__.build()")
    L = C.CDLL(RUN_LIB_PATH)
    L.ks_run_build_id.restype = C.c_char_p
    _check_build(RUN_LIB_PATH, L.ks_run_build_id())
    p = C.c_void_p
    L.ks_run.argtypes = [p, C.c_int64, C.c_int64, C.c_int32, p, p, p, C.c_int64, C.POINTER(C.c_int64),
                         C.POINTER(C.c_double)]
    L.ks_run.restype = C.c_int
    L.ks_trace_submit.argtypes = [p, C.c_int64, C.c_int64, p]
    L.ks_trace_submit.restype = C.c_int
    L.ks_local_exchange_create.argtypes = [C.c_int32]
    L.ks_local_exchange_create.restype = p
    L.ks_local_exchange_destroy.argtypes = [p]
    L.ks_local_exchange_destroy.restype = None
    L.ks_local_allgather.argtypes = [p, C.c_int32, C.c_int32, p, C.c_int64]
    L.ks_local_allgather.restype = C.c_int
    L.ks_local_exchange_abort.argtypes = [p]
    L.ks_local_exchange_abort.restype = None
    _run_lib = L
    return L


def load():
    """Load libks_engine.so (fails loudly if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc, gfx950)")
    L = C.CDLL(LIB_PATH)
    L.ks_build_id.restype = C.c_char_p
    _check_build(LIB_PATH, L.ks_build_id())
    p = C.c_void_p
    L.ks_create.argtypes = [C.POINTER(KsConfig), C.POINTER(C.c_void_p)]
    L.ks_create.restype = C.c_int
    L.ks_destroy.argtypes = [p]
    L.ks_destroy.restype = None
    L.ks_load_nodes.argtypes = [p, C.c_int64, p, p, p]
    L.ks_submit_pods.argtypes = [p, C.c_int64] + [p] * 10
    L.ks_step.argtypes = [p, C.c_int64, p, C.c_int64, C.POINTER(C.c_int64)]
    L.ks_filter.argtypes = [p, C.c_int64, p]
    L.ks_score.argtypes = [p, C.c_int64, p]
    L.ks_usage.argtypes = [p, p]
    L.ks_usage_at.argtypes = [p, C.c_int64, p]
    L.ks_usage_digest.argtypes = [p, C.c_int64, C.c_int64, p]
    L.ks_node_mix.argtypes = [C.c_int64]
    L.ks_node_mix.restype = C.c_uint64
    L.ks_pod_lookup.argtypes = [p, C.c_int32, C.c_int64, C.POINTER(C.c_int64)]
    L.ks_node_pods.argtypes = [p, C.c_int32, p, C.c_int64, C.POINTER(C.c_int64)]
    L.ks_shard_layout.argtypes = [C.c_int64, C.c_int32, C.c_int32, p]
    L.ks_shard_layout.restype = C.c_int
    L.ks_merge_candidates.argtypes = [p, C.c_int32, C.c_int32, p]
    L.ks_merge_candidates.restype = C.c_int
    for f in ("ks_load_nodes", "ks_submit_pods", "ks_step", "ks_filter", "ks_score", "ks_usage", "ks_usage_at",
              "ks_usage_digest", "ks_pod_lookup", "ks_node_pods"):
        getattr(L, f).restype = C.c_int
    L.ks_current_tick.argtypes = [p]
    L.ks_current_tick.restype = C.c_int64
    L.ks_tick_seconds.argtypes = [p]
    L.ks_tick_seconds.restype = C.c_int32
    L.ks_queued_pods.argtypes = [p]
    L.ks_queued_pods.restype = C.c_int64
    L.ks_last_error.argtypes = [p]
    L.ks_last_error.restype = C.c_char_p
    L.ks_last_step_stats.argtypes = [p, C.POINTER(KsStepStats)]
    L.ks_last_step_stats.restype = C.c_int
    L.ks_last_step_kernels.argtypes = [p, C.POINTER(KsKernelStats)]
    L.ks_last_step_kernels.restype = C.c_int
    L.ks_debug_counters.argtypes = [p, p]
    L.ks_debug_counters.restype = C.c_int
    L.ks_debug_invariants.argtypes = [p, p]
    L.ks_debug_invariants.restype = C.c_int
    L.ks_debug_window.argtypes = [p, p, C.c_int64, C.POINTER(C.c_int64)]
    L.ks_debug_window.restype = C.c_int
    L.ks_debug_watch.argtypes = [p, C.c_int64]
    L.ks_debug_watch.restype = C.c_int
    L.ks_set_profiling.argtypes = [p, C.c_int]
    L.ks_set_profiling.restype = None
    L.ks_selftest.argtypes = [C.c_int32, C.c_int32, p]
    L.ks_selftest.restype = C.c_int
    L.ks_comm_unique_id.argtypes = [p]
    L.ks_comm_unique_id.restype = C.c_int
    L.ks_shard.argtypes = [p, C.c_int32, C.c_int32, p, C.c_int32]
    L.ks_shard.restype = C.c_int
    L.ks_shard_host.argtypes = [p, C.c_int32, C.c_int32, C.c_int32, p, p]
    L.ks_shard_host.restype = C.c_int
    L.ks_group_create.argtypes = [C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]
    L.ks_group_create.restype = C.c_int
    L.ks_group_destroy.argtypes = [p]
    L.ks_group_destroy.restype = None
    L.ks_group_add.argtypes = [p, C.POINTER(KsConfig), C.POINTER(C.c_void_p)]
    L.ks_group_add.restype = C.c_int
    L.ks_group_size.argtypes = [p]
    L.ks_group_size.restype = C.c_int32
    L.ks_group_step.argtypes = [p, C.c_int64, p, C.c_int64, p, p, C.POINTER(KsStepStats)]
    L.ks_group_step.restype = C.c_int
    L.ks_pod_status.argtypes = [p, C.c_int64, C.c_int64, p]
    L.ks_pod_status.restype = C.c_int
    # ingest (include/ks_ingest.h)
    L.ks_parse_quantity.argtypes = [C.c_char_p, C.POINTER(C.c_int64)]
    L.ks_parse_quantity.restype = C.c_int
    L.ks_parse_simspec.argtypes = [C.c_char_p, C.c_int32, C.POINTER(C.c_int32), p, p, p, C.c_char_p, C.c_int32]
    L.ks_parse_simspec.restype = C.c_int
    L.ks_cluster_parse.argtypes = [C.c_char_p, C.POINTER(C.c_void_p), C.c_char_p, C.c_int32]
    L.ks_cluster_parse.restype = C.c_int
    L.ks_cluster_free.argtypes = [p]
    L.ks_cluster_free.restype = None
    L.ks_cluster_nodes.argtypes = [p]
    L.ks_cluster_nodes.restype = C.c_int64
    L.ks_cluster_tick.argtypes = [p]
    L.ks_cluster_tick.restype = C.c_int32
    L.ks_cluster_start_clock.argtypes = [p]
    L.ks_cluster_start_clock.restype = C.c_char_p
    L.ks_cluster_arrays.argtypes = [p, p, p, p]
    L.ks_cluster_arrays.restype = C.c_int
    L.ks_cluster_node_name.argtypes = [p, C.c_int64]
    L.ks_cluster_node_name.restype = C.c_char_p
    L.ks_cluster_tolerations.argtypes = [p, C.c_int32, p, p, p, p, C.POINTER(C.c_uint64)]
    L.ks_cluster_tolerations.restype = C.c_int
    L.ks_cluster_selector.argtypes = [p, C.c_int32, p, p, C.POINTER(C.c_uint64)]
    L.ks_cluster_selector.restype = C.c_int
    L.ks_cluster_parse_ex.argtypes = [C.c_char_p, C.c_int32, C.POINTER(C.c_void_p), C.c_char_p, C.c_int32]
    L.ks_cluster_parse_ex.restype = C.c_int
    L.ks_cluster_note_pod.argtypes = [p, C.c_int32, p, p, p, p, C.c_int32, p, p]
    L.ks_cluster_note_pod.restype = C.c_int
    L.ks_cluster_seal.argtypes = [p, C.c_char_p, C.c_int32]
    L.ks_cluster_seal.restype = C.c_int
    _lib = L
    return L
