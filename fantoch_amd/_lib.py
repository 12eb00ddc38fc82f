"""ctypes binding of the C-ABI in include/fantoch_amd.h.

The product is the in-tree `libfantoch_amd.so` (HIP kernels for gfx950 + the
C++ host side).  Every compute entry point runs on the GPU; there is no CPU
fallback — without the library, or without a GPU, calls raise.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# FX_LIB selects another build of the same library (tools: the FX_SIM_PROFILE build)
LIB_PATH = os.environ.get("FX_LIB") or os.path.join(HERE, "libfantoch_amd.so")

# status codes (fantoch_amd.h)
FX_OK = 0
FX_ERR_INVALID_ARG = 1
FX_ERR_CAPACITY = 2
FX_ERR_DOUBLE_INDEX = 3
FX_ERR_DEPS_UNSORTED = 4
FX_ERR_DOT_RANGE = 5
FX_ERR_HIP = 6
FX_ERR_UNSUPPORTED = 7
FX_ERR_ORDER_OVERFLOW = 8
FX_ERR_TIME_RANGE = 9
FX_ERR_NO_DEVICE = 10
FX_ERR_LOG_FORMAT = 11
FX_ERR_SIM_CAPACITY = 12
FX_ERR_SIM_LATE = 13
FX_ERR_SIM_EVENTS = 14
FX_ERR_TIMEOUT = 15
FX_PROTOCOL_ATLAS = 0
FX_PROTOCOL_EPAXOS = 1
FX_PROTOCOL_BASIC = 2
FX_SIM_FLAG_EXEC_NOTIFICATIONS = 1
FX_SIM_FLAG_LARGE = 2
FX_SIM_FLAG_GENERIC = 4
FX_SIM_FLAG_ARENA_FILL = 8
FX_SIM_STAT_FAST, FX_SIM_STAT_SLOW, FX_SIM_STAT_STABLE = 0, 8, 16
FX_SIM_STAT_EVENTS, FX_SIM_STAT_END_MS, FX_SIM_STAT_TRACE, FX_SIM_STAT_SEQ = 24, 25, 26, 27
FX_SIM_STAT_DEPS = 28
FX_SIM_STAT_LAT_SUM = 29
FX_SIM_STAT_ERR_SITE = 30
FX_SIM_STAT_FAST_READS, FX_SIM_STAT_SLOW_READS = 32, 40
FX_SIM_STATS = 48

FX_SEQ_BITS = 24
FX_SEQ_MASK = (1 << 24) - 1
FX_KIND_ADD = 0
FX_KIND_INDEX_ONLY = 1
FX_KIND_EXECUTED = 2
FX_ORDER_SCC_START = 0x80000000
FX_RELEASE_NONE = 0xFFFFFFFF
FX_FLAG_INIT = 1
FX_FLAG_EXECUTE_AT_COMMIT = 2
FX_FLAG_SAVE_STATE = 4
FX_TIER_WIDE, FX_TIER_WIDE_HBM = 7, 8
FX_NUM_TIERS = 9
FX_PRED_TIER_SMALL, FX_PRED_TIER_LDS, FX_PRED_TIER_HBM = 0, 1, 2
FX_PROFILE_SLOT_PRED = 16
FX_TIER_GROUP = 0
FX_TIER_WAVE = 4
FX_TIER_LANE_REG = 5
FX_TIER_SPLIT = 6
FX_TIER_DEFAULT = FX_TIER_SPLIT
FX_FLAG_TIER_SHIFT = 8


def first_tier_flag(t):
    return (t + 1) << FX_FLAG_TIER_SHIFT


class FxError(RuntimeError):
    def __init__(self, status, what=""):
        self.status = status
        super().__init__("%s: fantoch_amd status %d (%s)" % (what, status, status_string(status)))


u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)


class StreamBatch(ctypes.Structure):
    _fields_ = [("dot", ctypes.c_void_p), ("hdr", ctypes.c_void_p), ("deps", ctypes.c_void_p),
                ("lengths", ctypes.c_void_p), ("num_streams", ctypes.c_uint32),
                ("steps", ctypes.c_uint32), ("dmax", ctypes.c_uint32), ("n", ctypes.c_uint32)]


class OrderBatch(ctypes.Structure):
    _fields_ = [("order", ctypes.c_void_p), ("release", ctypes.c_void_p),
                ("nexec", ctypes.c_void_p), ("err", ctypes.c_void_p)]


class PredBatch(ctypes.Structure):
    """fx_pred_batch (predecessors executor input)."""
    _fields_ = [("base", StreamBatch), ("clock_lo", ctypes.c_void_p), ("clock_hi", ctypes.c_void_p),
                ("ndeps", ctypes.c_void_p)]


class CutStats(ctypes.Structure):
    """fx_cut_stats (fx_batch_run_cut)."""
    _fields_ = [("segments", ctypes.c_uint64), ("max_segment", ctypes.c_uint32),
                ("whole_streams", ctypes.c_uint32), ("failed_streams", ctypes.c_uint32),
                ("tier_counts", ctypes.c_uint32 * 16), ("single_segments", ctypes.c_uint64)]


class HistBatch(ctypes.Structure):
    _fields_ = [("chain_size", ctypes.c_void_p), ("nbins_chain", ctypes.c_uint32),
                ("execution_delay", ctypes.c_void_p), ("nbins_delay", ctypes.c_uint32)]


class TierInfo(ctypes.Structure):
    _fields_ = [("max_sources", ctypes.c_uint32), ("pending_cap", ctypes.c_uint32),
                ("window_bits", ctypes.c_uint32), ("state_words", ctypes.c_uint32)]


class SynthParams(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("instances", ctypes.c_uint32),
                ("instance_base", ctypes.c_uint32), ("n", ctypes.c_uint32),
                ("cmds_per_process", ctypes.c_uint32), ("window", ctypes.c_uint32),
                ("cycle_pct", ctypes.c_uint32), ("horizon", ctypes.c_uint32),
                ("num_conflicts", ctypes.c_uint32), ("conflict_pct", ctypes.c_uint32 * 8),
                ("conflict_block", ctypes.c_uint32), ("clients", ctypes.c_uint32),
                ("key_pool", ctypes.c_uint32)]


class Config(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("f", ctypes.c_uint32), ("shard_count", ctypes.c_uint32),
                ("execute_at_commit", ctypes.c_uint32),
                ("executor_monitor_execution_order", ctypes.c_uint32)]


class CDot(ctypes.Structure):
    _fields_ = [("source", ctypes.c_uint32), ("seq", ctypes.c_uint32)]


class CRifl(ctypes.Structure):
    _fields_ = [("source", ctypes.c_uint64), ("seq", ctypes.c_uint64)]


class ExecutorResultC(ctypes.Structure):
    _fields_ = [("rifl", CRifl), ("key", ctypes.c_uint32), ("read_only", ctypes.c_uint32)]


class RequestReplyC(ctypes.Structure):
    _fields_ = [("to_shard", ctypes.c_uint64), ("kind", ctypes.c_uint32), ("dot", CDot), ("rifl", CRifl),
                ("ndeps", ctypes.c_uint32), ("first_dep", ctypes.c_uint32), ("cmd_shards", ctypes.c_uint64)]


class LogSummary(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in
                ("records", "adds", "others", "keys", "deps", "distinct_keys")]


class LogAdd(ctypes.Structure):
    _fields_ = [("dot", CDot), ("rifl", CRifl), ("key_off", ctypes.c_uint64),
                ("dep_off", ctypes.c_uint64), ("nkeys", ctypes.c_uint32),
                ("ndeps", ctypes.c_uint32), ("read_only", ctypes.c_uint32),
                ("pad", ctypes.c_uint32)]


class HistStats(ctypes.Structure):
    _fields_ = [("count", ctypes.c_double), ("mean", ctypes.c_double), ("stddev", ctypes.c_double),
                ("cov", ctypes.c_double), ("mdtm", ctypes.c_double), ("min", ctypes.c_double),
                ("max", ctypes.c_double)]


class SimSpec(ctypes.Structure):
    """fx_sim_spec: one simulated instance (Runner::new + Runner::run)."""
    _fields_ = [("seed", ctypes.c_uint64), ("instance", ctypes.c_uint64),
                ("protocol", ctypes.c_uint32), ("n", ctypes.c_uint32), ("f", ctypes.c_uint32),
                ("gc_interval_ms", ctypes.c_uint32), ("executed_notification_ms", ctypes.c_uint32),
                ("clients_per_region", ctypes.c_uint32), ("commands_per_client", ctypes.c_uint32),
                ("keys_per_command", ctypes.c_uint32), ("conflict_rate", ctypes.c_uint32),
                ("pool_size", ctypes.c_uint32), ("read_only_pct", ctypes.c_uint32),
                ("extra_sim_time_ms", ctypes.c_int32), ("reorder_messages", ctypes.c_uint32),
                ("nfr", ctypes.c_uint32), ("num_client_regions", ctypes.c_uint32),
                ("process_regions", ctypes.c_uint8 * 8), ("client_regions", ctypes.c_uint8 * 20)]


class SimBatch(ctypes.Structure):
    _fields_ = [("specs", ctypes.c_void_p), ("host_specs", ctypes.c_void_p),
                ("instances", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("planet_ping", ctypes.c_void_p), ("planet_rank", ctypes.c_void_p),
                ("planet_regions", ctypes.c_uint32), ("planet_stride", ctypes.c_uint32),
                ("exec_cap", ctypes.c_uint32), ("lat_cap", ctypes.c_uint32),
                ("max_events", ctypes.c_uint32), ("ring_entries", ctypes.c_uint32),
                ("dot_slots", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


class SimOutput(ctypes.Structure):
    _fields_ = [("executed", ctypes.c_void_p), ("executed_len", ctypes.c_void_p),
                ("latency_log", ctypes.c_void_p), ("latency_hist", ctypes.c_void_p),
                ("chain_hist", ctypes.c_void_p), ("delay_hist", ctypes.c_void_p),
                ("stats", ctypes.c_void_p), ("err", ctypes.c_void_p),
                ("lat_bins", ctypes.c_uint32), ("chain_bins", ctypes.c_uint32),
                ("delay_bins", ctypes.c_uint32), ("pad", ctypes.c_uint32),
                ("dot_client", ctypes.c_void_p)]


# (name, restype, argtypes) of every symbol declared in include/fantoch_amd.h
SIGNATURES = [
    ("fx_tier_query", ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(TierInfo)]),
    ("fx_batch_state_bytes", ctypes.c_size_t, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    ("fx_batch_execute", ctypes.c_int,
     [ctypes.POINTER(StreamBatch), ctypes.POINTER(OrderBatch), ctypes.c_uint32, ctypes.c_void_p,
      ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.c_void_p, ctypes.c_void_p]),
    ("fx_batch_metrics", ctypes.c_int,
     [ctypes.POINTER(StreamBatch), ctypes.POINTER(OrderBatch), ctypes.POINTER(HistBatch),
      ctypes.c_void_p]),
    ("fx_batch_run_tiered", ctypes.c_int,
     [ctypes.POINTER(StreamBatch), ctypes.POINTER(OrderBatch), ctypes.c_uint32, ctypes.c_void_p,
      u32p]),
    ("fx_pred_execute", ctypes.c_int,
     [ctypes.POINTER(PredBatch), ctypes.POINTER(OrderBatch), ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
    ("fx_pred_state_bytes", ctypes.c_size_t, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    ("fx_pred_run", ctypes.c_int,
     [ctypes.POINTER(PredBatch), ctypes.POINTER(OrderBatch), ctypes.c_uint32, ctypes.c_void_p, u32p]),
    ("fx_partial_state_bytes", ctypes.c_size_t, [ctypes.c_uint32, ctypes.c_uint32]),
    ("fx_batch_execute_partial", ctypes.c_int,
     [ctypes.POINTER(StreamBatch), ctypes.POINTER(OrderBatch), ctypes.c_void_p, ctypes.c_uint32,
      ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
    ("fx_batch_run_cut", ctypes.c_int,
     [ctypes.POINTER(StreamBatch), ctypes.POINTER(OrderBatch), ctypes.c_uint32, ctypes.c_void_p,
      ctypes.c_void_p]),
    ("fx_synth_shape", ctypes.c_int, [ctypes.POINTER(SynthParams), u32p, u32p, u32p]),
    ("fx_synth_generate", ctypes.c_int,
     [ctypes.POINTER(SynthParams), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_void_p]),
    ("fx_synth_generate_host", ctypes.c_int,
     [ctypes.POINTER(SynthParams), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("fx_graph_executor_new", ctypes.c_void_p,
     [ctypes.c_uint8, ctypes.c_uint64, ctypes.POINTER(Config)]),
    ("fx_graph_executor_free", None, [ctypes.c_void_p]),
    ("fx_graph_executor_set_executor_index", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    ("fx_graph_executor_handle_add", ctypes.c_int,
     [ctypes.c_void_p, CDot, CRifl, u32p, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.POINTER(CDot), ctypes.c_uint32, ctypes.c_uint64]),
    ("fx_graph_executor_index_only", ctypes.c_int,
     [ctypes.c_void_p, CDot, CRifl, u32p, ctypes.c_uint32, ctypes.POINTER(CDot),
      ctypes.c_uint32, ctypes.c_uint64]),
    ("fx_graph_executor_set_executed_frontier", ctypes.c_int,
     [ctypes.c_void_p, u64p, ctypes.c_uint32]),
    ("fx_graph_executor_to_clients", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(ExecutorResultC), ctypes.c_uint32, u32p]),
    ("fx_graph_executor_drain_dots", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(CDot), ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint32,
      u32p]),
    ("fx_graph_executor_metrics", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, u64p, u64p, ctypes.c_uint32, u32p]),
    ("fx_graph_executor_monitor", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(CRifl), ctypes.c_uint32, u32p]),
    ("fx_graph_executor_pending", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(CDot), ctypes.POINTER(CDot), ctypes.c_uint32, u32p]),
    ("fx_graph_executor_handle_add_sharded", ctypes.c_int,
     [ctypes.c_void_p, CDot, CRifl, u32p, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.POINTER(CDot), u32p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64]),
    ("fx_graph_executor_handle_executed", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(CDot), ctypes.c_uint32, ctypes.c_uint64]),
    ("fx_graph_executor_requests", ctypes.c_int,
     [ctypes.c_void_p, u64p, ctypes.POINTER(CDot), ctypes.c_uint32, u32p]),
    ("fx_graph_executor_to_executors", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(CDot), ctypes.c_uint32, u32p]),
    ("fx_graph_executor_clone", ctypes.c_void_p, [ctypes.c_void_p]),
    ("fx_graph_executor_handle_executed_info", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(CDot), ctypes.c_uint32]),
    ("fx_graph_executor_handle_request", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(CDot), ctypes.c_uint32]),
    ("fx_graph_executor_cleanup", ctypes.c_int, [ctypes.c_void_p]),
    ("fx_graph_executor_request_replies", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(RequestReplyC), ctypes.c_uint32, ctypes.POINTER(CDot), u32p,
      ctypes.c_uint32, u32p]),
    ("fx_graph_executor_parallel", ctypes.c_int, []),
    ("fx_graph_executor_transfer_stats", ctypes.c_int, [ctypes.c_void_p, u64p, u64p]),
    ("fx_graph_executor_persist_stats", ctypes.c_int, [ctypes.c_void_p, u64p, ctypes.c_uint32]),
    ("fx_graph_executor_debug_hooks", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]),
    ("fx_sim_plan", ctypes.c_int,
     [ctypes.POINTER(SimSpec), ctypes.c_uint32, ctypes.c_uint32, u32p]),
    ("fx_sim_plan_large", ctypes.c_int,
     [ctypes.POINTER(SimSpec), ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]),
    ("fx_sim_run", ctypes.c_int,
     [ctypes.POINTER(SimBatch), ctypes.POINTER(SimOutput), ctypes.c_void_p]),
    ("fx_sim_run_tiered", ctypes.c_int,
     [ctypes.POINTER(SimBatch), ctypes.POINTER(SimOutput), ctypes.c_void_p, u32p]),
    ("fx_planet_load", ctypes.c_int,
     [ctypes.c_char_p, ctypes.c_uint32, u32p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p,
      ctypes.c_void_p]),
    ("fx_quorum_sizes", ctypes.c_int,
     [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p]),
    ("fx_exec_log_scan", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(LogSummary)]),
    ("fx_exec_log_decode", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(LogAdd), ctypes.c_uint64,
      u32p, ctypes.c_uint64, ctypes.POINTER(CDot), ctypes.c_uint64, ctypes.POINTER(LogSummary)]),
    ("fx_hist_stats_compute", ctypes.c_int,
     [u64p, u64p, ctypes.c_uint32, ctypes.POINTER(HistStats)]),
    ("fx_hist_percentile", ctypes.c_int,
     [u64p, u64p, ctypes.c_uint32, ctypes.c_double, ctypes.POINTER(ctypes.c_double)]),
    ("fx_device_count", ctypes.c_int, []),
    ("fx_dev_alloc", ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]),
    ("fx_dev_free", ctypes.c_int, [ctypes.c_void_p]),
    ("fx_dev_memset", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]),
    ("fx_dev_h2d", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    ("fx_dev_d2h", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    ("fx_dev_synchronize", ctypes.c_int, [ctypes.c_void_p]),
    ("fx_profile_enable", ctypes.c_int, [ctypes.c_int]),
    ("fx_profile_last_exec_ms", ctypes.c_int, [ctypes.POINTER(ctypes.c_float)]),
    ("fx_profile_last_kernel_ms", ctypes.c_int, [ctypes.c_uint32, ctypes.POINTER(ctypes.c_float)]),
    ("fx_profile_slot_ms", ctypes.c_int, [ctypes.c_uint32, ctypes.POINTER(ctypes.c_float)]),
    ("fx_status_string", ctypes.c_char_p, [ctypes.c_int]),
    ("fx_version", ctypes.c_char_p, []),
]

_lib = None


def load():
    """Loads libfantoch_amd.so (raises if it was not built: no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(
                "%s is missing: build it with `make` (or __graft_entry__.build())" % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def status_string(status):
    try:
        return load().fx_status_string(status).decode()
    except Exception:  # pragma: no cover - used while formatting errors only
        return "?"


def check(status, what="fantoch_amd"):
    if status != FX_OK:
        raise FxError(status, what)
    return status


def plane_words(num_streams, steps):
    return ((num_streams + 63) // 64) * 64 * ((steps + 3) // 4) * 4


def index(step, stream, steps):
    """fx_index: tiled plane position of (step, stream); numpy-vectorised."""
    step = np.asarray(step, dtype=np.int64)
    stream = np.asarray(stream, dtype=np.int64)
    steps4 = (steps + 3) // 4
    return ((stream >> 6) * steps4 + (step >> 2)) * 256 + ((stream & 63) << 2) + (step & 3)


def pack_dot(src, seq):
    return (int(src) << FX_SEQ_BITS) | (int(seq) & FX_SEQ_MASK)


def unpack_dot(d):
    return (int(d) >> FX_SEQ_BITS, int(d) & FX_SEQ_MASK)


def make_hdr(t, nd, kind=FX_KIND_ADD):
    return (int(t) & 0xFFFFFF) | ((int(nd) & 31) << 24) | ((int(kind) & 7) << 29)


def quorum_sizes(protocol, n, f=0):
    """(fast, write) quorum sizes (fantoch/src/config.rs:294-312) via fx_quorum_sizes."""
    fq, wq = ctypes.c_uint32(), ctypes.c_uint32()
    check(load().fx_quorum_sizes(protocol, n, f, ctypes.byref(fq), ctypes.byref(wq)),
          "fx_quorum_sizes")
    return fq.value, wq.value
