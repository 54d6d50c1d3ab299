"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the C restatement (oracle).

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
import this module.  It never backs the product: ``sentinel_amd`` has no
import path to it.

The wrapper exposes (1) the object-level API used by the known-answer tests
transcribed from the reference's JUnit suites and (2) ``OracleEngine``, the
single-threaded replay with the same call shapes as the HIP engine.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from sentinel_amd import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libsentinel_oracle.so")


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH) or \
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "sentinel_oracle.c")):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        _declare(_lib)
    return _lib


P = C.c_void_p
I32, I64, U32, U8, U64, D = C.c_int32, C.c_int64, C.c_uint32, C.c_uint8, C.c_uint64, C.c_double


def _declare(L):
    def f(name, res, *args):
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = list(args)
    f("so_set_time", None, I64)
    f("so_now", I64)
    f("so_set_statistic_max_rt", None, I64)
    f("so_java_round", I64, D)
    f("so_java_next_up", D, D)
    f("so_java_d2i", I32, D)
    f("so_java_d2l", I64, D)
    f("so_la_new", P, C.c_int, C.c_int, C.c_int)
    f("so_la_free", None, P)
    for n in ("so_la_current_window", "so_la_previous_window", "so_la_valid_head", "so_la_window_value"):
        f(n, P, P, I64)
    f("so_la_current_window_now", P, P)
    f("so_la_values", C.c_int, P, I64, C.POINTER(P), C.c_int)
    f("so_la_list_now", C.c_int, P, C.POINTER(P), C.c_int)
    f("so_la_current_waiting", I64, P)
    f("so_la_add_waiting", None, P, I64, I32)
    f("so_wrap_start", I64, P)
    f("so_wrap_length", I64, P)
    f("so_wrap_get", I64, P, C.c_int)
    f("so_wrap_add", None, P, C.c_int, I64)
    f("so_wrap_min_rt", I64, P)
    f("so_wrap_add_rt", None, P, I64)
    f("so_am_new", P, C.c_int, C.c_int, C.c_int)
    f("so_am_free", None, P)
    for n in ("pass", "block", "success", "exception", "rt", "min_rt", "max_success", "occupied_pass",
              "previous_window_pass", "previous_window_block", "waiting"):
        f("so_am_" + n, I64, P)
    f("so_am_window_pass", I64, P, I64)
    f("so_am_add", None, P, C.c_int, I32)
    f("so_am_add_rt", None, P, I64)
    f("so_am_add_waiting", None, P, I64, I32)
    f("so_am_details", C.c_int, P, C.c_int, I64, C.POINTER(abi.sf_metric_row), C.c_int)
    f("so_node_new", P)
    f("so_node_free", None, P)
    for n in ("pass_qps", "block_qps", "previous_pass_qps", "avg_rt", "min_rt", "success_qps", "max_success_qps"):
        f("so_node_" + n, D, P)
    f("so_node_cur_thread_num", I32, P)
    f("so_node_add_pass_request", None, P, I32)
    f("so_node_increase_block_qps", None, P, I32)
    f("so_node_add_rt_and_success", None, P, I64, I32)
    f("so_node_increase_exception_qps", None, P, I32)
    f("so_node_increase_thread_num", None, P)
    f("so_node_decrease_thread_num", None, P)
    f("so_node_try_occupy_next", I64, P, I64, I32, D)
    f("so_node_waiting", I64, P)
    f("so_node_add_waiting_request", None, P, I64, I32)
    f("so_node_add_occupied_pass", None, P, I32)
    f("so_node_read", None, P, C.POINTER(abi.sf_node_state))
    f("so_ctrl_default", P, D, C.c_int)
    f("so_ctrl_warm_up", P, D, C.c_int, C.c_int)
    f("so_ctrl_rate_limiter", P, C.c_int, D)
    f("so_ctrl_warm_up_rate_limiter", P, D, C.c_int, C.c_int, C.c_int)
    f("so_ctrl_free", None, P)
    f("so_ctrl_can_pass", C.c_int, P, P, C.POINTER(MockNode), I32, C.c_int, C.POINTER(I64), C.POINTER(C.c_int))
    f("so_ctrl_state", None, P, C.POINTER(abi.sf_rule_state))
    f("so_ctrl_warning_token", I32, P)
    f("so_ctrl_max_token", I32, P)
    f("so_ctrl_slope", D, P)
    f("so_pm_new", P)
    f("so_pm_new_mode", P, C.c_int)
    f("so_pm_evictions", U64, P)
    f("so_set_param_lru", C.c_int, P, C.c_int)
    f("so_param_lru_stats", C.c_int, P, C.POINTER(U64), C.POINTER(U64))
    f("so_pm_free", None, P)
    f("so_param_pass_single", C.c_int, P, C.c_int, C.POINTER(abi.sf_param_rule), C.POINTER(abi.sf_hot_item),
      I32, U8, U64, C.POINTER(I64))
    f("so_pm_initialize", None, P, C.c_int, C.POINTER(abi.sf_param_rule))
    f("so_pm_add_thread", None, P, C.c_int, U8, U64)
    f("so_pm_dec_thread", None, P, C.c_int, U8, U64)
    f("so_pm_thread_count", I64, P, C.c_int, U8, U64)
    f("so_pm_read", C.c_int, P, C.c_int, U8, U64, C.POINTER(I64), C.POINTER(I64), C.POINTER(C.c_int))
    f("so_cm_new", P, C.c_int, C.c_int)
    f("so_cm_free", None, P)
    f("so_cm_add", None, P, C.c_int, I64)
    f("so_cm_sum", I64, P, C.c_int)
    f("so_cm_avg", D, P, C.c_int)
    f("so_cm_try_occupy_next", I32, P, C.c_int, I32, D)
    f("so_cpm_new", P, C.c_int, C.c_int)
    f("so_cpm_free", None, P)
    f("so_cpm_add_value", None, P, U8, U64, I32)
    f("so_cpm_sum", I64, P, U8, U64)
    f("so_cpm_avg", D, P, U8, U64)
    f("so_rl_new", P, D)
    f("so_rl_free", None, P)
    f("so_rl_try_pass", C.c_int, P)
    f("so_rl_sum", I64, P)
    f("so_rl_can_pass", C.c_int, P)
    f("so_rl_add", None, P, I32)
    f("so_param_rule_idx", I32, P, U32)
    f("so_create", P, C.POINTER(abi.sf_config))
    f("so_destroy", None, P)
    f("so_load_flow_rules", C.c_int, P, C.POINTER(abi.sf_flow_rule), U32)
    f("so_load_param_rules", C.c_int, P, C.POINTER(abi.sf_param_rule), U32, C.POINTER(abi.sf_hot_item), U32)
    f("so_load_system_rules", C.c_int, P, C.POINTER(abi.sf_system_rule), U32)
    f("so_set_system_status", C.c_int, P, D, D)
    f("so_submit", C.c_int, P, C.POINTER(abi.sf_event_batch), C.POINTER(abi.sf_verdicts))
    f("so_read_node", C.c_int, P, U32, C.POINTER(abi.sf_node_state))
    f("so_read_origin_node", C.c_int, P, U32, U32, C.POINTER(abi.sf_node_state))
    f("so_read_context_node", C.c_int, P, U32, U32, C.POINTER(abi.sf_node_state))
    f("so_select_node", C.c_int, P, U32, U32, U32)
    f("so_read_entry_node", C.c_int, P, C.POINTER(abi.sf_node_state))
    f("so_system_plan", C.c_int, P, C.POINTER(abi.sf_event_batch), P, U32, C.POINTER(U32), P)
    f("so_submit_forced", C.c_int, P, C.POINTER(abi.sf_event_batch), C.POINTER(abi.sf_verdicts), P)
    f("so_entry_node_add", C.c_int, P, C.POINTER(abi.sf_event_batch), P)
    f("so_load_degrade_rules", C.c_int, P, C.POINTER(abi.sf_degrade_rule), U32, C.POINTER(U32))
    f("so_read_breaker", C.c_int, P, U32, C.POINTER(abi.sf_breaker_state))
    f("so_read_rule_state", C.c_int, P, U32, C.POINTER(abi.sf_rule_state))
    f("so_node_digest", U64, C.POINTER(abi.sf_node_state), C.c_int)
    f("so_node_digests", C.c_int, P, P, U32)
    f("so_read_rule_states", C.c_int, P, U32, U32, P)
    f("so_read_param", C.c_int, P, U32, U8, U64, C.POINTER(I64), C.POINTER(I64), C.POINTER(C.c_int))
    f("so_param_thread", I64, P, U32, C.c_int, U8, U64)
    f("so_snapshot", C.c_int, P, I64, C.POINTER(abi.sf_metric_row), U32, C.POINTER(U32))
    f("so_format_fat", C.c_int, C.POINTER(SoNames), C.POINTER(abi.sf_metric_row), U32, I64, C.c_char_p, U64,
      C.POINTER(U64))
    f("so_metric_log", C.c_int, P, C.POINTER(SoNames), I64, I64, C.c_int, C.c_char_p, U64, C.POINTER(U64),
      C.POINTER(U32))
    f("so_set_report_entry_node", C.c_int, P, C.POINTER(abi.sf_node_state))
    f("so_load_namespaces", C.c_int, P, C.POINTER(abi.sf_namespace), U32)
    f("so_load_cluster_rules", C.c_int, P, C.POINTER(abi.sf_cluster_flow_rule), U32,
      C.POINTER(abi.sf_cluster_param_rule), U32, C.POINTER(abi.sf_hot_item), U32)
    f("so_request_tokens", C.c_int, P, C.POINTER(abi.sf_token_batch), C.POINTER(abi.sf_token_results))
    f("so_serve_frames", C.c_int, P, C.POINTER(abi.sf_wire_batch), C.POINTER(abi.sf_wire_out))
    f("so_string_key", C.c_uint64, C.c_char_p, C.c_uint32)
    f("so_cluster_sum", I64, P, I64, C.c_int, I64)


class SoNames(C.Structure):
    _fields_ = [("bytes", C.c_char_p), ("offsets", C.POINTER(C.c_uint64)), ("types", C.POINTER(C.c_int32)),
                ("n", C.c_uint32)]


def names_struct(names, types=None):
    """(SoNames, keep-alive) of a list of resource names (str) and types."""
    data = b"".join(n.encode() for n in names)
    off = [0]
    for n in names:
        off.append(off[-1] + len(n.encode()))
    offs = (C.c_uint64 * len(off))(*off)
    ty = (C.c_int32 * len(names))(*types) if types is not None else None
    st = SoNames(data, offs, ty, len(names))
    return st, (data, offs, ty)


def format_fat(rows, names=None, types=None, tz_offset_ms=0):
    """MetricNode.toFatString of rows (sf_metric_row or dict) -> bytes."""
    arr = (abi.sf_metric_row * max(1, len(rows)))()
    for i, r in enumerate(rows):
        if isinstance(r, dict):
            for k, v in r.items():
                setattr(arr[i], k, v)
        else:
            arr[i] = r
    nt, keep = names_struct(names or [], types) if names is not None else (None, None)
    cap = 256 * max(1, len(rows)) + sum(len(n) for n in (names or []))
    buf = C.create_string_buffer(cap)
    n = U64(0)
    rc = lib().so_format_fat(C.byref(nt) if nt else None, arr, len(rows), tz_offset_ms, buf, cap, C.byref(n))
    assert rc == 0, rc
    return buf.raw[:n.value]


class MockNode(C.Structure):
    """Mockito ``when(node.passQps()).thenReturn(..)`` stand-in."""
    _fields_ = [("pass_qps", C.c_double), ("previous_pass_qps", C.c_double), ("cur_thread_num", C.c_int32)]


# MetricEvent ordinals (MetricEvent.java:21-39)
PASS, BLOCK, EXCEPTION, SUCCESS, RT, OCCUPIED_PASS = range(6)
# ClusterFlowEvent ordinals (ClusterFlowEvent.java:22-52)
C_PASS, C_BLOCK, C_PASS_REQUEST, C_BLOCK_REQUEST, C_OCCUPIED_PASS, C_OCCUPIED_BLOCK, C_WAITING = range(7)
LA_BUCKET, LA_OCCUPIABLE, LA_FUTURE, LA_UNARY, LA_CLUSTER = range(5)


def set_time(t: int):
    lib().so_set_time(t)


def now() -> int:
    return lib().so_now()


class LeapArray:
    def __init__(self, kind, sample_count, interval_ms):
        self.h = lib().so_la_new(kind, sample_count, interval_ms)
        assert self.h

    def __del__(self):
        if getattr(self, "h", None):
            lib().so_la_free(self.h)

    def current_window(self, t=None):
        return lib().so_la_current_window_now(self.h) if t is None else lib().so_la_current_window(self.h, t)

    def previous_window(self, t):
        return lib().so_la_previous_window(self.h, t)

    def valid_head(self, t):
        return lib().so_la_valid_head(self.h, t)

    def window_value(self, t):
        return lib().so_la_window_value(self.h, t)

    def values(self, t):
        buf = (P * 128)()
        n = lib().so_la_values(self.h, t, buf, 128)
        return [buf[i] for i in range(n)]

    def list_now(self):
        buf = (P * 128)()
        n = lib().so_la_list_now(self.h, buf, 128)
        return [buf[i] for i in range(n)]

    def current_waiting(self):
        return lib().so_la_current_waiting(self.h)

    def add_waiting(self, t, c):
        lib().so_la_add_waiting(self.h, t, c)


def wrap_start(w):
    return lib().so_wrap_start(w)


def wrap_length(w):
    return lib().so_wrap_length(w)


def wrap_get(w, ev):
    return lib().so_wrap_get(w, ev)


def wrap_add(w, ev, n):
    lib().so_wrap_add(w, ev, n)


class ArrayMetric:
    def __init__(self, sample_count=2, interval_ms=1000, occupy=True):
        self.h = lib().so_am_new(sample_count, interval_ms, int(occupy))

    def __del__(self):
        if getattr(self, "h", None):
            lib().so_am_free(self.h)

    def __getattr__(self, name):
        fn = getattr(lib(), "so_am_" + name)
        return lambda *a: fn(self.h, *a)

    def details(self, lo=None):
        rows = (abi.sf_metric_row * 128)()
        n = lib().so_am_details(self.h, 0 if lo is None else 1, lo or 0, rows, 128)
        return [rows[i] for i in range(n)]


class Node:
    def __init__(self):
        self.h = lib().so_node_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib().so_node_free(self.h)

    def __getattr__(self, name):
        fn = getattr(lib(), "so_node_" + name)
        return lambda *a: fn(self.h, *a)

    def state(self):
        st = abi.sf_node_state()
        lib().so_node_read(self.h, C.byref(st))
        return st


class Controller:
    """TrafficShapingController (DefaultController / WarmUp / RateLimiter / WarmUpRateLimiter)."""

    def __init__(self, handle):
        assert handle, "controller construction failed"
        self.h = handle

    @classmethod
    def default(cls, count, grade=abi.GRADE_QPS):
        return cls(lib().so_ctrl_default(count, grade))

    @classmethod
    def warm_up(cls, count, period, cold_factor=3):
        return cls(lib().so_ctrl_warm_up(count, period, cold_factor))

    @classmethod
    def rate_limiter(cls, timeout_ms, count):
        return cls(lib().so_ctrl_rate_limiter(timeout_ms, count))

    @classmethod
    def warm_up_rate_limiter(cls, count, period, timeout_ms, cold_factor=3):
        return cls(lib().so_ctrl_warm_up_rate_limiter(count, period, timeout_ms, cold_factor))

    def __del__(self):
        if getattr(self, "h", None):
            lib().so_ctrl_free(self.h)

    def can_pass(self, node=None, acquire=1, prioritized=False, mock=None):
        w = I64(0)
        pw = C.c_int(0)
        ok = lib().so_ctrl_can_pass(self.h, node.h if node is not None else None,
                                    C.byref(mock) if mock is not None else None,
                                    acquire, int(prioritized), C.byref(w), C.byref(pw))
        self.last_wait, self.last_prio_wait = w.value, bool(pw.value)
        return bool(ok)

    def state(self):
        s = abi.sf_rule_state()
        lib().so_ctrl_state(self.h, C.byref(s))
        return s

    @property
    def warning_token(self):
        return lib().so_ctrl_warning_token(self.h)

    @property
    def max_token(self):
        return lib().so_ctrl_max_token(self.h)

    @property
    def slope(self):
        return lib().so_ctrl_slope(self.h)


class ParameterMetric:
    def __init__(self, lru: bool = False):
        self.h = lib().so_pm_new_mode(int(lru))

    def __del__(self):
        if getattr(self, "h", None):
            lib().so_pm_free(self.h)

    def initialize(self, key, rule):
        lib().so_pm_initialize(self.h, key, C.byref(rule))

    def pass_single(self, key, rule, value, acquire=1, items=None):
        tag, bits = value
        arr = abi.rules_array(abi.sf_hot_item, items or [])
        w = I64(0)
        ok = lib().so_param_pass_single(self.h, key, C.byref(rule), arr, acquire, tag, bits, C.byref(w))
        self.last_wait = w.value
        return bool(ok)

    def add_thread(self, idx, value):
        lib().so_pm_add_thread(self.h, idx, *value)

    def dec_thread(self, idx, value):
        lib().so_pm_dec_thread(self.h, idx, *value)

    def thread_count(self, idx, value):
        return lib().so_pm_thread_count(self.h, idx, *value)

    def evictions(self):
        return int(lib().so_pm_evictions(self.h))


class ClusterMetric:
    def __init__(self, sample_count=10, interval_ms=1000):
        self.h = lib().so_cm_new(sample_count, interval_ms)

    def __del__(self):
        if getattr(self, "h", None):
            lib().so_cm_free(self.h)

    def add(self, ev, n):
        lib().so_cm_add(self.h, ev, n)

    def sum(self, ev):
        return lib().so_cm_sum(self.h, ev)

    def avg(self, ev):
        return lib().so_cm_avg(self.h, ev)

    def try_occupy_next(self, ev, c, threshold):
        return lib().so_cm_try_occupy_next(self.h, ev, c, threshold)


class ClusterParamMetric:
    def __init__(self, sample_count=10, interval_ms=1000):
        self.h = lib().so_cpm_new(sample_count, interval_ms)

    def __del__(self):
        if getattr(self, "h", None):
            lib().so_cpm_free(self.h)

    def add_value(self, value, c):
        lib().so_cpm_add_value(self.h, value[0], value[1], c)

    def sum(self, value):
        return lib().so_cpm_sum(self.h, *value)

    def avg(self, value):
        return lib().so_cpm_avg(self.h, *value)


class RequestLimiter:
    def __init__(self, qps):
        self.h = lib().so_rl_new(qps)

    def __del__(self):
        if getattr(self, "h", None):
            lib().so_rl_free(self.h)

    def try_pass(self):
        return bool(lib().so_rl_try_pass(self.h))

    def can_pass(self):
        return bool(lib().so_rl_can_pass(self.h))

    def sum(self):
        return lib().so_rl_sum(self.h)

    def add(self, x):
        lib().so_rl_add(self.h, x)


class OracleEngine:
    """Single-threaded replay of StatisticSlot + SystemSlot + ParamFlowSlot + FlowSlot."""

    def __init__(self, cfg: abi.sf_config):
        self.cfg = cfg
        self.h = lib().so_create(C.byref(cfg))

    def close(self):
        if getattr(self, "h", None):
            lib().so_destroy(self.h)
            self.h = None

    __del__ = close

    def load_flow_rules(self, rules):
        ptr, n = abi.flow_rules_ptr(rules)
        rc = lib().so_load_flow_rules(self.h, ptr, n)
        assert rc == 0, rc

    def load_param_rules(self, rules, items=()):
        rc = lib().so_load_param_rules(self.h, abi.rules_array(abi.sf_param_rule, rules), len(rules),
                                       abi.rules_array(abi.sf_hot_item, list(items)), len(items))
        assert rc == 0, rc

    def load_system_rules(self, rules):
        rc = lib().so_load_system_rules(self.h, abi.rules_array(abi.sf_system_rule, rules), len(rules))
        assert rc == 0, rc

    def set_system_status(self, load, cpu):
        lib().so_set_system_status(self.h, load, cpu)

    def set_param_lru(self, on: bool = True):
        """ParameterMetric's CacheMaps as the reference's ConcurrentLinkedHashMap
        LRUs (capacity min(4000*durationInSec, 200000); thread maps 4000),
        instead of the exact maps the engine keeps.  Before the first batch."""
        lib().so_set_param_lru(self.h, int(on))

    def param_lru_stats(self):
        """(evictions, evicted-token spins) over every resource's maps."""
        ev, sp = U64(0), U64(0)
        lib().so_param_lru_stats(self.h, C.byref(ev), C.byref(sp))
        return int(ev.value), int(sp.value)

    def submit(self, batch: abi.HostBatch) -> abi.HostVerdicts:
        out = abi.HostVerdicts(batch.n)
        b = batch.c_struct()
        v = out.c_struct()
        rc = lib().so_submit(self.h, C.byref(b), C.byref(v))
        assert rc == 0, rc
        return out

    def load_degrade_rules(self, rules) -> int:
        """DegradeSlot inside the chain (after FlowSlot); rules as for
        FlowEngine.load_degrade_rules (dicts of sf_degrade_rule fields)."""
        arr = (abi.sf_degrade_rule * max(1, len(rules)))()
        for i, r in enumerate(rules):
            for k, v in r.items():
                setattr(arr[i], k, v)
        n = U32(0)
        rc = lib().so_load_degrade_rules(self.h, arr, len(rules), C.byref(n))
        if rc:
            raise ValueError(f"so_load_degrade_rules: {rc}")
        return int(n.value)

    def read_breaker(self, k) -> abi.sf_breaker_state:
        st = abi.sf_breaker_state()
        assert lib().so_read_breaker(self.h, k, C.byref(st)) == 0
        return st

    # node-wide SystemRule rounds (sentinel_amd/system_shard.py), one IN event per round
    def system_plan(self, merged: abi.HostBatch, status, p: int, sys_mask) -> int:
        b = merged.c_struct()
        q = U32(0)
        rc = lib().so_system_plan(self.h, C.byref(b), None, p, C.byref(q), sys_mask.ctypes.data)
        assert rc == 0, rc
        return int(q.value)

    def submit_forced(self, batch: abi.HostBatch, sys_mask) -> abi.HostVerdicts:
        m = np.ascontiguousarray(sys_mask, np.uint8)
        out = abi.HostVerdicts(batch.n)
        b, v = batch.c_struct(), out.c_struct()
        rc = lib().so_submit_forced(self.h, C.byref(b), C.byref(v), m.ctypes.data)
        assert rc == 0, rc
        return out

    def entry_node_add(self, batch: abi.HostBatch, status):
        st = np.ascontiguousarray(status, np.uint8)
        b = batch.c_struct()
        assert lib().so_entry_node_add(self.h, C.byref(b), st.ctypes.data) == 0

    def read_node(self, res):
        st = abi.sf_node_state()
        assert lib().so_read_node(self.h, res, C.byref(st)) == 0
        return st

    def read_origin_node(self, res, origin):
        st = abi.sf_node_state()
        rc = lib().so_read_origin_node(self.h, res, origin, C.byref(st))
        if rc:
            raise KeyError((res, origin))
        return st

    def read_context_node(self, context, res):
        st = abi.sf_node_state()
        rc = lib().so_read_context_node(self.h, context, res, C.byref(st))
        if rc:
            raise KeyError((context, res))
        return st

    # FlowRuleChecker.selectNodeByRequesterAndStrategy of a loaded rule (SEL_*)
    SEL_NONE, SEL_CLUSTER, SEL_ORIGIN, SEL_CONTEXT, SEL_REF = range(5)

    def select_node(self, rule_index, origin=abi.ORIGIN_NONE, context=0):
        return lib().so_select_node(self.h, rule_index, origin, context)

    def read_entry_node(self):
        st = abi.sf_node_state()
        lib().so_read_entry_node(self.h, C.byref(st))
        return st

    def read_rule_state(self, idx):
        s = abi.sf_rule_state()
        assert lib().so_read_rule_state(self.h, idx, C.byref(s)) == 0
        return s

    def node_digests(self, n_rows):
        """FNV-1a digest of every local row's canonical node state (so_node_digests)."""
        out = np.empty(n_rows, np.uint64)
        assert lib().so_node_digests(self.h, out.ctypes.data, n_rows) == 0
        return out

    def rule_states(self, first, n):
        """(n, 3) int64: stored_tokens, last_filled_time, latest_passed_time of rules first..first+n-1."""
        out = np.empty((n, 3), np.int64)
        assert lib().so_read_rule_states(self.h, first, n, out.ctypes.data) == 0
        return out

    def read_param(self, rule_idx, value):
        t, k, h = I64(0), I64(0), C.c_int(0)
        present = lib().so_read_param(self.h, rule_idx, value[0], value[1], C.byref(t), C.byref(k), C.byref(h))
        return bool(present), t.value, (k.value if h.value else None)

    def param_rule_idx(self, k):
        return lib().so_param_rule_idx(self.h, k)

    def param_thread(self, res, idx, value):
        return lib().so_param_thread(self.h, res, idx, value[0], value[1])

    def snapshot(self, now, cap=1 << 16):
        rows = (abi.sf_metric_row * cap)()
        n = U32(0)
        rc = lib().so_snapshot(self.h, now, rows, cap, C.byref(n))
        assert rc == 0, rc
        return [rows[i] for i in range(n.value)]

    def metric_log(self, now, names=None, types=None, tz_offset_ms=0, entry_node=True, cap=1 << 22):
        nt, keep = names_struct(names, types) if names is not None else (None, None)
        buf = C.create_string_buffer(cap)
        n, k = U64(0), U32(0)
        rc = lib().so_metric_log(self.h, C.byref(nt) if nt else None, now, tz_offset_ms, int(entry_node), buf, cap,
                                 C.byref(n), C.byref(k))
        assert rc == 0, rc
        return buf.raw[:n.value]

    def set_report_entry_node(self, node=None):
        lib().so_set_report_entry_node(self.h, None if node is None else C.byref(node))

    def load_namespaces(self, ns):
        lib().so_load_namespaces(self.h, abi.rules_array(abi.sf_namespace, ns), len(ns))

    def load_cluster_rules(self, flow=(), param=(), items=()):
        lib().so_load_cluster_rules(self.h, abi.rules_array(abi.sf_cluster_flow_rule, list(flow)), len(flow),
                                    abi.rules_array(abi.sf_cluster_param_rule, list(param)), len(param),
                                    abi.rules_array(abi.sf_hot_item, list(items)), len(items))

    def request_tokens(self, batch: abi.HostTokenBatch) -> abi.HostTokenResults:
        out = abi.HostTokenResults(batch.n)
        b = batch.c_struct()
        r = out.c_struct()
        rc = lib().so_request_tokens(self.h, C.byref(b), C.byref(r))
        assert rc == 0, rc
        return out

    def serve_frames(self, streams, now_ms) -> abi.WireResult:
        r = abi.WireResult(streams, now_ms)
        b, o = r.c_structs()
        rc = lib().so_serve_frames(self.h, C.byref(b), C.byref(o))
        assert rc == 0, rc
        return r.finish(o)

    def cluster_sum(self, flow_id, event, now):
        return lib().so_cluster_sum(self.h, flow_id, event, now)
