"""ctypes mirror of ``include/sentinel_flow.h`` (the C-ABI drop-in boundary).

Every structure here matches the header field for field; ``tests/test_abi.py``
checks the sizes against the compiled library.  Nothing in this module touches
a GPU: it only describes memory layouts and wraps numpy arrays.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

SF_ABI_VERSION = 1

SF_OK = 0
SF_ERR_INVALID = -1
SF_ERR_NOMEM = -2
SF_ERR_DEVICE = -3
SF_ERR_UNSUPPORTED = -4
SF_ERR_CAPACITY = -5

# RuleConstant.java:26-66
GRADE_THREAD, GRADE_QPS = 0, 1
STRATEGY_DIRECT, STRATEGY_RELATE, STRATEGY_CHAIN = 0, 1, 2
BEHAVIOR_DEFAULT, BEHAVIOR_WARM_UP, BEHAVIOR_RATE_LIMITER, BEHAVIOR_WARM_UP_RATE_LIMITER = 0, 1, 2, 3
THRESHOLD_AVG_LOCAL, THRESHOLD_GLOBAL = 0, 1

SF_MAX_SAMPLE_COUNT = 16
SF_MINUTE_BUCKETS = 60
SF_WS_ABSENT = -(2 ** 63)
RES_ENTRY_NODE = 0xFFFFFFFF      # sf_metric_row.resource of Constants.ENTRY_NODE
SF_MAX_RULES_PER_RESOURCE = 8
SF_MAX_ARGS = 4

TAG_NULL, TAG_INT, TAG_LONG, TAG_STRING, TAG_DOUBLE, TAG_BOOL, TAG_OTHER, TAG_BYTE, TAG_SHORT, TAG_FLOAT = range(10)
TAG_COLLECTION = 0x40        # a Collection / array argument: elements listed in the CSR

EV_EXIT, EV_IN, EV_PRIO, EV_ERROR = 0x01, 0x02, 0x04, 0x08
EV_BLOCKED = 0x10            # entry blocked by a slot the engine wraps but does not run (AuthoritySlot)
MEM_HOST, MEM_DEVICE = 0, 1

V_PASS, V_PASS_WAIT, V_PRIORITY_WAIT, V_BLOCK_FLOW, V_BLOCK_PARAM, V_BLOCK_SYSTEM, V_EXIT, V_EXIT_IGNORED = range(8)
PASSED = (V_PASS, V_PASS_WAIT, V_PRIORITY_WAIT)

TOKEN_OK, TOKEN_BLOCKED, TOKEN_SHOULD_WAIT, TOKEN_NO_RULE_EXISTS = 0, 1, 2, 3
TOKEN_BAD_REQUEST, TOKEN_TOO_MANY_REQUEST, TOKEN_FAIL = -4, -2, -1
TOK_PRIORITIZED, TOK_PARAM = 0x01, 0x02

WS_ABSENT = -(2 ** 63)


class sf_config(C.Structure):
    _fields_ = [
        ("sample_count", C.c_int32), ("interval_ms", C.c_int32),
        ("occupy_timeout_ms", C.c_int32), ("cold_factor", C.c_int32),
        ("statistic_max_rt", C.c_int64),
        ("max_resources", C.c_uint32), ("max_batch", C.c_uint32),
        ("param_capacity", C.c_uint32), ("shard_count", C.c_uint32),
        ("shard_index", C.c_uint32), ("device", C.c_int32),
        ("cluster_sample_count", C.c_int32), ("cluster_interval_ms", C.c_int32),
        ("exceed_count", C.c_double), ("max_occupy_ratio", C.c_double),
        ("max_flow_ids", C.c_uint32), ("heavy_min_events", C.c_uint32),
        ("aux_capacity", C.c_uint32), ("pad", C.c_uint32),
    ]


def default_config(**kw) -> sf_config:
    """``sf_config_default`` restated in Python (reference defaults)."""
    cfg = sf_config(sample_count=2, interval_ms=1000, occupy_timeout_ms=500, cold_factor=3,
                    statistic_max_rt=5000, max_resources=1024, max_batch=1 << 20,
                    param_capacity=1 << 16, shard_count=1, shard_index=0, device=0,
                    cluster_sample_count=10, cluster_interval_ms=1000, exceed_count=1.0,
                    max_occupy_ratio=1.0, max_flow_ids=1024, heavy_min_events=0, aux_capacity=65536)
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


# origin / limitApp ids (sentinel_flow.h): 0 "default", 1 "other", >= 2 an origin name, NONE = ""
APP_DEFAULT, APP_OTHER = 0, 1
ORIGIN_NONE = 0xFFFFFFFF
REF_NONE = 0xFFFFFFFF


class sf_flow_rule(C.Structure):
    _fields_ = [
        ("resource", C.c_uint32), ("grade", C.c_int32), ("count", C.c_double),
        ("strategy", C.c_int32), ("control_behavior", C.c_int32),
        ("warm_up_period_sec", C.c_int32), ("max_queueing_time_ms", C.c_int32),
        ("cluster_mode", C.c_int32), ("ref_resource", C.c_uint32),
        ("limit_app", C.c_uint32), ("cluster_fallback", C.c_int32),
    ]


class sf_hot_item(C.Structure):
    _fields_ = [("tag", C.c_uint8), ("pad", C.c_uint8 * 3), ("count", C.c_int32), ("bits", C.c_uint64)]


class sf_param_rule(C.Structure):
    _fields_ = [
        ("resource", C.c_uint32), ("grade", C.c_int32), ("param_idx", C.c_int32),
        ("control_behavior", C.c_int32), ("count", C.c_double),
        ("max_queueing_time_ms", C.c_int32), ("burst_count", C.c_int32),
        ("duration_in_sec", C.c_int64), ("item_offset", C.c_uint32), ("item_count", C.c_uint32),
    ]


class sf_rule_key(C.Structure):
    """Java hash codes of a rule's String fields (sentinel_flow.h sf_rule_key)."""
    _fields_ = [("resource_hash", C.c_int32), ("limit_app_id", C.c_uint32),
                ("limit_app_hash", C.c_int32), ("extra_hash", C.c_int32),
                ("cluster_hash", C.c_int32)]


class sf_system_rule(C.Structure):
    _fields_ = [
        ("highest_system_load", C.c_double), ("highest_cpu_usage", C.c_double),
        ("qps", C.c_double), ("avg_rt", C.c_int64), ("max_thread", C.c_int64),
    ]


class sf_event_batch(C.Structure):
    _fields_ = [
        ("n", C.c_uint32), ("mem", C.c_int32),
        ("res_id", C.c_void_p), ("ts_ms", C.c_void_p), ("count", C.c_void_p),
        ("flags", C.c_void_p), ("entry_ref", C.c_void_p), ("create_ts", C.c_void_p),
        ("arg_slots", C.c_uint32), ("n_args", C.c_void_p),
        ("arg_tag", C.c_void_p), ("arg_bits", C.c_void_p),
        ("arg_elem_off", C.c_void_p), ("elem_tag", C.c_void_p), ("elem_bits", C.c_void_p),
        ("n_elems", C.c_uint32), ("origin", C.c_void_p), ("context", C.c_void_p),
    ]


class sf_verdicts(C.Structure):
    _fields_ = [("mem", C.c_int32), ("status", C.c_void_p), ("wait_ms", C.c_void_p), ("rule_idx", C.c_void_p)]


class sf_cluster_flow_rule(C.Structure):
    _fields_ = [
        ("flow_id", C.c_int64), ("count", C.c_double), ("threshold_type", C.c_int32),
        ("namespace_id", C.c_uint32), ("sample_count", C.c_int32), ("window_interval_ms", C.c_int32),
    ]


class sf_cluster_param_rule(C.Structure):
    _fields_ = [
        ("flow_id", C.c_int64), ("count", C.c_double), ("threshold_type", C.c_int32),
        ("namespace_id", C.c_uint32), ("sample_count", C.c_int32), ("window_interval_ms", C.c_int32),
        ("item_offset", C.c_uint32), ("item_count", C.c_uint32),
    ]


class sf_namespace(C.Structure):
    _fields_ = [("namespace_id", C.c_uint32), ("connected_count", C.c_int32), ("max_allowed_qps", C.c_double)]


class sf_token_batch(C.Structure):
    _fields_ = [
        ("n", C.c_uint32), ("mem", C.c_int32), ("flow_id", C.c_void_p), ("count", C.c_void_p),
        ("flags", C.c_void_p), ("ts_ms", C.c_void_p), ("param_tag", C.c_void_p), ("param_bits", C.c_void_p),
        ("param_off", C.c_void_p),
    ]


class sf_token_results(C.Structure):
    _fields_ = [("mem", C.c_int32), ("status", C.c_void_p), ("remaining", C.c_void_p), ("wait_ms", C.c_void_p)]


class sf_bucket(C.Structure):
    _fields_ = [(n, C.c_int64) for n in
                ("window_start", "pass_", "block", "exception", "success", "rt", "occupied_pass", "min_rt")]


class sf_node_state(C.Structure):
    _fields_ = [
        ("second", sf_bucket * SF_MAX_SAMPLE_COUNT),
        ("borrow_ws", C.c_int64 * SF_MAX_SAMPLE_COUNT),
        ("borrow_pass", C.c_int64 * SF_MAX_SAMPLE_COUNT),
        ("minute", sf_bucket * SF_MINUTE_BUCKETS),
        ("cur_thread_num", C.c_int64),
    ]


class sf_sparse_verdicts(C.Structure):
    _fields_ = [("status", C.c_void_p), ("waits", C.c_void_p), ("rules", C.c_void_p), ("counts", C.c_void_p),
                ("prefetch", C.c_uint32), ("pad", C.c_uint32)]


class HostSparseVerdicts:
    """sf_sparse_verdicts in numpy arrays: 1 status byte per event plus the
    lists of nonzero waits / rule indices (index << 32 | value, any order)."""

    def __init__(self, n: int, prefetch: int = 0, alloc=None):
        alloc = alloc or (lambda shape, dtype: np.zeros(shape, dtype))
        self.n = n
        self.status = alloc((n,), np.uint8)
        self.waits = alloc((max(n, 1),), np.uint64)
        self.rules = alloc((max(n, 1),), np.uint64)
        self.counts = alloc((2,), np.uint32)
        self.prefetch = int(prefetch)

    def c_struct(self) -> sf_sparse_verdicts:
        return sf_sparse_verdicts(self.status.ctypes.data, self.waits.ctypes.data, self.rules.ctypes.data,
                                  self.counts.ctypes.data, self.prefetch, 0)

    def dense(self) -> "HostVerdicts":
        v = HostVerdicts(self.n)
        v.status[:] = self.status
        w = self.waits[:int(self.counts[0])]
        r = self.rules[:int(self.counts[1])]
        v.wait_ms[(w >> np.uint64(32)).astype(np.int64)] = (w & np.uint64(0xffffffff)).astype(np.uint32).view(np.int32)
        v.rule_idx[(r >> np.uint64(32)).astype(np.int64)] = (r & np.uint64(0xffff)).astype(np.uint16)
        return v


class sf_rule_state(C.Structure):
    _fields_ = [("stored_tokens", C.c_int64), ("last_filled_time", C.c_int64), ("latest_passed_time", C.c_int64)]


class sf_metric_row(C.Structure):
    _fields_ = [("resource", C.c_uint32), ("concurrency", C.c_int32), ("timestamp", C.c_int64),
                ("pass_qps", C.c_int64), ("block_qps", C.c_int64), ("success_qps", C.c_int64),
                ("exception_qps", C.c_int64), ("rt", C.c_int64), ("occupied_pass_qps", C.c_int64)]


class sf_stats(C.Structure):
    _fields_ = [("total_ms", C.c_double), ("sort_ms", C.c_double), ("decide_ms", C.c_double),
                ("scatter_ms", C.c_double), ("n_events", C.c_uint64), ("n_segments", C.c_uint64),
                ("n_launches", C.c_uint64), ("light_ms", C.c_double), ("heavy_decide_ms", C.c_double),
                ("heavy_fill_ms", C.c_double), ("classify_ms", C.c_double),
                ("stream_ms", C.c_double), ("metric_scan_ms", C.c_double), ("metric_log_ms", C.c_double),
                ("wire_ms", C.c_double), ("sys_rounds", C.c_uint64), ("aux_nodes", C.c_uint64),
                ("aux_capacity", C.c_uint64), ("aux_index_grows", C.c_uint64), ("param_table_grows", C.c_uint64),
                ("xw_chunks_exact", C.c_uint64), ("xw_chunks_serial", C.c_uint64), ("xw_rounds", C.c_uint64),
                ("xw_serial_events", C.c_uint64), ("sys_exchanges", C.c_uint64)]


class sf_heavy_profile(C.Structure):
    _fields_ = [("resource", C.c_uint32), ("events", C.c_uint32), ("mode", C.c_uint32), ("start", C.c_uint32),
                ("ticks", C.c_uint64)]


STRUCT_SIZES = {name: C.sizeof(cls) for name, cls in [
    ("sf_config", sf_config), ("sf_flow_rule", sf_flow_rule), ("sf_hot_item", sf_hot_item),
    ("sf_param_rule", sf_param_rule), ("sf_system_rule", sf_system_rule), ("sf_rule_key", sf_rule_key),
    ("sf_event_batch", sf_event_batch), ("sf_verdicts", sf_verdicts),
    ("sf_cluster_flow_rule", sf_cluster_flow_rule), ("sf_cluster_param_rule", sf_cluster_param_rule),
    ("sf_namespace", sf_namespace), ("sf_heavy_profile", sf_heavy_profile), ("sf_token_batch", sf_token_batch),
    ("sf_token_results", sf_token_results), ("sf_bucket", sf_bucket), ("sf_node_state", sf_node_state),
    ("sf_rule_state", sf_rule_state), ("sf_metric_row", sf_metric_row), ("sf_stats", sf_stats)]}


def node_state_to_dict(st: sf_node_state, sample_count: int = 2) -> dict:
    """Plain-python view of a node state, for equality checks in tests."""
    def b(x):
        return (x.window_start, x.pass_, x.block, x.exception, x.success, x.rt, x.occupied_pass, x.min_rt)
    return {
        "second": [b(st.second[i]) for i in range(sample_count)],
        "borrow": [(st.borrow_ws[i], st.borrow_pass[i]) for i in range(sample_count)],
        "minute": [b(st.minute[i]) for i in range(SF_MINUTE_BUCKETS)],
        "threads": st.cur_thread_num,
    }


def _ptr(a):
    return None if a is None else a.ctypes.data


PK_COUNT_SHIFT, PK_FLAGS_SHIFT = 52, 59
PK4_COUNT_SHIFT, PK4_FLAGS_SHIFT = 24, 27


class sf_packed_batch(C.Structure):
    _fields_ = [("n", C.c_uint32), ("mem", C.c_int32), ("ts_base", C.c_int64), ("ev", C.c_void_p),
                ("exit_ref", C.c_void_p), ("exit_cts", C.c_void_p), ("count_ext", C.c_void_p),
                ("origin", C.c_void_p), ("n_exit", C.c_uint32), ("n_count_ext", C.c_uint32),
                ("ev4", C.c_void_p), ("ms_end", C.c_void_p), ("n_ms", C.c_uint32), ("pad0", C.c_uint32)]


STRUCT_SIZES["sf_packed_batch"] = C.sizeof(sf_packed_batch)


class PackedBatch:
    """A batch in the compact form of sf_submit_packed (8 bytes per event:
    resource | ts - ts_base << 32 | acquireCount << 52 | flags << 59, plus the
    EXIT events' entry_ref / create_ts and the acquireCounts outside 1..127 as
    sparse arrays).  ``alloc`` places the arrays (np.empty by default; a
    PinnedArrays.array for page-locked memory)."""

    def __init__(self, hb: "HostBatch", alloc=None, narrow=False):
        """narrow: the 4-byte form (resource ids below 2^24; acquireCounts 1..7
        inline, the time as the per-millisecond table ms_end); "auto" picks it
        when the resource ids fit."""
        alloc = alloc or (lambda shape, dtype: np.empty(shape, dtype))
        n = hb.n
        self.n = n
        self.ts_base = int(hb.ts_ms[0]) if n else 0
        d = (hb.ts_ms - self.ts_base).astype(np.int64)
        if n and (d.min() < 0 or d.max() >= (1 << 20)):
            # the 20-bit delta would spill into the acquireCount bits (sf_packed_batch)
            raise ValueError("a packed batch must be time-ordered and span less than 2^20 ms")
        if narrow == "auto":
            narrow = n > 0 and int(hb.res_id.max()) < (1 << 24)
        if narrow and n and int(hb.res_id.max()) >= (1 << 24):
            raise ValueError("the narrow packed form takes resource ids below 2^24")
        self.narrow = bool(narrow)
        if self.narrow and n and (np.diff(d) < 0).any():
            raise ValueError("the narrow packed form takes a time-ordered batch")
        c = hb.count.astype(np.int64)
        self.ev = self.ev4 = self.ms_end = None
        self.n_ms = 0
        if self.narrow:
            small = (c >= 1) & (c <= 7)
            w = hb.res_id.astype(np.uint32) | (np.where(small, c, 0).astype(np.uint32) << np.uint32(PK4_COUNT_SHIFT)) | \
                ((hb.flags.astype(np.uint32) & np.uint32(0x1f)) << np.uint32(PK4_FLAGS_SHIFT))
            self.ev4 = alloc((n,), np.uint32)
            self.ev4[...] = w
            self.n_ms = int(d[-1]) + 1 if n else 1
            self.ms_end = alloc((self.n_ms,), np.uint32)
            self.ms_end[...] = np.cumsum(np.bincount(d, minlength=self.n_ms)).astype(np.uint32)
        else:
            small = (c >= 1) & (c <= 127)
            w = hb.res_id.astype(np.uint64) | (d.astype(np.uint64) << np.uint64(32)) | \
                (np.where(small, c, 0).astype(np.uint64) << np.uint64(PK_COUNT_SHIFT)) | \
                ((hb.flags.astype(np.uint64) & np.uint64(0x1f)) << np.uint64(PK_FLAGS_SHIFT))
            self.ev = alloc((n,), np.uint64)
            self.ev[...] = w
        ex = np.nonzero(hb.flags & EV_EXIT)[0]
        self.n_exit = int(ex.size)
        self.exit_ref = self.exit_cts = None
        if ex.size:
            self.exit_ref = alloc((ex.size,), np.int64)
            self.exit_ref[...] = hb.entry_ref[ex] if hb.entry_ref is not None else -1
            if hb.create_ts is not None:
                self.exit_cts = alloc((ex.size,), np.int64)
                self.exit_cts[...] = hb.create_ts[ex]
        big = np.nonzero(~small)[0]
        self.n_count_ext = int(big.size)
        self.count_ext = None
        if big.size:
            self.count_ext = alloc((big.size,), np.int32)
            self.count_ext[...] = hb.count[big]
        self.origin = None
        if hb.origin is not None:
            self.origin = alloc((n,), np.uint32)
            self.origin[...] = hb.origin

    def nbytes(self) -> int:
        return sum(a.nbytes for a in (self.ev, self.ev4, self.ms_end, self.exit_ref, self.exit_cts, self.count_ext,
                                      self.origin) if a is not None)

    def c_struct(self) -> sf_packed_batch:
        b = sf_packed_batch()
        b.n, b.mem, b.ts_base = self.n, MEM_HOST, self.ts_base
        b.ev, b.exit_ref, b.exit_cts = _ptr(self.ev), _ptr(self.exit_ref), _ptr(self.exit_cts)
        b.count_ext, b.origin = _ptr(self.count_ext), _ptr(self.origin)
        b.n_exit, b.n_count_ext = self.n_exit, self.n_count_ext
        b.ev4, b.ms_end, b.n_ms = _ptr(self.ev4), _ptr(self.ms_end), self.n_ms
        return b


class HostBatch:
    """A time-ordered event batch held in host numpy arrays (SoA).

    Keeps the arrays alive while the ``sf_event_batch`` that points at them is
    in use.
    """

    def __init__(self, res_id, ts_ms, count, flags, entry_ref=None, create_ts=None,
                 arg_tag=None, arg_bits=None, n_args=None, elem_off=None, elem_tag=None, elem_bits=None,
                 origin=None, context=None):
        self.res_id = np.ascontiguousarray(res_id, dtype=np.uint32)
        self.ts_ms = np.ascontiguousarray(ts_ms, dtype=np.int64)
        self.count = np.ascontiguousarray(count, dtype=np.int32)
        self.flags = np.ascontiguousarray(flags, dtype=np.uint8)
        n = self.res_id.shape[0]
        assert self.ts_ms.shape == (n,) and self.count.shape == (n,) and self.flags.shape == (n,)
        self.entry_ref = None if entry_ref is None else np.ascontiguousarray(entry_ref, dtype=np.int64)
        self.create_ts = None if create_ts is None else np.ascontiguousarray(create_ts, dtype=np.int64)
        if arg_tag is not None:
            arg_tag = np.ascontiguousarray(arg_tag, dtype=np.uint8)
            arg_bits = np.ascontiguousarray(arg_bits, dtype=np.uint64)
            if arg_tag.ndim == 1:
                arg_tag = arg_tag.reshape(1, n)
                arg_bits = arg_bits.reshape(1, n)
            assert arg_tag.shape[1] == n and arg_bits.shape == arg_tag.shape
        self.arg_tag = arg_tag
        self.arg_bits = arg_bits
        self.n_args = None if n_args is None else np.ascontiguousarray(n_args, dtype=np.uint8)
        self.n = n
        # collection / array args: elements of arg k = slot*n + i at [elem_off[k], elem_off[k+1])
        self.elem_off = None if elem_off is None else np.ascontiguousarray(elem_off, dtype=np.uint32)
        self.elem_tag = None if elem_tag is None else np.ascontiguousarray(elem_tag, dtype=np.uint8)
        self.elem_bits = None if elem_bits is None else np.ascontiguousarray(elem_bits, dtype=np.uint64)
        if self.elem_off is not None:
            assert arg_tag is not None and self.elem_off.shape == (arg_tag.shape[0] * n + 1,)
            assert self.elem_tag.shape == self.elem_bits.shape == (int(self.elem_off[-1]),)
        # Context origin / name ids per event (ORIGIN_NONE = ""); None: no origin, context 0
        self.origin = None if origin is None else np.ascontiguousarray(origin, dtype=np.uint32)
        self.context = None if context is None else np.ascontiguousarray(context, dtype=np.uint32)
        assert self.origin is None or self.origin.shape == (n,)
        assert self.context is None or self.context.shape == (n,)

    def _take_ctx(self, sel):
        return (None if self.origin is None else self.origin[sel].copy(),
                None if self.context is None else self.context[sel].copy())

    @staticmethod
    def collections(slots, n, values):
        """(arg_tag, arg_bits, elem_off, elem_tag, elem_bits) from values[slot][i]:
        None (null), (tag, bits), or a list of (tag, bits) / None elements (a
        Collection or array)."""
        at = np.zeros((slots, n), np.uint8)
        ab = np.zeros((slots, n), np.uint64)
        off = np.zeros(slots * n + 1, np.uint32)
        et, eb = [], []
        for a in range(slots):
            for i in range(n):
                v = values[a][i]
                if isinstance(v, list):
                    at[a, i] = TAG_COLLECTION
                    for x in v:
                        et.append(TAG_NULL if x is None else x[0])
                        eb.append(0 if x is None else x[1])
                elif v is not None:
                    at[a, i], ab[a, i] = v[0], v[1]
                off[a * n + i + 1] = len(et)
        return at, ab, off, np.array(et, np.uint8), np.array(eb, np.uint64)

    def _take_args(self, sel):
        """args of the events sel (ascending), collections re-packed."""
        at = None if self.arg_tag is None else self.arg_tag[:, sel].copy()
        ab = None if self.arg_bits is None else self.arg_bits[:, sel].copy()
        na = None if self.n_args is None else self.n_args[sel]
        if self.elem_off is None:
            return at, ab, na, None, None, None
        slots = self.arg_tag.shape[0]
        off, et, eb = [0], [], []
        for a in range(slots):
            for i in sel:
                k = a * self.n + int(i)
                lo, hi = int(self.elem_off[k]), int(self.elem_off[k + 1])
                et.append(self.elem_tag[lo:hi]); eb.append(self.elem_bits[lo:hi])
                off.append(off[-1] + hi - lo)
        cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)  # noqa: E731
        return at, ab, na, np.array(off, np.uint32), cat(et, np.uint8), cat(eb, np.uint64)

    def shard(self, world: int, rank: int) -> "HostBatch":
        """The events of the resources ``res % world == rank`` (hash sharding),
        time order kept; entry_ref indices are remapped into the shard."""
        sel = np.nonzero(self.res_id % world == rank)[0]
        er = ct = None
        if self.entry_ref is not None:
            pos = np.full(self.n, -1, np.int64)
            pos[sel] = np.arange(sel.size)
            er = self.entry_ref[sel].copy()
            er[er >= 0] = pos[er[er >= 0]]
            ct = None if self.create_ts is None else self.create_ts[sel].copy()
        at, ab, na, eo, et, eb = self._take_args(sel)
        og, cx = self._take_ctx(sel)
        return HostBatch(self.res_id[sel], self.ts_ms[sel], self.count[sel], self.flags[sel], er, ct, at, ab, na,
                         eo, et, eb, og, cx)

    def subset(self, lo: int, hi: int) -> "HostBatch":
        """Contiguous slice [lo, hi); entry_ref indices are rebased (refs before lo become -1)."""
        er = None
        ct = None
        if self.entry_ref is not None:
            er = self.entry_ref[lo:hi].copy()
            ct = np.zeros(hi - lo, np.int64) if self.create_ts is None else self.create_ts[lo:hi].copy()
            prior = (er >= 0) & (er < lo)
            ct[prior] = self.ts_ms[er[prior]]
            er[prior] = -1
            er[er >= lo] -= lo
        at, ab, na, eo, et, eb = self._take_args(np.arange(lo, hi))
        og, cx = self._take_ctx(np.arange(lo, hi))
        return HostBatch(self.res_id[lo:hi], self.ts_ms[lo:hi], self.count[lo:hi], self.flags[lo:hi],
                         er, ct, at, ab, na, eo, et, eb, og, cx)

    def c_struct(self) -> sf_event_batch:
        b = sf_event_batch()
        b.n = self.n
        b.mem = MEM_HOST
        b.res_id, b.ts_ms, b.count, b.flags = (_ptr(self.res_id), _ptr(self.ts_ms), _ptr(self.count), _ptr(self.flags))
        b.entry_ref = _ptr(self.entry_ref)
        b.create_ts = _ptr(self.create_ts)
        if self.arg_tag is not None:
            b.arg_slots = self.arg_tag.shape[0]
            b.arg_tag = _ptr(self.arg_tag)
            b.arg_bits = _ptr(self.arg_bits)
        else:
            b.arg_slots = 0
        b.n_args = _ptr(self.n_args)
        if self.elem_off is not None:
            b.arg_elem_off, b.elem_tag, b.elem_bits = _ptr(self.elem_off), _ptr(self.elem_tag), _ptr(self.elem_bits)
            b.n_elems = int(self.elem_off[-1])
        b.origin, b.context = _ptr(self.origin), _ptr(self.context)
        return b


class HostVerdicts:
    def __init__(self, n: int):
        self.status = np.full(n, 255, np.uint8)
        self.wait_ms = np.zeros(n, np.int32)
        self.rule_idx = np.zeros(n, np.uint16)

    def c_struct(self) -> sf_verdicts:
        v = sf_verdicts()
        v.mem = MEM_HOST
        v.status, v.wait_ms, v.rule_idx = _ptr(self.status), _ptr(self.wait_ms), _ptr(self.rule_idx)
        return v


class HostTokenBatch:
    def __init__(self, flow_id, count, flags, ts_ms, param_tag=None, param_bits=None, param_off=None):
        self.flow_id = np.ascontiguousarray(flow_id, np.int64)
        self.count = np.ascontiguousarray(count, np.int32)
        self.flags = np.ascontiguousarray(flags, np.uint8)
        self.ts_ms = np.ascontiguousarray(ts_ms, np.int64)
        self.param_tag = None if param_tag is None else np.ascontiguousarray(param_tag, np.uint8)
        self.param_bits = None if param_bits is None else np.ascontiguousarray(param_bits, np.uint64)
        self.n = self.flow_id.shape[0]
        # Collection<Object> params: request i's values at [param_off[i], param_off[i+1])
        self.param_off = None if param_off is None else np.ascontiguousarray(param_off, np.uint32)
        if self.param_off is not None:
            assert self.param_off.shape == (self.n + 1,) and self.param_tag.shape == (int(self.param_off[-1]),)

    def c_struct(self) -> sf_token_batch:
        t = sf_token_batch()
        t.n, t.mem = self.n, MEM_HOST
        t.flow_id, t.count, t.flags, t.ts_ms = (_ptr(self.flow_id), _ptr(self.count), _ptr(self.flags), _ptr(self.ts_ms))
        t.param_tag, t.param_bits = _ptr(self.param_tag), _ptr(self.param_bits)
        t.param_off = _ptr(self.param_off)
        return t

    def take(self, sel) -> "HostTokenBatch":
        """The requests sel (ascending), values re-packed."""
        sel = np.asarray(sel, np.int64)
        if self.param_off is None:
            pt = None if self.param_tag is None else self.param_tag[sel]
            pb = None if self.param_bits is None else self.param_bits[sel]
            return HostTokenBatch(self.flow_id[sel], self.count[sel], self.flags[sel], self.ts_ms[sel], pt, pb)
        lo, hi = self.param_off[sel], self.param_off[sel + 1]
        idx = np.concatenate([np.arange(a, b) for a, b in zip(lo, hi)]) if sel.size else np.zeros(0, np.int64)
        off = np.concatenate([[0], np.cumsum(hi - lo)]).astype(np.uint32)
        return HostTokenBatch(self.flow_id[sel], self.count[sel], self.flags[sel], self.ts_ms[sel],
                              self.param_tag[idx], self.param_bits[idx], off)


class HostTokenResults:
    def __init__(self, n: int):
        self.status = np.full(n, 99, np.int8)
        self.remaining = np.zeros(n, np.int32)
        self.wait_ms = np.zeros(n, np.int32)

    def c_struct(self) -> sf_token_results:
        r = sf_token_results()
        r.mem = MEM_HOST
        r.status, r.remaining, r.wait_ms = _ptr(self.status), _ptr(self.remaining), _ptr(self.wait_ms)
        return r


def rules_array(cls, rules):
    arr = (cls * max(1, len(rules)))()
    for i, r in enumerate(rules):
        arr[i] = r
    return arr


# numpy views of the rule structs, for loading millions of rules without
# building Python objects (layouts pinned by tests/test_abi.py).
FLOW_RULE_DTYPE = np.dtype({
    "names": [n for n, _ in sf_flow_rule._fields_],
    "formats": [{C.c_uint32: np.uint32, C.c_int32: np.int32, C.c_double: np.float64}[t] for _, t in sf_flow_rule._fields_],
    "offsets": [getattr(sf_flow_rule, n).offset for n, _ in sf_flow_rule._fields_],
    "itemsize": C.sizeof(sf_flow_rule)})


def flow_rules_np(resource, grade, count, behavior, warm_up=10, max_queue=500) -> np.ndarray:
    n = len(resource)
    a = np.zeros(n, FLOW_RULE_DTYPE)
    a["resource"] = resource
    a["grade"] = grade
    a["count"] = count
    a["control_behavior"] = behavior
    a["warm_up_period_sec"] = warm_up
    a["max_queueing_time_ms"] = max_queue
    return a


def flow_rules_ptr(rules):
    """(pointer, n) for a list of sf_flow_rule or a FLOW_RULE_DTYPE array."""
    if isinstance(rules, np.ndarray):
        assert rules.dtype == FLOW_RULE_DTYPE
        return C.cast(rules.ctypes.data, C.POINTER(sf_flow_rule)), rules.shape[0]
    return rules_array(sf_flow_rule, list(rules)), len(rules)


WIRE_DONE, WIRE_PARTIAL, WIRE_HOST = 0, 1, 2
WIRE_RESP_BYTES = 16


class sf_wire_batch(C.Structure):
    _fields_ = [("mem", C.c_int32), ("n_streams", C.c_uint32), ("bytes", C.c_void_p), ("stream_off", C.c_void_p),
                ("now_ms", C.c_int64)]


class sf_wire_out(C.Structure):
    _fields_ = [("resp", C.c_void_p), ("cap", C.c_uint64), ("resp_off", C.c_void_p), ("consumed", C.c_void_p),
                ("stop", C.c_void_p), ("n_frames", C.c_uint64), ("n_requests", C.c_uint64),
                ("n_responses", C.c_uint64)]


STRUCT_SIZES.update({"sf_wire_batch": C.sizeof(sf_wire_batch), "sf_wire_out": C.sizeof(sf_wire_out)})


class WireResult:
    """Result of one sf_serve_frames / so_serve_frames call over host memory."""

    def __init__(self, streams, now_ms):
        self.streams = [bytes(x) for x in streams]
        S = len(self.streams)
        self.data = np.frombuffer(b"".join(self.streams) + b"\0" * 16, dtype=np.uint8)
        self.off = np.zeros(S + 1, np.uint64)
        self.off[1:] = np.cumsum([len(x) for x in self.streams])
        total = int(self.off[-1])
        self.resp = np.zeros(max(total // 2 + 1, 1) * WIRE_RESP_BYTES, np.uint8)
        self.resp_off = np.zeros(S + 1, np.uint64)
        self.consumed = np.zeros(S, np.uint64)
        self.stop = np.zeros(S, np.uint8)
        self.now_ms = now_ms

    def c_structs(self):
        b = sf_wire_batch(MEM_HOST, len(self.streams), self.data.ctypes.data, self.off.ctypes.data, self.now_ms)
        o = sf_wire_out(self.resp.ctypes.data, self.resp.size, self.resp_off.ctypes.data, self.consumed.ctypes.data,
                        self.stop.ctypes.data, 0, 0, 0)
        return b, o

    def finish(self, o):
        self.n_frames, self.n_requests, self.n_responses = o.n_frames, o.n_requests, o.n_responses
        self.resp = self.resp[: int(self.resp_off[-1])]
        return self

    def responses(self, s):
        return bytes(self.resp[int(self.resp_off[s]): int(self.resp_off[s + 1])])


# ---- DegradeSlot circuit breakers (include/sentinel_flow.h, sf_degrade_*) ----
V_BLOCK_DEGRADE = 8
V_BLOCK_OTHER = 9            # SF_EV_BLOCKED entry: counted as a block by StatisticSlot, no check ran
DEGRADE_GRADE_RT, DEGRADE_GRADE_EXCEPTION_RATIO, DEGRADE_GRADE_EXCEPTION_COUNT = 0, 1, 2
CB_CLOSED, CB_OPEN, CB_HALF_OPEN = 0, 1, 2


class sf_degrade_rule(C.Structure):
    _fields_ = [("resource", C.c_uint32), ("grade", C.c_int32), ("count", C.c_double),
                ("time_window_s", C.c_int32), ("min_request_amount", C.c_int32),
                ("slow_ratio_threshold", C.c_double), ("stat_interval_ms", C.c_int32), ("pad", C.c_int32)]


class sf_breaker_state(C.Structure):
    _fields_ = [("state", C.c_int32), ("pad", C.c_int32), ("next_retry_ms", C.c_int64),
                ("window_start", C.c_int64), ("hit_count", C.c_int64), ("total_count", C.c_int64)]


def degrade_rule(resource, grade, count, time_window_s, min_request_amount=5, slow_ratio_threshold=1.0,
                 stat_interval_ms=1000) -> dict:
    """DegradeRule with the reference defaults (DegradeRule.java: minRequestAmount 5,
    slowRatioThreshold 1.0, statIntervalMs 1000)."""
    return dict(resource=resource, grade=grade, count=float(count), time_window_s=time_window_s,
                min_request_amount=min_request_amount, slow_ratio_threshold=float(slow_ratio_threshold),
                stat_interval_ms=stat_interval_ms)


DEGRADE_RULE_DTYPE = np.dtype([(n, {C.c_uint32: "<u4", C.c_int32: "<i4", C.c_double: "<f8"}[t])
                               for n, t in sf_degrade_rule._fields_])
assert DEGRADE_RULE_DTYPE.itemsize == C.sizeof(sf_degrade_rule)

STRUCT_SIZES.update({"sf_degrade_rule": C.sizeof(sf_degrade_rule), "sf_breaker_state": C.sizeof(sf_breaker_state)})
