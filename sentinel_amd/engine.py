"""Python binding of the HIP engine (``libsentinel_flow.so``) through its C-ABI.

This is the host-side mirror of the reference's operator interfaces for the
hot path: ``FlowEngine.submit`` plays ``ProcessorSlot.entry/exit`` for a batch
of events (StatisticSlot + SystemSlot + ParamFlowSlot + FlowSlot), and
``FlowEngine.request_tokens`` plays ``TokenService.requestToken``.

There is no CPU fallback: importing works without a GPU (the library links
the HIP runtime lazily), but ``FlowEngine(...)`` raises ``EngineError`` unless
a gfx950 device is visible.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
# SENTINEL_FLOW_LIB selects a diagnostics build (e.g. libsentinel_flow_prof.so); default: the product library
LIB_PATH = os.environ.get("SENTINEL_FLOW_LIB") or os.path.join(_HERE, "libsentinel_flow.so")


# sf_allgather_fn: (ctx, send, recv, bytes) -> 0 on success
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64)


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"sentinel_flow error {code}: {msg}")
        self.code = code


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        _declare(L)
        _lib = L
    return _lib


P = C.c_void_p


def _declare(L):
    def f(name, res, *args):
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = list(args)
    I, U32 = C.c_int, C.c_uint32
    f("sf_abi_version", I)
    f("sf_config_default", None, C.POINTER(abi.sf_config))
    f("sf_create", I, C.POINTER(abi.sf_config), C.POINTER(P))
    f("sf_destroy", None, P)
    f("sf_last_error", C.c_char_p)
    f("sf_load_flow_rules", I, P, C.POINTER(abi.sf_flow_rule), U32)
    f("sf_load_param_rules", I, P, C.POINTER(abi.sf_param_rule), U32, C.POINTER(abi.sf_hot_item), U32)
    f("sf_load_system_rules", I, P, C.POINTER(abi.sf_system_rule), U32)
    f("sf_set_system_status", I, P, C.c_double, C.c_double)
    f("sf_submit", I, P, C.POINTER(abi.sf_event_batch), C.POINTER(abi.sf_verdicts))
    f("sf_submit_async", I, P, C.POINTER(abi.sf_event_batch), C.POINTER(abi.sf_verdicts))
    f("sf_submit_packed", I, P, C.POINTER(abi.sf_packed_batch), C.POINTER(abi.sf_verdicts))
    f("sf_submit_packed_async", I, P, C.POINTER(abi.sf_packed_batch), C.POINTER(abi.sf_verdicts))
    f("sf_sync_packed", I, P, C.POINTER(abi.sf_verdicts))
    f("sf_submit_packed_sparse_async", I, P, C.POINTER(abi.sf_packed_batch), C.POINTER(abi.sf_sparse_verdicts))
    f("sf_sync_packed_sparse", I, P, C.POINTER(abi.sf_sparse_verdicts))
    f("sf_load_namespaces", I, P, C.POINTER(abi.sf_namespace), U32)
    f("sf_load_cluster_rules", I, P, C.POINTER(abi.sf_cluster_flow_rule), U32,
      C.POINTER(abi.sf_cluster_param_rule), U32, C.POINTER(abi.sf_hot_item), U32)
    f("sf_request_tokens", I, P, C.POINTER(abi.sf_token_batch), C.POINTER(abi.sf_token_results))
    f("sf_serve_frames", I, P, C.POINTER(abi.sf_wire_batch), C.POINTER(abi.sf_wire_out))
    f("sf_string_key", C.c_uint64, C.c_char_p, C.c_uint32)
    f("sf_cluster_sum", I, P, C.c_int64, I, C.c_int64, C.POINTER(C.c_int64))
    f("sf_comm_unique_id", I, C.c_char_p, C.c_size_t)
    f("sf_comm_init", I, P, I, I, C.c_char_p, C.c_size_t)
    f("sf_entry_node_allreduce", I, P, C.POINTER(abi.sf_node_state))
    f("sf_set_report_entry_node", I, P, C.POINTER(abi.sf_node_state))
    f("sf_read_node", I, P, U32, C.POINTER(abi.sf_node_state))
    f("sf_read_entry_node", I, P, C.POINTER(abi.sf_node_state))
    f("sf_read_rule_state", I, P, U32, C.POINTER(abi.sf_rule_state))
    f("sf_node_digests", I, P, P, U32)
    f("sf_read_rule_states", I, P, U32, U32, P)
    f("sf_read_origin_node", I, P, U32, U32, C.POINTER(abi.sf_node_state))
    f("sf_read_context_node", I, P, U32, U32, C.POINTER(abi.sf_node_state))
    f("sf_load_degrade_rules", I, P, C.POINTER(abi.sf_degrade_rule), U32, C.POINTER(U32))
    f("sf_degrade_submit", I, P, C.POINTER(abi.sf_event_batch), C.POINTER(abi.sf_verdicts))
    f("sf_read_breaker", I, P, U32, C.POINTER(abi.sf_breaker_state))
    f("sf_snapshot", I, P, C.c_int64, C.POINTER(abi.sf_metric_row), U32, C.POINTER(U32))
    f("sf_load_resource_names", I, P, C.c_char_p, C.POINTER(C.c_uint64), C.POINTER(C.c_int32), U32)
    f("sf_metric_log", I, P, C.c_int64, C.c_int64, I, C.c_char_p, C.c_uint64, C.POINTER(C.c_uint64),
      C.POINTER(U32))
    f("sf_format_metric_rows", I, P, C.POINTER(abi.sf_metric_row), U32, C.c_int64, C.c_char_p, C.c_uint64,
      C.POINTER(C.c_uint64))
    f("sf_device_alloc", I, P, C.c_size_t, C.POINTER(P))
    f("sf_device_free", I, P, P)
    f("sf_host_alloc", I, P, C.c_size_t, C.POINTER(P))
    f("sf_host_free", I, P, P)
    f("sf_memcpy", I, P, P, P, C.c_size_t, I)
    f("sf_sync", I, P)
    f("sf_get_stats", I, P, C.POINTER(abi.sf_stats))
    f("sf_set_timing", I, P, I)
    f("sf_heavy_profile_read", I, P, C.POINTER(abi.sf_heavy_profile), U32, C.POINTER(U32))
    f("sf_param_table_stats", I, P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(U32))
    f("sf_read_param_thread", I, P, U32, C.c_int, C.c_uint8, C.c_uint64, C.POINTER(C.c_int64))
    f("sf_token_shard", I, C.POINTER(abi.sf_cluster_flow_rule), U32, C.POINTER(abi.sf_cluster_param_rule), U32,
      C.POINTER(abi.sf_namespace), U32, U32, P, P, U32, P)
    f("sf_system_plan", I, P, C.POINTER(abi.sf_event_batch), P, U32, C.POINTER(U32), P)
    f("sf_submit_forced", I, P, C.POINTER(abi.sf_event_batch), C.POINTER(abi.sf_verdicts), P)
    f("sf_entry_node_add", I, P, C.POINTER(abi.sf_event_batch), P)
    f("sf_submit_node", I, P, C.POINTER(abi.sf_event_batch), P, C.POINTER(abi.sf_verdicts), ALLGATHER_FN, P)
    f("sf_flow_rule_order", I, C.POINTER(abi.sf_flow_rule), C.POINTER(abi.sf_rule_key), U32, P, C.POINTER(U32))
    f("sf_param_rule_order", I, C.POINTER(abi.sf_param_rule), C.POINTER(abi.sf_rule_key), U32,
      C.POINTER(abi.sf_hot_item), U32, P, C.POINTER(U32))


def flow_rule_order(rules, keys) -> np.ndarray:
    """Indices of ``rules`` in the order FlowRuleManager holds them (invalid
    and duplicate rules dropped; sf_flow_rule_order, host only)."""
    n = len(rules)
    out, m = np.zeros(max(n, 1), np.uint32), C.c_uint32(0)
    _check(lib().sf_flow_rule_order(abi.rules_array(abi.sf_flow_rule, list(rules)),
                                    abi.rules_array(abi.sf_rule_key, list(keys)), n, out.ctypes.data, C.byref(m)))
    return out[:m.value].copy()


def param_rule_order(rules, keys, items=()) -> np.ndarray:
    """Indices of ``rules`` in the order ParamFlowRuleManager holds them
    (sf_param_rule_order, host only)."""
    n = len(rules)
    out, m = np.zeros(max(n, 1), np.uint32), C.c_uint32(0)
    _check(lib().sf_param_rule_order(abi.rules_array(abi.sf_param_rule, list(rules)),
                                     abi.rules_array(abi.sf_rule_key, list(keys)), n,
                                     abi.rules_array(abi.sf_hot_item, list(items)), len(items),
                                     out.ctypes.data, C.byref(m)))
    return out[:m.value].copy()


def token_shard(flow, param, namespaces, shard_count: int, batch: abi.HostTokenBatch) -> np.ndarray:
    """Owner shard of every request of ``batch`` on a token server sharded
    over ``shard_count`` GPUs (sf_token_shard: host only, no GPU needed)."""
    out = np.zeros(batch.n, np.uint32)
    _check(lib().sf_token_shard(abi.rules_array(abi.sf_cluster_flow_rule, list(flow)), len(flow),
                                abi.rules_array(abi.sf_cluster_param_rule, list(param)), len(param),
                                abi.rules_array(abi.sf_namespace, list(namespaces)), len(namespaces), shard_count,
                                batch.flow_id.ctypes.data, batch.flags.ctypes.data, batch.n, out.ctypes.data))
    return out


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id (rank 0), to be distributed to every rank."""
    buf = C.create_string_buffer(128)
    _check(lib().sf_comm_unique_id(buf, 128))
    return buf.raw


def _check(rc):
    if rc != 0:
        raise EngineError(rc, lib().sf_last_error().decode(errors="replace"))


class DeviceArray:
    """A device (HBM) buffer owned by an engine, filled from a numpy array."""

    def __init__(self, eng: "FlowEngine", host: np.ndarray):
        self.eng = eng
        self.dtype = host.dtype
        self.shape = host.shape
        self.nbytes = host.nbytes
        p = P()
        _check(lib().sf_device_alloc(eng.h, max(16, self.nbytes), C.byref(p)))
        self.ptr = p.value
        if self.nbytes:
            _check(lib().sf_memcpy(eng.h, self.ptr, host.ctypes.data, self.nbytes, 0))

    @classmethod
    def empty(cls, eng, shape, dtype):
        return cls(eng, np.zeros(shape, dtype))

    def numpy(self) -> np.ndarray:
        out = np.empty(self.shape, self.dtype)
        if self.nbytes:
            _check(lib().sf_memcpy(self.eng.h, out.ctypes.data, self.ptr, self.nbytes, 1))
        return out

    def free(self):
        if self.ptr:
            lib().sf_device_free(self.eng.h, self.ptr)
            self.ptr = None


class PinnedArrays:
    """numpy arrays in page-locked host memory (sf_host_alloc), freed together."""

    def __init__(self, eng: "FlowEngine"):
        self.eng, self.ptrs = eng, []

    def array(self, shape, dtype, fill=None) -> np.ndarray:
        dtype = np.dtype(dtype)
        n = int(np.prod(shape)) * dtype.itemsize
        p = P()
        _check(lib().sf_host_alloc(self.eng.h, max(16, n), C.byref(p)))
        self.ptrs.append(p.value)
        a = np.ctypeslib.as_array((C.c_uint8 * max(16, n)).from_address(p.value))[:n].view(dtype).reshape(shape)
        if fill is not None:
            a[...] = fill
        return a

    def batch(self, hb: abi.HostBatch) -> abi.HostBatch:
        """A copy of hb (res, ts, count, flags, entry_ref, create_ts) in pinned memory."""
        def cp(x):
            return None if x is None else self.array(x.shape, x.dtype, x)
        return abi.HostBatch(cp(hb.res_id), cp(hb.ts_ms), cp(hb.count), cp(hb.flags), entry_ref=cp(hb.entry_ref),
                             create_ts=cp(hb.create_ts))

    def verdicts(self, n: int, with_wait=True, with_rule=True) -> abi.HostVerdicts:
        v = abi.HostVerdicts(n)
        v.status = self.array((n,), np.uint8)
        v.wait_ms = self.array((n,), np.int32) if with_wait else None
        v.rule_idx = self.array((n,), np.uint16) if with_rule else None
        return v

    def sparse_verdicts(self, n: int, prefetch: int) -> abi.HostSparseVerdicts:
        return abi.HostSparseVerdicts(n, prefetch, alloc=self.array)

    def free(self):
        for p in self.ptrs:
            lib().sf_host_free(self.eng.h, p)
        self.ptrs = []


class DeviceBatch:
    """An event batch resident in HBM (inputs already on the GPU)."""

    def __init__(self, eng: "FlowEngine", hb: abi.HostBatch):
        self.n = hb.n
        self.arrays = {k: DeviceArray(eng, getattr(hb, k)) for k in ("res_id", "ts_ms", "count", "flags")}
        for k in ("entry_ref", "create_ts", "arg_tag", "arg_bits", "n_args", "elem_off", "elem_tag", "elem_bits",
                  "origin", "context"):
            a = getattr(hb, k)
            self.arrays[k] = DeviceArray(eng, a) if a is not None else None
        self.arg_slots = 0 if hb.arg_tag is None else hb.arg_tag.shape[0]

    @classmethod
    def with_ts(cls, eng: "FlowEngine", base: "DeviceBatch", ts_ms: np.ndarray) -> "DeviceBatch":
        """The events of ``base`` at other times: only the timestamps are
        uploaded, every other array is shared with ``base`` (free() frees only
        the timestamps)."""
        self = cls.__new__(cls)
        self.n = base.n
        self.arg_slots = base.arg_slots
        self.arrays = dict(base.arrays)
        self.arrays["ts_ms"] = DeviceArray(eng, np.ascontiguousarray(ts_ms, dtype=np.int64))
        self._owned = ("ts_ms",)
        return self

    def c_struct(self) -> abi.sf_event_batch:
        b = abi.sf_event_batch()
        b.n, b.mem = self.n, abi.MEM_DEVICE
        g = lambda k: None if self.arrays[k] is None else self.arrays[k].ptr  # noqa: E731
        b.res_id, b.ts_ms, b.count, b.flags = g("res_id"), g("ts_ms"), g("count"), g("flags")
        b.entry_ref, b.create_ts = g("entry_ref"), g("create_ts")
        b.arg_slots = self.arg_slots
        b.arg_tag, b.arg_bits, b.n_args = g("arg_tag"), g("arg_bits"), g("n_args")
        if self.arrays.get("elem_off") is not None:
            b.arg_elem_off, b.elem_tag, b.elem_bits = g("elem_off"), g("elem_tag"), g("elem_bits")
            b.n_elems = self.arrays["elem_tag"].shape[0]
        b.origin, b.context = g("origin"), g("context")
        return b

    def free(self):
        owned = getattr(self, "_owned", None)
        for k, a in self.arrays.items():
            if a is not None and (owned is None or k in owned):
                a.free()


class DeviceVerdicts:
    def __init__(self, eng: "FlowEngine", n: int, with_wait=True, with_rule=False):
        self.status = DeviceArray.empty(eng, n, np.uint8)
        self.wait_ms = DeviceArray.empty(eng, n, np.int32) if with_wait else None
        self.rule_idx = DeviceArray.empty(eng, n, np.uint16) if with_rule else None

    def c_struct(self) -> abi.sf_verdicts:
        v = abi.sf_verdicts()
        v.mem = abi.MEM_DEVICE
        v.status = self.status.ptr
        v.wait_ms = self.wait_ms.ptr if self.wait_ms else None
        v.rule_idx = self.rule_idx.ptr if self.rule_idx else None
        return v

    def free(self):
        for a in (self.status, self.wait_ms, self.rule_idx):
            if a is not None:
                a.free()


class FlowEngine:
    """One GPU's flow-check engine (sf_create .. sf_destroy)."""

    def __init__(self, cfg: abi.sf_config):
        self.cfg = cfg
        h = P()
        _check(lib().sf_create(C.byref(cfg), C.byref(h)))
        self.h = h.value

    def close(self):
        if getattr(self, "h", None):
            lib().sf_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_flow_rules(self, rules):
        ptr, n = abi.flow_rules_ptr(rules)
        _check(lib().sf_load_flow_rules(self.h, ptr, n))

    def load_param_rules(self, rules, items=()):
        _check(lib().sf_load_param_rules(self.h, abi.rules_array(abi.sf_param_rule, rules), len(rules),
                                         abi.rules_array(abi.sf_hot_item, list(items)), len(items)))

    def load_system_rules(self, rules):
        _check(lib().sf_load_system_rules(self.h, abi.rules_array(abi.sf_system_rule, rules), len(rules)))

    def set_system_status(self, load, cpu):
        _check(lib().sf_set_system_status(self.h, load, cpu))

    def submit(self, batch: abi.HostBatch, out: abi.HostVerdicts = None) -> abi.HostVerdicts:
        out = abi.HostVerdicts(batch.n) if out is None else out
        b = batch.c_struct()
        v = out.c_struct()
        _check(lib().sf_submit(self.h, C.byref(b), C.byref(v)))
        return out

    def submit_packed(self, batch: abi.PackedBatch, out: abi.HostVerdicts = None) -> abi.HostVerdicts:
        """sf_submit_packed: the compact 8-B-per-event form from host memory."""
        out = abi.HostVerdicts(batch.n) if out is None else out
        b, v = batch.c_struct(), out.c_struct()
        _check(lib().sf_submit_packed(self.h, C.byref(b), C.byref(v)))
        return out

    def submit_packed_async(self, batch: abi.PackedBatch, out: abi.HostVerdicts):
        """sf_submit_packed_async: enqueued; H2D of this batch overlaps the decision of the
        previous one and the copy back of the one before.  Arrays stay untouched until sync()."""
        b, v = batch.c_struct(), out.c_struct()
        _check(lib().sf_submit_packed_async(self.h, C.byref(b), C.byref(v)))

    def sync_packed(self, out: abi.HostVerdicts):
        """sf_sync_packed: waits for the one async packed batch whose verdicts go to `out`
        (the batch enqueued after it keeps running); raises that batch's error."""
        v = out.c_struct()
        _check(lib().sf_sync_packed(self.h, C.byref(v)))

    def submit_packed_sparse_async(self, batch: abi.PackedBatch, out: abi.HostSparseVerdicts):
        """sf_submit_packed_sparse_async: as submit_packed_async, the verdicts copied back
        sparse (1 B per event plus the nonzero waits / rule indices)."""
        b, v = batch.c_struct(), out.c_struct()
        _check(lib().sf_submit_packed_sparse_async(self.h, C.byref(b), C.byref(v)))

    def sync_packed_sparse(self, out: abi.HostSparseVerdicts):
        v = out.c_struct()
        _check(lib().sf_sync_packed_sparse(self.h, C.byref(v)))

    def submit_device(self, batch: DeviceBatch, out: DeviceVerdicts):
        b = batch.c_struct()
        v = out.c_struct()
        _check(lib().sf_submit(self.h, C.byref(b), C.byref(v)))

    # ---- node-wide SystemRule rounds of a sharded node (sentinel_flow.h; system_shard.py)
    def system_plan(self, merged: abi.HostBatch, status: np.ndarray, p: int, sys_mask: np.ndarray) -> int:
        """Plans merged[p, q) (the node's IN events; status = verdicts of
        merged[0, p)); fills sys_mask[p:q], returns q."""
        assert sys_mask.dtype == np.uint8 and sys_mask.shape == (merged.n,)
        st = np.ascontiguousarray(status, np.uint8)
        b = merged.c_struct()
        q = C.c_uint32(0)
        _check(lib().sf_system_plan(self.h, C.byref(b), st.ctypes.data if p else None, p, C.byref(q),
                                    sys_mask.ctypes.data))
        return int(q.value)

    def submit_forced(self, batch: abi.HostBatch, sys_mask: np.ndarray) -> abi.HostVerdicts:
        """A (sub-)batch whose SystemRule verdicts were planned node-wide."""
        m = np.ascontiguousarray(sys_mask, np.uint8)
        assert m.shape == (batch.n,)
        out = abi.HostVerdicts(batch.n)
        b = batch.c_struct()
        v = out.c_struct()
        _check(lib().sf_submit_forced(self.h, C.byref(b), C.byref(v), m.ctypes.data))
        return out

    def entry_node_add(self, batch: abi.HostBatch, status: np.ndarray):
        """ENTRY_NODE update with decided IN events of the node."""
        st = np.ascontiguousarray(status, np.uint8)
        assert st.shape == (batch.n,)
        b = batch.c_struct()
        _check(lib().sf_entry_node_add(self.h, C.byref(b), st.ctypes.data))

    def submit_node(self, batch: abi.HostBatch, seq: np.ndarray, comm=None) -> abi.HostVerdicts:
        """sf_submit_node: this rank's shard of a node batch (``seq`` = the
        events' global sequence numbers) with the node-wide SystemRule
        semantics, by the per-window exchange (sf_sysx.h).  ``comm``: an object
        with ``allgather_bytes(np.uint8 array) -> [rank 0's bytes, rank 1's,
        ...]`` (e.g. system_shard.TorchComm over gloo), or None for the
        engine's RCCL communicator (sf_comm_init).  Raises EngineError with
        code SF_ERR_UNSUPPORTED on every rank alike when the SystemRules need
        the event all-gather protocol."""
        out = abi.HostVerdicts(batch.n)
        b, v = batch.c_struct(), out.c_struct()
        sq = np.ascontiguousarray(seq, np.int64)
        assert sq.shape == (batch.n,)
        errs = []
        if comm is None:
            cb = ALLGATHER_FN()
        else:
            def fn(ctx, send, recv, nbytes):
                try:
                    x = np.ctypeslib.as_array(C.cast(send, C.POINTER(C.c_uint8)), shape=(nbytes,))
                    off = 0
                    for p in comm.allgather_bytes(x):
                        p = np.ascontiguousarray(p, np.uint8).reshape(-1)
                        assert p.nbytes == nbytes
                        C.memmove(recv + off, p.ctypes.data, nbytes)
                        off += nbytes
                    return 0
                except BaseException as ex:          # noqa: BLE001 -- re-raised after the call
                    errs.append(ex)
                    return 1
            cb = ALLGATHER_FN(fn)
        rc = lib().sf_submit_node(self.h, C.byref(b), sq.ctypes.data if batch.n else None, C.byref(v), cb, None)
        if errs:
            raise errs[0]
        _check(rc)
        return out

    def submit_device_async(self, batch: DeviceBatch, out: DeviceVerdicts):
        """Enqueue a batch (HBM arrays; keep them alive until sync()): batch k+1 is
        sorted while batch k is decided; sync() waits and reports errors."""
        b = batch.c_struct()
        v = out.c_struct()
        _check(lib().sf_submit_async(self.h, C.byref(b), C.byref(v)))

    def read_node(self, res) -> abi.sf_node_state:
        st = abi.sf_node_state()
        _check(lib().sf_read_node(self.h, res, C.byref(st)))
        return st

    def read_origin_node(self, res, origin) -> abi.sf_node_state:
        """Origin node of (res, origin) (ClusterNode.getOrCreateOriginNode), if the engine keeps it."""
        st = abi.sf_node_state()
        _check(lib().sf_read_origin_node(self.h, res, origin, C.byref(st)))
        return st

    def read_context_node(self, context, res) -> abi.sf_node_state:
        """DefaultNode of (context, res) (NodeSelectorSlot), if the engine keeps it."""
        st = abi.sf_node_state()
        _check(lib().sf_read_context_node(self.h, context, res, C.byref(st)))
        return st

    has_entry_node = True

    def read_entry_node(self) -> abi.sf_node_state:
        st = abi.sf_node_state()
        _check(lib().sf_read_entry_node(self.h, C.byref(st)))
        return st

    def comm_init(self, nranks: int, rank: int, unique_id: bytes):
        """Join the node's RCCL communicator (one engine per GPU)."""
        _check(lib().sf_comm_init(self.h, nranks, rank, unique_id, len(unique_id)))

    def entry_node_allreduce(self) -> abi.sf_node_state:
        """Node-wide ENTRY_NODE merged over all ranks with RCCL (exact; see sentinel_amd/dist.py)."""
        st = abi.sf_node_state()
        _check(lib().sf_entry_node_allreduce(self.h, C.byref(st)))
        return st

    def set_report_entry_node(self, node: abi.sf_node_state = None):
        """The ENTRY_NODE metric_log reports (None: this engine's own)."""
        _check(lib().sf_set_report_entry_node(self.h, None if node is None else C.byref(node)))

    def snapshot(self, now, cap=1 << 20):
        """StatisticNode.metrics() of every node (MetricTimerListener): MetricNode rows."""
        rows = (abi.sf_metric_row * cap)()
        n = C.c_uint32()
        _check(lib().sf_snapshot(self.h, now, rows, cap, C.byref(n)))
        return [rows[i] for i in range(n.value)]

    def load_resource_names(self, names, types=None):
        """ResourceWrapper names (and ResourceTypeConstants) by global resource id, for metrics.log."""
        enc = [n.encode() if isinstance(n, str) else bytes(n) for n in names]
        off = np.zeros(len(enc) + 1, np.uint64)
        off[1:] = np.cumsum([len(x) for x in enc], dtype=np.uint64)
        data = b"".join(enc)
        ty = None if types is None else np.ascontiguousarray(types, dtype=np.int32)
        _check(lib().sf_load_resource_names(self.h, data, off.ctypes.data_as(C.POINTER(C.c_uint64)),
                                            None if ty is None else ty.ctypes.data_as(C.POINTER(C.c_int32)),
                                            len(enc)))

    def load_resource_names_raw(self, data: bytes, offsets, types=None):
        """Names as one byte string and n+1 offsets (uint64)."""
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ty = None if types is None else np.ascontiguousarray(types, dtype=np.int32)
        _check(lib().sf_load_resource_names(self.h, data, off.ctypes.data_as(C.POINTER(C.c_uint64)),
                                            None if ty is None else ty.ctypes.data_as(C.POINTER(C.c_int32)),
                                            off.shape[0] - 1))

    def metric_log(self, now, tz_offset_ms=0, entry_node=True, cap=1 << 24, buf=None) -> bytes:
        """One MetricTimerListener.run at ``now``: the metrics.log bytes MetricWriter appends
        (``buf``: a reusable ctypes char buffer of at least ``cap`` bytes)."""
        if buf is None or len(buf) < cap:
            buf = C.create_string_buffer(max(1, cap))
        n, k = C.c_uint64(), C.c_uint32()
        _check(lib().sf_metric_log(self.h, now, tz_offset_ms, int(entry_node), buf, cap, C.byref(n), C.byref(k)))
        return buf.raw[:n.value]

    def format_metric_rows(self, rows, tz_offset_ms=0) -> bytes:
        """MetricNode.toFatString of the given rows, formatted on the GPU."""
        arr = (abi.sf_metric_row * max(1, len(rows)))(*rows)
        cap = 256 * max(1, len(rows)) + (1 << 16)
        buf = C.create_string_buffer(cap)
        n = C.c_uint64()
        _check(lib().sf_format_metric_rows(self.h, arr, len(rows), tz_offset_ms, buf, cap, C.byref(n)))
        return buf.raw[:n.value]

    # ---- DegradeSlot circuit breakers (DegradeSlot.java:50-94) ----
    def load_degrade_rules(self, rules) -> int:
        """rules: dicts of sf_degrade_rule fields (abi.degrade_rule), or a numpy
        array of abi.DEGRADE_RULE_DTYPE; returns breakers installed."""
        if isinstance(rules, np.ndarray):
            assert rules.dtype == abi.DEGRADE_RULE_DTYPE
            rules = np.ascontiguousarray(rules)
            arr = C.cast(rules.ctypes.data, C.POINTER(abi.sf_degrade_rule))
        else:
            arr = (abi.sf_degrade_rule * max(1, len(rules)))()
            for i, r in enumerate(rules):
                for k, v in r.items():
                    setattr(arr[i], k, v)
        n = C.c_uint32(0)
        _check(lib().sf_load_degrade_rules(self.h, arr, len(rules), C.byref(n)))
        return n.value

    def degrade_submit(self, batch: abi.HostBatch) -> abi.HostVerdicts:
        out = abi.HostVerdicts(batch.n)
        b = batch.c_struct()
        v = out.c_struct()
        _check(lib().sf_degrade_submit(self.h, C.byref(b), C.byref(v)))
        return out

    def degrade_submit_device(self, batch: DeviceBatch, out: DeviceVerdicts):
        b = batch.c_struct()
        v = out.c_struct()
        _check(lib().sf_degrade_submit(self.h, C.byref(b), C.byref(v)))

    def read_breaker(self, idx) -> dict:
        s = abi.sf_breaker_state()
        _check(lib().sf_read_breaker(self.h, idx, C.byref(s)))
        ws = None if s.window_start == abi.SF_WS_ABSENT else s.window_start
        return dict(state=s.state, next_retry_ms=s.next_retry_ms, window_start=ws, hit_count=s.hit_count,
                    total_count=s.total_count)

    def read_rule_state(self, idx) -> abi.sf_rule_state:
        s = abi.sf_rule_state()
        _check(lib().sf_read_rule_state(self.h, idx, C.byref(s)))
        return s

    def node_digests(self, n_rows=None) -> np.ndarray:
        """One FNV-1a 64 digest per local row's canonical node state (sf_node_digests)."""
        n = self.cfg.max_resources if n_rows is None else n_rows
        out = np.empty(n, np.uint64)
        _check(lib().sf_node_digests(self.h, out.ctypes.data, n))
        return out

    def rule_states(self, first=0, n=None) -> np.ndarray:
        """(n, 3) int64 stored_tokens, last_filled_time, latest_passed_time (sf_read_rule_states)."""
        out = np.empty((n, 3), np.int64)
        _check(lib().sf_read_rule_states(self.h, first, n, out.ctypes.data))
        return out

    def param_table_stats(self) -> dict:
        """Exact hot-parameter table: occupied slots, capacity, load factor, longest probe."""
        u, c, m = C.c_uint64(), C.c_uint64(), C.c_uint32()
        _check(lib().sf_param_table_stats(self.h, C.byref(u), C.byref(c), C.byref(m)))
        return dict(used=u.value, capacity=c.value, load_factor=round(u.value / max(1, c.value), 4),
                    max_probe=m.value)

    def param_thread(self, res, idx, value) -> int:
        """ParameterMetric.getThreadCount(idx, value) of resource ``res``; value = (tag, bits)."""
        out = C.c_int64()
        _check(lib().sf_read_param_thread(self.h, res, idx, value[0], value[1], C.byref(out)))
        return out.value

    def set_timing(self, on=True):
        _check(lib().sf_set_timing(self.h, int(on)))

    def stats(self) -> abi.sf_stats:
        s = abi.sf_stats()
        _check(lib().sf_get_stats(self.h, C.byref(s)))
        return s

    def heavy_profile(self, cap=1 << 20):
        """Per heavy segment of the last submit: (resource, events, mode, microseconds, start microseconds);
        start is relative to the first k_heavy_stream segment (0 for k_heavy_decide segments)."""
        buf = (abi.sf_heavy_profile * cap)()
        n = C.c_uint32()
        _check(lib().sf_heavy_profile_read(self.h, buf, cap, C.byref(n)))
        return [(b.resource, b.events, b.mode, b.ticks / 100.0, b.start / 100.0) for b in buf[:n.value]]

    # ---- cluster token server (TokenService.requestToken / requestParamToken)
    def load_namespaces(self, ns):
        _check(lib().sf_load_namespaces(self.h, abi.rules_array(abi.sf_namespace, list(ns)), len(ns)))

    def load_cluster_rules(self, flow=(), param=(), items=()):
        _check(lib().sf_load_cluster_rules(self.h, abi.rules_array(abi.sf_cluster_flow_rule, list(flow)), len(flow),
                                           abi.rules_array(abi.sf_cluster_param_rule, list(param)), len(param),
                                           abi.rules_array(abi.sf_hot_item, list(items)), len(items)))

    def request_tokens(self, batch: abi.HostTokenBatch) -> abi.HostTokenResults:
        out = abi.HostTokenResults(batch.n)
        b = batch.c_struct()
        r = out.c_struct()
        _check(lib().sf_request_tokens(self.h, C.byref(b), C.byref(r)))
        return out

    def serve_frames(self, streams, now_ms) -> abi.WireResult:
        """Inbound C1 bytes of each connection -> response frames (sf_serve_frames)."""
        r = abi.WireResult(streams, now_ms)
        b, o = r.c_structs()
        _check(lib().sf_serve_frames(self.h, C.byref(b), C.byref(o)))
        return r.finish(o)

    def cluster_sum(self, flow_id, event, now):
        v = C.c_int64()
        _check(lib().sf_cluster_sum(self.h, flow_id, event, now, C.byref(v)))
        return v.value

    def sync(self):
        _check(lib().sf_sync(self.h))
