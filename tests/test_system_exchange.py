"""SystemRules on a resource-sharded node, the per-window exchange
(sentinel_amd/csrc/sf_sysx.h, sf_submit_node).

CPU: the protocol restated over oracle engines (tests/sysx_sim.py) on two
ranks -- threads of this process and a gloo world of two processes -- equals
one replay of the whole node batch: every verdict and every rank's ENTRY_NODE
(SystemRuleManager.checkSystem, SystemRuleManager.java:291-348).  The
product's plan step (sx_reduce, host build in tests/hostsim) equals the
restatement's on random messages.  GPU: two engines deciding their shards
through sf_submit_node (threads, LocalComm) equal the oracle's one replay,
with the inert entries of ParamFlow workloads, exits, mixed acquireCounts,
another window geometry, pipelined batches, and the fallback to the event
all-gather protocol for a thread rule."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from sentinel_amd import abi, system_shard, trace
from tests import sysx_sim, workloads
from tests.test_system_shard import _load, _merge


def _qps_rule(q):
    return [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=float(q), avg_rt=-1, max_thread=-1)]


def exchange_workload(kind, n=8000):
    """(w, batches) of an eligible SystemRule: "param" = config 4's shape, inbound QPS at 0.6x;
    "mixed" = config 3's traffic (exits, acquireCount 1-5, all controllers) with inbound QPS;
    "cpu" = QPS + a CPU threshold that fires; "geom" = "mixed" on 1 bucket of 1500 ms."""
    if kind == "param":
        rules, b = trace.param_zipf(60, n, 2000, duration_ms=2000, seed=17)
        w = dict(cfg=abi.default_config(max_resources=60, max_batch=b.n, param_capacity=1 << 16), param=rules,
                 system=_qps_rule(0.6 * n / 2.0), status=(0.0, 0.0))
        return w, [b.subset(0, n // 2), b.subset(n // 2, n)]
    R = 80
    full = trace.mixed_zipf(R, n, duration_ms=3000, seed=19)
    cfg = abi.default_config(max_resources=R, max_batch=full.n)
    if kind == "geom":
        cfg = abi.default_config(max_resources=R, max_batch=full.n, sample_count=1, interval_ms=1500)
    sysr = _qps_rule(0.45 * n / 3.0)
    status = (0.0, 0.0)
    if kind == "cpu":
        sysr = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=0.6, qps=0.5 * n / 3.0, avg_rt=-1,
                                   max_thread=-1)]
        status = (0.3, 0.9)
    w = dict(cfg=cfg, flow=trace.mixed_rules(R, seed=19), system=sysr, status=status)
    cuts = np.linspace(0, full.n, 3).astype(int)
    return w, [full.subset(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:])]


def _geometry(w):
    c = w["cfg"]
    r = w["system"][0]
    return dict(S=c.sample_count, interval=c.interval_ms, qps=min(x.qps for x in w["system"] if x.qps >= 0),
                cpu_fires=any(x.highest_cpu_usage >= 0 for x in w["system"]) and w["status"][1] > r.highest_cpu_usage)


def _rank_cfg(w, batches, world, rank):
    c = w["cfg"]
    return abi.default_config(max_resources=(c.max_resources + world - 1) // world,
                              max_batch=max(b.n for b in batches), shard_count=world, shard_index=rank,
                              param_capacity=c.param_capacity, sample_count=c.sample_count,
                              interval_ms=c.interval_ms)


def _sim_rank(w, batches, world, rank, comm, log=None):
    from oracle import oracle as so
    cfg = _rank_cfg(w, batches, world, rank)
    o = so.OracleEngine(cfg)
    _load(o, w, world, rank)
    pos, cols, off = [], [], 0
    for b in batches:
        sel = np.nonzero(b.res_id % world == rank)[0]
        st = {}
        v = sysx_sim.submit_node_windows(o, b.shard(world, rank), sel + off, comm, stats_out=st, **_geometry(w))
        if log is not None:
            log.append(st)
        pos.append(sel + off)
        cols.append(np.stack([v.status, v.wait_ms, v.rule_idx]).astype(np.int64))
        off += b.n
    return np.concatenate(pos), np.concatenate(cols, axis=1), abi.node_state_to_dict(o.read_entry_node(),
                                                                                      cfg.sample_count)


def _reference(w, batches):
    from oracle import oracle as so
    c = w["cfg"]
    cfg = abi.default_config(max_resources=c.max_resources, max_batch=max(b.n for b in batches),
                             param_capacity=c.param_capacity, sample_count=c.sample_count, interval_ms=c.interval_ms)
    o = so.OracleEngine(cfg)
    _load(o, w)
    vs = [o.submit(b) for b in batches]
    want = np.concatenate([np.stack([v.status, v.wait_ms, v.rule_idx]).astype(np.int64) for v in vs], axis=1)
    return want, abi.node_state_to_dict(o.read_entry_node(), cfg.sample_count)


def _threads(fn, world):
    import threading
    comms = system_shard.LocalComm.group(world)
    parts, errs = [None] * world, []

    def run(r):
        try:
            parts[r] = fn(r, comms[r])
        except BaseException as ex:          # noqa: BLE001 -- re-raised below
            errs.append(ex)
            comms[r].s["bar"].abort()
    ths = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errs:
        raise errs[0]
    return parts


def _check(w, batches, parts):
    want, want_en = _reference(w, batches)
    got = _merge(parts, sum(b.n for b in batches))
    bad = np.nonzero((got != want).any(axis=0))[0]
    assert bad.size == 0, f"{bad.size} verdicts differ; first {bad[0]}: got {got[:, bad[0]]} want {want[:, bad[0]]}"
    assert (want[0] == abi.V_BLOCK_SYSTEM).sum() > 0, "the SystemRule never fired"
    for p in parts:
        assert p[2] == want_en


@pytest.mark.parametrize("kind", ["param", "mixed", "cpu", "geom"])
@pytest.mark.parametrize("world", [2, 3])
def test_exchange_protocol_local_ranks(kind, world):
    w, batches = exchange_workload(kind)
    logs = []
    parts = _threads(lambda r, c: _sim_rank(w, batches, world, r, c, logs if r == 0 else None), world)
    _check(w, batches, parts)
    assert sum(x["rounds"] for x in logs) >= 2


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w, batches = exchange_workload("mixed", 5000)
    q.put((rank, _sim_rank(w, batches, world, rank, system_shard.TorchComm())))
    dist.destroy_process_group()


def test_exchange_protocol_gloo_two_ranks():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    parts = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w, batches = exchange_workload("mixed", 5000)
    _check(w, batches, [parts[0], parts[1]])


def test_product_reduce_equals_restatement():
    """hostsim's build of sf_sysx.h sx_reduce (the product's plan step) against
    sysx_sim.sx_reduce on random node messages, every level."""
    from tests.hostsim import hostsim
    L = hostsim.lib()
    rng = np.random.default_rng(5)
    for trial in range(300):
        N = int(rng.integers(1, 5))
        lo = int(rng.integers(0, 1000))
        span = int(rng.choice([1, 7, 128, 129, 5000, 1 << 20]))
        plan = sysx_sim.begin(lo, lo + span)
        plan["P"] = int(rng.integers(0, 3000))
        qps, isec = float(rng.integers(100, 4000)), float(rng.choice([1.0, 0.5, 1.5]))
        for _level in range(6):
            m = np.zeros((N, sysx_sim.SX_WORDS), np.int64)
            n = rng.integers(0, 3, size=(N, sysx_sim.SX_B)) * (rng.random((N, sysx_sim.SX_B)) < 0.5)
            cmin = rng.integers(1, 4, size=(N, sysx_sim.SX_B))
            cmax = cmin + rng.integers(0, 3, size=(N, sysx_sim.SX_B))
            m[:, 16 + 128:16 + 256] = n
            m[:, 16:16 + 128] = n * cmin
            m[:, 16 + 256:16 + 384] = np.where(n > 0, cmin, sysx_sim.I64_MAX)
            m[:, 16 + 384:] = np.where(n > 0, cmax, sysx_sim.I64_MIN)
            hp = np.array([plan["lo"], plan["hi"], plan["w"], plan["ub"], plan["P"], plan["q"],
                           plan["done"] | (plan["level"] << 32), 0], np.int64)       # SxPlan
            L.hs_sx_reduce(m.ctypes.data, N, hp.ctypes.data, C.c_double(qps), C.c_double(isec))
            sysx_sim.sx_reduce(m, plan, qps, isec)
            got = dict(lo=hp[0], hi=hp[1], w=hp[2], ub=hp[3], q=hp[5], done=int(hp[6] & 0xffffffff),
                       level=int(hp[6] >> 32))
            for k, v in got.items():
                assert int(v) == plan[k], (trial, k, int(v), plan[k])
            if plan["done"]:
                break


# ---------------------------------------------------------------- GPU: the product
def _gpu_rank(w, batches, world, rank, comm):
    from sentinel_amd import engine
    cfg = _rank_cfg(w, batches, world, rank)
    e = engine.FlowEngine(cfg)
    try:
        _load(e, w, world, rank)
        pos, cols, off = [], [], 0
        for b in batches:
            sel = np.nonzero(b.res_id % world == rank)[0]
            v = system_shard.submit_node(e, b.shard(world, rank), sel + off, comm)
            pos.append(sel + off)
            cols.append(np.stack([v.status, v.wait_ms, v.rule_idx]).astype(np.int64))
            off += b.n
        return np.concatenate(pos), np.concatenate(cols, axis=1), abi.node_state_to_dict(e.read_entry_node(),
                                                                                          cfg.sample_count)
    finally:
        e.close()


class _CountingComm:
    def __init__(self, inner):
        self.inner, self.calls, self.bytes = inner, 0, 0

    def allgather_bytes(self, x):
        self.calls += 1
        self.bytes += x.nbytes
        return self.inner.allgather_bytes(x)

    def allgather_i64(self, x):
        return self.inner.allgather_i64(x)

    def allreduce_max_i32(self, x):
        return self.inner.allreduce_max_i32(x)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["param", "mixed", "cpu", "geom"])
def test_gpu_exchange_two_engines(kind):
    w, batches = exchange_workload(kind, 30_000)
    comms = []

    def rank(r, c):
        cc = _CountingComm(c)
        comms.append(cc)
        return _gpu_rank(w, batches, 2, r, cc)
    parts = _threads(rank, 2)
    _check(w, batches, parts)
    assert all(c.calls > 0 and c.bytes / c.calls <= 4400 for c in comms)   # the exchange ran: no event gather


@pytest.mark.gpu
def test_gpu_exchange_config4_shape_three_ranks():
    """Config 4's shape (ParamFlow over Zipf keys, inbound QPS at 0.6x: the
    rule fires between the ParamFlow blocks) on three engines."""
    w = workloads.system_large("param06")
    b = w["batches"][0].subset(0, 1 << 19)
    w["system"] = _qps_rule(0.6 * b.n / 4.0)
    parts = _threads(lambda r, c: _gpu_rank(w, [b], 3, r, c), 3)
    _check(w, [b], parts)


@pytest.mark.gpu
def test_gpu_exchange_thread_rule_falls_back():
    """A thread rule needs the event all-gather protocol: sf_submit_node
    refuses it on every rank, system_shard.submit_node falls back, exact."""
    w = workloads.system("thread")
    batches = w["batches"]
    parts = _threads(lambda r, c: _gpu_rank(w, batches, 2, r, c), 2)
    _check(w, batches, parts)


@pytest.mark.gpu
def test_gpu_exchange_rccl_single_rank():
    """The exchange over the engine's RCCL communicator (device buffers,
    ncclAllGather on the engine's stream) on a one-rank node: equal to one
    engine deciding the batches with sf_submit, ENTRY_NODE included."""
    from sentinel_amd import engine
    w, batches = exchange_workload("mixed", 30_000)
    c = w["cfg"]
    e, ref = engine.FlowEngine(c), engine.FlowEngine(c)
    try:
        for x in (e, ref):
            _load(x, w)
        e.comm_init(1, 0, engine.comm_unique_id())
        off = 0
        for b in batches:
            got = e.submit_node(b, np.arange(off, off + b.n, dtype=np.int64), None)
            want = ref.submit(b)
            off += b.n
            assert np.array_equal(got.status, want.status) and np.array_equal(got.wait_ms, want.wait_ms)
            assert np.array_equal(got.rule_idx, want.rule_idx)
            assert (want.status == abi.V_BLOCK_SYSTEM).sum() > 0
        assert abi.node_state_to_dict(e.read_entry_node()) == abi.node_state_to_dict(ref.read_entry_node())
    finally:
        e.close()
        ref.close()
