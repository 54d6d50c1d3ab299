"""CPU check of the engine's decision code (sf_decide.h + sf_heavy.h, host
build) against the oracle on every seeded parity workload, both with the
default light/heavy split and with a tiny heavy threshold so the window/skip
algorithms run on every non-trivial segment.  The GPU parity suite
(test_gpu_parity.py) runs the same workloads through libsentinel_flow.so."""
import ctypes as C

import numpy as np
import pytest

from sentinel_amd import abi
from tests import workloads


@pytest.fixture(scope="module")
def hs():
    from tests.hostsim import hostsim
    L = hostsim.lib()
    L.hs_heavy_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.hs_mode_counts.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    return hostsim


@pytest.mark.parametrize("heavy_min", [0, 8])
@pytest.mark.parametrize("name", list(workloads.ALL))
def test_workload(hs, so, name, heavy_min):
    w = workloads.ALL[name]()
    w["cfg"].heavy_min_events = heavy_min
    eng, _, outs = workloads.run(hs.HostSimEngine, so.OracleEngine, w)
    if name == "config1":
        b = w["batches"][0]
        st = outs[0][1].status
        ent = (b.flags & abi.EV_EXIT) == 0
        pt = b.ts_ms[ent][st[ent] == abi.V_PASS]
        hw = pt // 500
        c = np.bincount(hw - hw.min())
        assert (c[:-1] + c[1:]).max() <= 20     # FlowQpsDemo: <= 20 passes per 1 s window
    if name == "prioritized":
        assert (outs[0][1].status == abi.V_PRIORITY_WAIT).sum() > 0
    if heavy_min and name in ("config1", "config2", "config3"):
        h, it = C.c_uint64(), C.c_uint64()
        hs.lib().hs_heavy_stats(eng.h, C.byref(h), C.byref(it))
        assert it.value > 0, "window/skip path not exercised"


@pytest.mark.parametrize("heavy_min", [0, 4])
def test_config3_more_seeds(hs, so, heavy_min):
    for seed in (11, 23):
        w = workloads.config3(seed=seed, split=3)
        w["cfg"].heavy_min_events = heavy_min
        workloads.run(hs.HostSimEngine, so.OracleEngine, w)


@pytest.mark.parametrize("seed", range(6))
def test_heavy_edge_traces(hs, so, seed):
    """Dense single-resource traces with mixed acquireCount, long gaps, second
    boundaries and exits, through every heavy class at threshold 2."""
    rng = np.random.default_rng(100 + seed)
    R = 4
    rules = [abi.sf_flow_rule(resource=0, grade=abi.GRADE_QPS, count=float(rng.integers(1, 30)), control_behavior=0,
                              warm_up_period_sec=10, max_queueing_time_ms=500),
             abi.sf_flow_rule(resource=1, grade=abi.GRADE_QPS, count=float(rng.integers(5, 60)), control_behavior=1,
                              warm_up_period_sec=int(rng.integers(1, 5)), max_queueing_time_ms=500),
             abi.sf_flow_rule(resource=2, grade=abi.GRADE_QPS, count=float(rng.integers(1, 200)), control_behavior=2,
                              warm_up_period_sec=10, max_queueing_time_ms=int(rng.integers(1, 900)))]
    n = 40000
    gaps = rng.choice([0, 0, 0, 1, 2, 7, 450, 1700], size=n)
    ts = 1_700_000_000_000 + np.cumsum(gaps)
    res = rng.integers(0, R, n).astype(np.uint32)
    cnt = np.where(rng.random(n) < 0.7, 1, rng.integers(1, 7, n)).astype(np.int32)
    flags = np.full(n, abi.EV_IN, np.uint8)
    # exits for a third of the entries, 0..50 ms later
    ent = np.nonzero(rng.random(n) < 0.33)[0]
    ex_ts = ts[ent] + rng.integers(0, 50, ent.size)
    all_ts = np.concatenate([ts, ex_ts])
    key = np.lexsort((np.concatenate([np.zeros(n), np.ones(ent.size)]), all_ts))
    pos = np.empty(key.size, np.int64)
    pos[key] = np.arange(key.size)
    src = np.concatenate([np.arange(n), ent])
    fl = np.concatenate([flags, np.full(ent.size, abi.EV_EXIT | abi.EV_IN, np.uint8)])
    eref = np.full(key.size, -1, np.int64)
    eref[pos[n:]] = pos[ent]
    b = abi.HostBatch(res[src][key], all_ts[key], cnt[src][key], fl[key], entry_ref=eref)
    half = b.n // 2
    w = dict(cfg=abi.default_config(max_resources=R, max_batch=b.n, heavy_min_events=2), flow=rules,
             batches=[b.subset(0, half), b.subset(half, b.n)], nodes=list(range(R)), n_flow=3)
    workloads.run(hs.HostSimEngine, so.OracleEngine, w)


def thread_trace(seed, R=3, n=60000, exit_frac=0.9, max_rt=60, gaps=(0, 0, 0, 0, 1, 1, 3, 40)):
    """Entry/exit traces for THREAD-grade rules: most entries exit 0..max_rt ms
    later (many in the same millisecond), mixed acquireCount, rule counts small
    enough that the thread gate saturates."""
    rng = np.random.default_rng(300 + seed)
    ts = 1_700_000_000_000 + np.cumsum(rng.choice(list(gaps), size=n))
    res = rng.integers(0, R, n).astype(np.uint32)
    cnt = np.where(rng.random(n) < 0.85, 1, rng.integers(1, 5, n)).astype(np.int32)
    flags = np.full(n, abi.EV_IN, np.uint8)
    ent = np.nonzero(rng.random(n) < exit_frac)[0]
    ex_ts = ts[ent] + np.where(rng.random(ent.size) < 0.3, 0, rng.integers(0, max_rt, ent.size))
    all_ts = np.concatenate([ts, ex_ts])
    key = np.lexsort((np.concatenate([np.zeros(n), np.ones(ent.size)]), all_ts))
    pos = np.empty(key.size, np.int64)
    pos[key] = np.arange(key.size)
    src = np.concatenate([np.arange(n), ent])
    fl = np.concatenate([flags, np.full(ent.size, abi.EV_EXIT | abi.EV_IN, np.uint8)])
    fl[n:][rng.random(ent.size) < 0.1] |= abi.EV_ERROR
    eref = np.full(key.size, -1, np.int64)
    eref[pos[n:]] = pos[ent]
    return abi.HostBatch(res[src][key], all_ts[key], cnt[src][key], fl[key], entry_ref=eref)


def thread_workload(seed, R=3, n=60000, max_rt=60, gaps=(0, 0, 0, 0, 1, 1, 3, 40), heavy_min=2):
    rng = np.random.default_rng(400 + seed)
    rules = [abi.sf_flow_rule(resource=r, grade=abi.GRADE_THREAD, count=float(rng.integers(1, 40)) + (0.5 if r == 2 else 0),
                              control_behavior=0) for r in range(R)]
    b = thread_trace(seed, R, n=n, max_rt=max_rt, gaps=gaps)
    k = b.n // 3
    return dict(cfg=abi.default_config(max_resources=R, max_batch=b.n, heavy_min_events=heavy_min), flow=rules,
                batches=[b.subset(0, k), b.subset(k, 2 * k), b.subset(2 * k, b.n)], nodes=list(range(R)), n_flow=R)


@pytest.mark.parametrize("seed", range(4))
def test_heavy_thread_traces(hs, so, seed):
    """THREAD-grade heavy segments (SM_THREAD) against the oracle, split into
    three batches so exits reference entries of earlier batches."""
    w = thread_workload(seed)
    eng, _, _ = workloads.run(hs.HostSimEngine, so.OracleEngine, w)
    mc = (C.c_uint64 * 8)()
    hs.lib().hs_mode_counts(eng.h, mc)
    assert mc[6] >= 8     # SM_THREAD segments


def test_long_run_minute_wrap(hs, so):
    """70 s of config-3 traffic in 7 batches on the host build of the lane
    walk and the window paths: minute-bucket reuse after the 60 s wrap,
    controller state carried across batches."""
    w = workloads.long_run(R=4000, n=300_000)
    workloads.run(hs.HostSimEngine, so.OracleEngine, w)
