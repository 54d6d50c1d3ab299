"""DegradeSlot inside sf_submit's slot chain (after SystemSlot, ParamFlowSlot
and FlowSlot; DegradeSlot.java:42-94): a degrade block counts as a block in
StatisticSlot, an entry blocked earlier in the chain (or waiting on a
PriorityWaitException) never reaches the breakers, and only the exits of
entries that passed the whole chain complete a request on them.

Pinning: with degrade rules alone the C oracle's chain must reproduce the
committed degrade golden vectors and the degrade-only oracle (itself pinned
by the reference's breaker KATs in tests/test_degrade.py).  Then the engine's
own decision code (tests/hostsim: sf_decide.h built for the CPU) runs flow +
param + degrade rules against the C oracle; tests/test_gpu_parity.py repeats
it on the GPU."""
import numpy as np
import pytest

from oracle import degrade as od
from oracle import oracle as so
from sentinel_amd import abi, trace
from tests import parity
from tests.test_golden import _degrade_case, _state_row


def _breaker_rows(e, n):
    out = []
    for k in range(n):
        s = e.read_breaker(k)
        if isinstance(s, dict):                              # FlowEngine.read_breaker
            ws = abi.SF_WS_ABSENT if s["window_start"] is None else s["window_start"]
            out.append([s["state"], s["next_retry_ms"], ws, s["hit_count"], s["total_count"]])
        else:
            out.append([s.state, s.next_retry_ms, s.window_start, s.hit_count, s.total_count])
    return np.array(out, np.int64).reshape(n, 5)


def test_chain_oracle_degrade_only_reproduces_golden():
    R, rules, batches, breakers = _degrade_case()
    o = so.OracleEngine(abi.default_config(max_resources=R, max_batch=max(b.n for b, _, _ in batches)))
    assert o.load_degrade_rules(rules) == breakers.shape[0]
    for b, st, ri in batches:
        v = o.submit(b)
        assert np.array_equal(v.status, st)
        blk = st == abi.V_BLOCK_DEGRADE
        assert np.array_equal(v.rule_idx[blk], ri[blk])
    assert np.array_equal(_breaker_rows(o, breakers.shape[0]), breakers)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_chain_oracle_degrade_only_equals_degrade_oracle(seed):
    R = 300
    rules = trace.degrade_rules(R, seed=seed)
    b = trace.degrade_workload(R, 20_000, duration_ms=5000, seed=seed, err_p=0.25)
    o = so.OracleEngine(abi.default_config(max_resources=R, max_batch=b.n))
    n = o.load_degrade_rules(rules)
    d = od.DegradeOracle()
    assert d.load_rules(rules) == n
    v = o.submit(b)
    want, wri = d.submit(b.res_id, b.ts_ms, b.flags, b.entry_ref, b.create_ts)
    assert np.array_equal(v.status, want)
    blk = want == od.V_BLOCK_DEGRADE
    assert blk.sum() > 0
    assert np.array_equal(v.rule_idx[blk], wri[blk])
    assert np.array_equal(_breaker_rows(o, n), np.array([_state_row(d.state(k)) for k in range(n)], np.int64))


def chain_workload(seed, R=400, n=30_000, duration_ms=4000, prio=0.0):
    """Mixed flow rules (all four controllers, QPS and THREAD) plus breakers on
    half of the resources, over entries with exits (RT ~ Exp(20 ms), errors 25 %),
    IN and OUT entries, optional prioritized entries."""
    rng = np.random.default_rng(seed)
    flow = trace.mixed_rules(R, seed=seed)
    rules = trace.degrade_rules(R, seed=seed + 100)
    b = trace.degrade_workload(R, n, duration_ms=duration_ms, seed=seed, err_p=0.25)
    fl = b.flags.copy()
    ent = (fl & abi.EV_EXIT) == 0
    # IN entries (and their exits) on the even resources; prioritized entries
    fl[(b.res_id % 2 == 0)] |= abi.EV_IN
    if prio:
        fl[ent & (rng.random(b.n) < prio)] |= abi.EV_PRIO
    cnt = np.where(ent, rng.integers(1, 3, b.n), 1).astype(np.int32)
    b = abi.HostBatch(b.res_id, b.ts_ms, cnt, fl, entry_ref=b.entry_ref)
    cfg = abi.default_config(max_resources=R, max_batch=b.n)
    return cfg, flow, rules, b


def run_chain(make, cfg, flow, rules, batches, system=None):
    e = make(cfg)
    if system:
        e.load_system_rules(system)
    e.load_flow_rules(flow)
    n = e.load_degrade_rules(rules)
    return e, [e.submit(b) for b in batches], n


@pytest.mark.parametrize("seed", [11, 12])
@pytest.mark.parametrize("prio", [0.0, 0.2])
def test_hostsim_chain_matches_oracle(seed, prio):
    from tests.hostsim import hostsim
    cfg, flow, rules, b = chain_workload(seed, prio=prio)
    cut = b.n // 2
    batches = [b.subset(0, cut), b.subset(cut, b.n)]
    h, got, n = run_chain(hostsim.HostSimEngine, cfg, flow, rules, batches)
    o, want, n2 = run_chain(so.OracleEngine, cfg, flow, rules, batches)
    assert n == n2
    for k, (g, w) in enumerate(zip(got, want)):
        parity.compare_verdicts(g, w, f"batch{k}")
    st = np.concatenate([w.status for w in want])
    assert (st == abi.V_BLOCK_DEGRADE).sum() > 0 and (st == abi.V_BLOCK_FLOW).sum() > 0
    assert np.array_equal(_breaker_rows(h, n), _breaker_rows(o, n))
    parity.compare_nodes(h, o, range(0, cfg.max_resources, 7), sample_count=cfg.sample_count)
