"""SF_EV_BLOCKED: an entry blocked by a slot that StatisticSlot wraps but the
engine does not run (AuthoritySlot, order -6000, between StatisticSlot -7000
and SystemSlot -5000, Constants.java:80-84).  StatisticSlot.entry catches its
BlockException (StatisticSlot.java:102-124): block += count on the resource's
node and, for EntryType.IN, on ENTRY_NODE; SystemSlot, ParamFlowSlot, FlowSlot
and DegradeSlot never see the entry; its exit records nothing (blockError,
:139).  CPU: the oracle's semantics (known answers), the host build of the
decision code (hostsim) against the oracle on mixed workloads, and the
degrade-only chain (oracle/degrade.py)."""
import numpy as np
import pytest

from sentinel_amd import abi, trace
from tests import workloads
from tests.test_hostsim_parity import thread_workload

T0 = trace.T0


def _qps_rule(res, count, behavior=0, **kw):
    return abi.sf_flow_rule(resource=res, grade=abi.GRADE_QPS, count=float(count), control_behavior=behavior,
                            warm_up_period_sec=10, max_queueing_time_ms=500, **kw)


def test_oracle_preblocked_counts_block_and_skips_rules(so):
    """QPS count 1: a pre-blocked entry does not consume the window's single
    pass; it is a block on the node and on ENTRY_NODE; its exit is ignored."""
    cfg = abi.default_config(max_resources=2, max_batch=16)
    o = so.OracleEngine(cfg)
    o.load_flow_rules([_qps_rule(0, 1)])
    IN, X, B = abi.EV_IN, abi.EV_EXIT | abi.EV_IN, abi.EV_IN | abi.EV_BLOCKED
    b = abi.HostBatch([0, 0, 0, 0, 0], [T0, T0 + 1, T0 + 2, T0 + 3, T0 + 4], [3, 1, 1, 1, 3],
                      [B, IN, IN, X, X], entry_ref=[-1, -1, -1, 1, 0])
    v = o.submit(b)
    assert list(v.status) == [abi.V_BLOCK_OTHER, abi.V_PASS, abi.V_BLOCK_FLOW, abi.V_EXIT, abi.V_EXIT_IGNORED]
    n = abi.node_state_to_dict(o.read_node(0), 2)
    en = abi.node_state_to_dict(o.read_entry_node(), 2)
    for d in (n, en):
        live = [bk for bk in d["second"] if bk[0] != abi.SF_WS_ABSENT]   # (ws, pass, block, ...)
        assert (sum(bk[2] for bk in live), sum(bk[1] for bk in live)) == (3 + 1, 1), d["second"]
        assert d["threads"] == 0


def test_oracle_preblocked_before_system_rule(so):
    """The inbound-QPS SystemRule never sees a pre-blocked entry (AuthoritySlot
    runs before SystemSlot): with qps 1 the first checked entry still passes."""
    cfg = abi.default_config(max_resources=1, max_batch=8)
    o = so.OracleEngine(cfg)
    o.load_system_rules([abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=1.0, avg_rt=-1,
                                            max_thread=-1)])
    IN, B = abi.EV_IN, abi.EV_IN | abi.EV_BLOCKED
    v = o.submit(abi.HostBatch([0, 0, 0], [T0, T0, T0], [1, 1, 1], [B, IN, IN]))
    assert list(v.status) == [abi.V_BLOCK_OTHER, abi.V_PASS, abi.V_BLOCK_SYSTEM]


def test_oracle_preblocked_param_and_breaker(so):
    """No ParamFlow token is consumed and no breaker is probed by a pre-blocked
    entry; the ParamFlow thread counter is untouched."""
    cfg = abi.default_config(max_resources=1, max_batch=8, param_capacity=64)
    o = so.OracleEngine(cfg)
    o.load_param_rules([abi.sf_param_rule(resource=0, grade=abi.GRADE_QPS, param_idx=0, control_behavior=0,
                                          count=1.0, max_queueing_time_ms=0, burst_count=0, duration_in_sec=1)], [])
    IN, B = abi.EV_IN, abi.EV_IN | abi.EV_BLOCKED
    tag = np.full((1, 3), abi.TAG_LONG, np.uint8)
    bits = np.full((1, 3), 7, np.uint64)
    v = o.submit(abi.HostBatch([0, 0, 0], [T0, T0, T0], [1, 1, 1], [B, IN, IN], arg_tag=tag, arg_bits=bits))
    assert list(v.status) == [abi.V_BLOCK_OTHER, abi.V_PASS, abi.V_BLOCK_PARAM]


def test_degrade_only_chain_skips_preblocked():
    """sf_degrade_submit's oracle: a pre-blocked entry never reaches
    DegradeSlot (V_BLOCK_OTHER) and its exit (same batch, or entry_ref -2) is
    ignored by the breakers (DegradeSlot.java:72-77)."""
    from oracle import degrade as od
    o = od.DegradeOracle()
    o.load_rules([dict(resource=0, grade=od.GRADE_EXC_COUNT, count=1.0, time_window_s=10,
                       min_request_amount=1, slow_ratio_threshold=1.0, stat_interval_ms=1000)])
    E, X, B = 0, od.EV_EXIT | od.EV_ERROR, od.EV_BLOCKED
    st, _ = o.submit([0, 0, 0, 0], [0, 1, 2, 3], [B, X, X, E], [-1, 0, -2, -1], [0, 0, 0, 0])
    assert list(st) == [od.V_BLOCK_OTHER, od.V_EXIT_IGNORED, od.V_EXIT_IGNORED, od.V_PASS]


PRE = {
    "config3": lambda: workloads.config3(),
    "config3_heavy": lambda: workloads.config3(seed=5, split=3),
    "multi_rule": workloads.multi_rule,
    "prioritized": workloads.prioritized,
    "param_mixed": workloads.param_mixed,
    "config4": workloads.config4,
    "thread": lambda: thread_workload(2),
}


@pytest.mark.parametrize("heavy_min", [0, 4])
@pytest.mark.parametrize("name", list(PRE))
def test_hostsim_preblocked(so, name, heavy_min):
    """The engine's decision code (host build) equals the oracle with 5 % of
    the entries pre-blocked, on the lane walk and (heavy_min 4) the window paths."""
    from tests.hostsim import hostsim
    w = workloads.preblocked(PRE[name](), frac=0.05, seed=7)
    if heavy_min:
        w["cfg"].heavy_min_events = heavy_min
    _, _, outs = workloads.run(hostsim.HostSimEngine, so.OracleEngine, w)
    st = np.concatenate([o[1].status for o in outs])
    assert (st == abi.V_BLOCK_OTHER).sum() > 0


@pytest.mark.parametrize("seed", [31, 32])
def test_hostsim_preblocked_degrade_chain(so, seed):
    """Degrade chain inside sf_submit (host build): breakers never see a
    pre-blocked entry or its exit."""
    from tests.hostsim import hostsim
    from tests import parity, test_degrade_chain as tc
    cfg, flow, rules, b = tc.chain_workload(seed, prio=0.1)
    cut = b.n // 2
    w = workloads.preblocked(dict(batches=[b.subset(0, cut), b.subset(cut, b.n)]), frac=0.08, seed=seed)
    h, got, n = tc.run_chain(hostsim.HostSimEngine, cfg, flow, rules, w["batches"])
    o, want, n2 = tc.run_chain(so.OracleEngine, cfg, flow, rules, w["batches"])
    assert n == n2
    for k, (g, x) in enumerate(zip(got, want)):
        parity.compare_verdicts(g, x, f"batch{k}")
    st = np.concatenate([x.status for x in want])
    assert (st == abi.V_BLOCK_OTHER).sum() > 0 and (st == abi.V_BLOCK_DEGRADE).sum() > 0
    assert np.array_equal(tc._breaker_rows(h, n), tc._breaker_rows(o, n))
