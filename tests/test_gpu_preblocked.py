"""GPU parity of SF_EV_BLOCKED entries (blocked by AuthoritySlot, which
StatisticSlot wraps but the engine does not run; StatisticSlot.java:102-124,
Constants.java:80-84) through libsentinel_flow.so: verdicts, nodes, ENTRY_NODE
and controller state equal the oracle's on config-3 traffic (lane walk, the
heavy QPS / WarmUp / RateLimiter / THREAD / no-rule / ParamFlow window paths),
on the degrade chain inside sf_submit, under SystemRules (planner) and on the
degrade-only chain."""
import numpy as np
import pytest

from sentinel_amd import abi, trace
from tests import parity, workloads
from tests.test_preblocked import PRE

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng_mod():
    from sentinel_amd import engine
    engine.lib()
    return engine


def _count(outs, v):
    return sum(int((o[1].status == v).sum()) for o in outs)


@pytest.mark.parametrize("heavy_min", [0, 8])
@pytest.mark.parametrize("name", list(PRE))
def test_preblocked_workloads(eng_mod, so, name, heavy_min):
    w = workloads.preblocked(PRE[name](), frac=0.05, seed=3)
    if heavy_min:
        w["cfg"].heavy_min_events = heavy_min
    _, _, outs = workloads.run(eng_mod.FlowEngine, so.OracleEngine, w)
    assert _count(outs, abi.V_BLOCK_OTHER) > 0


@pytest.mark.parametrize("heavy_min", [0, 64])
def test_preblocked_config3_large(eng_mod, so, heavy_min):
    """600k events of config 3 over 5 batches with 3 % pre-blocked entries:
    the stream kernel's THREAD / RateLimiter segments and the heavy fill."""
    w = workloads.preblocked(workloads.config3(R=20_000, n=600_000, seed=17, split=5), frac=0.03, seed=5)
    w["cfg"].heavy_min_events = heavy_min
    _, _, outs = workloads.run(eng_mod.FlowEngine, so.OracleEngine, w)
    assert _count(outs, abi.V_BLOCK_OTHER) > 1000


@pytest.mark.parametrize("seed", range(2))
def test_preblocked_thread_stream(eng_mod, so, seed):
    """THREAD-grade heavy segments (k_heavy_stream) with pre-blocked entries
    and their in-window / far / cross-batch exits."""
    from tests.test_hostsim_parity import thread_workload
    w = workloads.preblocked(thread_workload(seed, heavy_min=2), frac=0.1, seed=seed)
    _, _, outs = workloads.run(eng_mod.FlowEngine, so.OracleEngine, w)
    assert _count(outs, abi.V_BLOCK_OTHER) > 0


@pytest.mark.parametrize("kind", ["qps", "thread", "rt"])
def test_preblocked_system_rule(eng_mod, so, kind):
    """AuthoritySlot runs before SystemSlot: pre-blocked IN entries are blocks
    on ENTRY_NODE that the planner never classifies."""
    w = workloads.preblocked(workloads.system(kind), frac=0.05, seed=11)
    _, _, outs = workloads.run(eng_mod.FlowEngine, so.OracleEngine, w)
    assert _count(outs, abi.V_BLOCK_OTHER) > 0
    if kind != "rt":
        assert _count(outs, abi.V_BLOCK_SYSTEM) > 0


@pytest.mark.parametrize("seed,heavy_min,system", [(21, 512, False), (22, 8, True)])
def test_preblocked_degrade_chain(eng_mod, so, seed, heavy_min, system):
    """Breakers inside sf_submit never see a pre-blocked entry or its exit."""
    from tests import test_degrade_chain as tc
    cfg, flow, rules, b = tc.chain_workload(seed, prio=0.1, n=60_000)
    cfg.heavy_min_events = heavy_min
    cut = b.n // 3
    w = workloads.preblocked(dict(batches=[b.subset(0, cut), b.subset(cut, b.n)]), frac=0.08, seed=seed)
    sysr = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=-1, avg_rt=-1,
                               max_thread=60)] if system else None
    e, got, n = tc.run_chain(eng_mod.FlowEngine, cfg, flow, rules, w["batches"], sysr)
    o, want, n2 = tc.run_chain(so.OracleEngine, cfg, flow, rules, w["batches"], sysr)
    assert n == n2
    for k, (g, x) in enumerate(zip(got, want)):
        parity.compare_verdicts(g, x, f"batch{k}")
    st = np.concatenate([x.status for x in want])
    assert (st == abi.V_BLOCK_OTHER).sum() > 0 and (st == abi.V_BLOCK_DEGRADE).sum() > 0
    assert np.array_equal(tc._breaker_rows(e, n), tc._breaker_rows(o, n))
    parity.compare_nodes(e, o, range(0, cfg.max_resources, 3), sample_count=cfg.sample_count)
    parity.compare_entry_node(e, o, sample_count=cfg.sample_count)


def test_preblocked_degrade_only_chain(eng_mod):
    """sf_degrade_submit: pre-blocked entries and their exits skip the breakers
    (oracle/degrade.py)."""
    from tests import test_degrade as td
    R = 3000
    rules = trace.degrade_rules(R, seed=7)
    full = trace.degrade_workload(R, 60_000, duration_ms=8000, seed=7, err_p=0.2)
    cut = [0, full.n // 2, full.n]
    w = workloads.preblocked(dict(batches=[full.subset(cut[i], cut[i + 1]) for i in range(2)]), frac=0.1, seed=7)
    outs = td.check_gpu(rules, w["batches"], R, "preblocked")
    allst = np.concatenate([x[0] for x in outs])
    assert (allst == abi.V_BLOCK_OTHER).sum() > 0 and (allst == abi.V_BLOCK_DEGRADE).sum() > 0
