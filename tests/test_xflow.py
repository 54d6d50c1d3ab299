"""Flow rules that read a node other than the resource's ClusterNode:
origin-specific / "other" limitApp, RELATE, CHAIN, cluster rules without a
token service (FlowRuleChecker.java:61-229, FlowRuleManager.isOtherOrigin
:132-148).  The oracle is pinned by FlowRuleCheckerTest's node-selection
cases; the engine's xflow walk (sf_xflow.h) is checked against it on the CPU
(hostsim build) and on the GPU."""
import numpy as np
import pytest

from oracle.oracle import OracleEngine
from sentinel_amd import abi, trace
from tests import workloads

SEL = OracleEngine
APP_A, APP_B = 2, 3          # interned origin names "appA", "appB"


def _rule(res=0, count=1.0, grade=abi.GRADE_QPS, **kw):
    return abi.sf_flow_rule(resource=res, grade=grade, count=count, control_behavior=0, warm_up_period_sec=10,
                            max_queueing_time_ms=500, **kw)


def _oracle(rules, R=4):
    o = OracleEngine(abi.default_config(max_resources=R, max_batch=1024))
    o.load_flow_rules(rules)
    return o


# ---- FlowRuleCheckerTest (sentinel-core/src/test/.../flow/FlowRuleCheckerTest.java) ----
def test_kat_default_limit_app_selects_cluster_node():            # :40-50
    o = _oracle([_rule()])
    assert o.select_node(0, abi.ORIGIN_NONE) == SEL.SEL_CLUSTER
    assert o.select_node(0, APP_A) == SEL.SEL_CLUSTER


def test_kat_custom_origin_selects_origin_node():                   # :52-73
    assert _oracle([_rule(limit_app=APP_A)]).select_node(0, APP_A) == SEL.SEL_ORIGIN
    assert _oracle([_rule(limit_app=APP_B)]).select_node(0, APP_A) == SEL.SEL_NONE


def test_kat_other_origin():                                        # :75-100
    o = _oracle([_rule(limit_app=APP_A, count=1), _rule(limit_app=abi.APP_OTHER, count=2)])
    assert o.select_node(1, APP_B) == SEL.SEL_ORIGIN                # origin matches "other"
    assert o.select_node(1, APP_A) == SEL.SEL_NONE                  # origin named by an existing rule


def test_kat_empty_reference():                                     # :102-111
    # a blank refResource: the QPS rule is invalid at load (checkStrategyField), a THREAD one selects no node
    o = _oracle([_rule(grade=abi.GRADE_THREAD, strategy=abi.STRATEGY_CHAIN, ref_resource=abi.REF_NONE),
                 _rule(strategy=abi.STRATEGY_CHAIN, ref_resource=abi.REF_NONE)])
    assert o.select_node(0, abi.ORIGIN_NONE, 0) == SEL.SEL_NONE
    assert o.select_node(1) == -1                                   # only one valid rule loaded


def test_kat_relate_reference():                                    # :113-127
    assert _oracle([_rule(strategy=abi.STRATEGY_RELATE, ref_resource=1)]).select_node(0) == SEL.SEL_REF


def test_kat_chain_context_entrance():                              # :129-146
    good, other = 5, 6
    o = _oracle([_rule(strategy=abi.STRATEGY_CHAIN, ref_resource=good)])
    assert o.select_node(0, abi.ORIGIN_NONE, good) == SEL.SEL_CONTEXT
    assert o.select_node(0, abi.ORIGIN_NONE, other) == SEL.SEL_NONE


def _entries(res, origin=None, context=None, ts=None, n=None):
    n = n if n is not None else len(res)
    ts = np.full(n, trace.T0, np.int64) if ts is None else np.asarray(ts, np.int64)
    return abi.HostBatch(np.asarray(res, np.uint32), ts, np.ones(n, np.int32), np.full(n, abi.EV_IN, np.uint8),
                         origin=origin, context=context)


def test_kat_select_empty_node_passes():                            # :156-167 testPassCheckSelectEmptyNodeSuccess
    o = _oracle([_rule(count=1, limit_app=APP_A)])
    v = o.submit(_entries([0] * 5, origin=[APP_B] * 5))
    assert list(v.status) == [abi.V_PASS] * 5


# ---- hand-checked scenarios on the oracle ----
def test_origin_rule_counts_per_origin():
    o = _oracle([_rule(count=2, limit_app=APP_A)])
    v = o.submit(_entries([0] * 6, origin=[APP_A, APP_A, APP_B, APP_A, abi.ORIGIN_NONE, APP_B]))
    assert list(v.status) == [0, 0, 0, abi.V_BLOCK_FLOW, 0, 0]
    st = abi.node_state_to_dict(o.read_origin_node(0, APP_A))
    assert sum(b[1] for b in st["second"]) == 2 and sum(b[2] for b in st["second"]) == 1
    with pytest.raises(KeyError):
        o.read_origin_node(0, abi.ORIGIN_NONE)


def test_origin_node_exists_without_rules():
    """ClusterBuilderSlot creates the origin node of every entry with an origin
    (ClusterBuilderSlot.java:107-110), whatever the rules: an origin rule loaded
    mid-stream sees the traffic before it (QPS), and the exits of entries made
    before it keep the origin node's thread count exact (THREAD grade)."""
    o = _oracle([])
    o.submit(_entries([0] * 4, origin=[APP_A] * 4))                   # no rules: 4 passes on A's node
    st = abi.node_state_to_dict(o.read_origin_node(0, APP_A))
    assert sum(b[1] for b in st["second"]) == 4
    o.load_flow_rules([_rule(count=5, limit_app=APP_A)])
    v = o.submit(_entries([0] * 3, origin=[APP_A] * 3, ts=[trace.T0 + 1] * 3))
    assert list(v.status) == [0, abi.V_BLOCK_FLOW, abi.V_BLOCK_FLOW]   # (int)passQps 4 + 1 <= 5, then 5 + 1 > 5


def _threads_trace(seed, n=4000, R=3):
    """Entries with origins and their exits; a THREAD-grade origin rule is
    loaded after the first batch (mid-stream)."""
    rng = np.random.default_rng(seed)
    ts = trace.T0 + np.cumsum(rng.integers(0, 3, n))
    res = rng.integers(0, R, n).astype(np.uint32)
    org = rng.choice([APP_A, APP_B, abi.ORIGIN_NONE], n).astype(np.uint32)
    ent = np.nonzero(rng.random(n) < 0.8)[0]
    ex_ts = ts[ent] + rng.integers(0, 40, ent.size)
    all_ts = np.concatenate([ts, ex_ts])
    key = np.lexsort((np.concatenate([np.zeros(n), np.ones(ent.size)]), all_ts))
    pos = np.empty(key.size, np.int64)
    pos[key] = np.arange(key.size)
    src = np.concatenate([np.arange(n), ent])
    fl = np.concatenate([np.full(n, abi.EV_IN, np.uint8), np.full(ent.size, abi.EV_IN | abi.EV_EXIT, np.uint8)])
    eref = np.full(key.size, -1, np.int64)
    eref[pos[n:]] = pos[ent]
    return abi.HostBatch(res[src][key], all_ts[key], np.ones(key.size, np.int32), fl[key], entry_ref=eref,
                         origin=org[src][key])


@pytest.mark.parametrize("seed", [61, 62])
def test_hostsim_origin_rules_loaded_mid_stream(seed):
    """The engine's xflow walk (host build) against the oracle when THREAD /
    QPS origin rules are loaded after traffic with origins has flowed: every
    verdict, every ClusterNode and origin node equal, no origin node with a
    negative thread count."""
    from tests.hostsim.hostsim import HostSimEngine
    b = _threads_trace(seed)
    cut = b.n // 2
    batches = [b.subset(0, cut), b.subset(cut, b.n)]
    cfg = abi.default_config(max_resources=3, max_batch=b.n)
    rules = [_rule(0, count=3, grade=abi.GRADE_THREAD, limit_app=APP_A),
             _rule(1, count=2, grade=abi.GRADE_THREAD, limit_app=abi.APP_OTHER),
             _rule(2, count=4, limit_app=APP_B)]
    h, o = HostSimEngine(cfg), OracleEngine(cfg)
    from tests import parity
    parity.compare_verdicts(h.submit(batches[0]), o.submit(batches[0]), "before the rules")
    for x in (h, o):
        x.load_flow_rules(rules)
    v = o.submit(batches[1])
    parity.compare_verdicts(h.submit(batches[1]), v, "after the rules")
    assert (v.status == abi.V_BLOCK_FLOW).sum() > 0
    parity.compare_nodes(h, o, range(3))
    pairs = [(r, g) for r in range(3) for g in (APP_A, APP_B)]
    parity.compare_aux_nodes(h, o, origin_nodes=pairs)
    for r, g in pairs:
        assert abi.node_state_to_dict(o.read_origin_node(r, g))["threads"] >= 0


def test_relate_reads_the_referenced_cluster_node():
    o = _oracle([_rule(0, count=1, strategy=abi.STRATEGY_RELATE, ref_resource=1)])
    # resource 1 has no node yet -> pass; after two passes of 1, (int)passQps = 2 > 1 - 1 -> block
    v = o.submit(_entries([0, 1, 1, 0, 0], ts=[trace.T0] * 5))
    assert list(v.status) == [0, 0, 0, abi.V_BLOCK_FLOW, abi.V_BLOCK_FLOW]


def test_chain_reads_the_context_node():
    o = _oracle([_rule(count=1, strategy=abi.STRATEGY_CHAIN, ref_resource=7)])
    v = o.submit(_entries([0] * 4, context=[7, 0, 7, 0]))
    assert list(v.status) == [0, 0, abi.V_BLOCK_FLOW, 0]


def test_cluster_rule_without_token_service():
    o = _oracle([_rule(0, count=0, cluster_mode=1, cluster_fallback=0),
                 _rule(1, count=0, cluster_mode=1, cluster_fallback=1)])
    v = o.submit(_entries([0, 1, 0, 1]))
    assert list(v.status) == [0, abi.V_BLOCK_FLOW, 0, abi.V_BLOCK_FLOW]


# ---- engine logic vs oracle on the CPU (hostsim build of sf_xflow.h) ----
@pytest.mark.parametrize("seed", [51, 52, 53])
def test_hostsim_xflow_parity(seed):
    from tests.hostsim.hostsim import HostSimEngine
    w = workloads.xflow(seed=seed, R=300, n=30_000)
    workloads.run(HostSimEngine, OracleEngine, w)


def test_hostsim_xflow_geometry():
    from tests.hostsim.hostsim import HostSimEngine
    w = workloads.xflow(seed=54, R=200, n=20_000)
    w["cfg"] = abi.default_config(max_resources=200, max_batch=w["cfg"].max_batch, sample_count=4, interval_ms=2000)
    workloads.run(HostSimEngine, OracleEngine, w)


# ---- GPU: the HIP xflow walk through the C-ABI ----
@pytest.mark.gpu
@pytest.mark.parametrize("seed,R,n", [(51, 400, 60_000), (55, 3000, 400_000)])
def test_gpu_xflow_parity(seed, R, n):
    from sentinel_amd.engine import FlowEngine
    w = workloads.xflow(seed=seed, R=R, n=n)
    workloads.run(FlowEngine, OracleEngine, w)


@pytest.mark.gpu
def test_gpu_xflow_with_system_rule():
    """xflow groups inside the SystemRule planner's sub-batches (views)."""
    from sentinel_amd.engine import FlowEngine
    w = workloads.xflow(seed=56, R=300, n=60_000)
    w["system"] = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=0.5 * 60_000 / 6.0,
                                      avg_rt=-1, max_thread=-1)]
    w["status"] = (0.0, 0.0)
    workloads.run(FlowEngine, OracleEngine, w)


@pytest.mark.gpu
def test_gpu_xflow_sharded_colocated():
    """RELATE pairs on one shard (res % 2): two engines equal one replay."""
    from sentinel_amd.engine import FlowEngine
    from tests import parity
    w = workloads.xflow(seed=57, R=400, n=60_000)
    for r in w["flow"]:                      # co-locate: refResource on the resource's shard
        ref = r.ref_resource
        if r.strategy == abi.STRATEGY_RELATE and ref != abi.REF_NONE and ref % 2 != r.resource % 2:
            r.ref_resource = ref + 1 if ref >= 400 else (ref + 1) % 400   # (beyond 400: never a node)
    cfg1 = w["cfg"]
    ora = OracleEngine(cfg1)
    ora.load_flow_rules(w["flow"])
    outs = [ora.submit(b) for b in w["batches"]]
    for k in range(2):
        cfg = abi.default_config(max_resources=200, max_batch=cfg1.max_batch, shard_count=2, shard_index=k)
        eng = FlowEngine(cfg)
        eng.load_flow_rules([r for r in w["flow"] if r.resource % 2 == k])
        for b, o in zip(w["batches"], outs):
            sel = np.nonzero(b.res_id % 2 == k)[0]
            v = eng.submit(b.shard(2, k))
            for f in ("status", "wait_ms", "rule_idx"):
                assert np.array_equal(getattr(v, f), getattr(o, f)[sel]), f
        parity.compare_aux_nodes(eng, ora, [x for x in w["origin_nodes"] if x[0] % 2 == k],
                                 [x for x in w["context_nodes"] if x[1] % 2 == k])
        eng.close()


@pytest.mark.gpu
def test_gpu_xflow_pool_capacity():
    """More origin / context nodes than aux_capacity: the pool grows between
    batches (the sort phase's index pass sizes it), nothing fails or drops."""
    from sentinel_amd.engine import FlowEngine
    w = workloads.xflow(seed=58, R=300, n=30_000)
    w["cfg"].aux_capacity = 8
    workloads.run(FlowEngine, OracleEngine, w)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [61, 62])
def test_gpu_origin_rules_loaded_mid_stream(seed):
    """Origin nodes for every entry with an origin (the origin-node pass while
    no rule reads them, sf_origin.hip) and origin rules loaded mid-stream (the
    xflow walk from then on): verdicts, ClusterNodes and origin nodes equal
    the oracle's."""
    from sentinel_amd.engine import FlowEngine
    from tests import parity
    b = _threads_trace(seed)
    cut = b.n // 2
    batches = [b.subset(0, cut), b.subset(cut, b.n)]
    cfg = abi.default_config(max_resources=3, max_batch=b.n)
    rules = [_rule(0, count=3, grade=abi.GRADE_THREAD, limit_app=APP_A),
             _rule(1, count=2, grade=abi.GRADE_THREAD, limit_app=abi.APP_OTHER),
             _rule(2, count=4, limit_app=APP_B)]
    e, o = FlowEngine(cfg), OracleEngine(cfg)
    try:
        parity.compare_verdicts(e.submit(batches[0]), o.submit(batches[0]), "before the rules")
        for x in (e, o):
            x.load_flow_rules(rules)
        parity.compare_verdicts(e.submit(batches[1]), o.submit(batches[1]), "after the rules")
        parity.compare_nodes(e, o, range(3))
        parity.compare_aux_nodes(e, o, origin_nodes=[(r, g) for r in range(3) for g in (APP_A, APP_B)])
    finally:
        e.close()
