"""Origin nodes of traffic no rule reads: the origin-node pass (sf_origin.hip)
against the C oracle.

ClusterBuilderSlot creates the origin node of every entry with an origin
(ClusterBuilderSlot.java:107-110) and StatisticSlot updates it beside the
resource's node (StatisticSlot.java:64-178).  Resources whose rules read an
origin node run on the xflow walk; every other resource's segments stay on the
ordinary light / heavy / stream kernels and their origin nodes are updated
after the verdicts (k_ox_light for segments of at most 512 events, k_ox_hacc +
k_ox_happly for longer ones).  These tests compare every verdict, a sample of
ClusterNodes, a sample of origin nodes (the busiest pairs of the long segments
and random pairs of the short ones) and ENTRY_NODE with the oracle, and check
that the pool and its index grow instead of failing a batch."""
import numpy as np
import pytest

from oracle.oracle import OracleEngine
from sentinel_amd import abi, trace
from tests import parity

pytestmark = pytest.mark.gpu


def _sample_pairs(hb, k_busy=24, k_rand=400, seed=5):
    """(resource, origin) pairs: every origin of the k_busy busiest resources
    and k_rand random pairs of the batch."""
    ent = hb.origin != abi.ORIGIN_NONE
    key = hb.res_id[ent].astype(np.uint64) << np.uint64(32) | hb.origin[ent].astype(np.uint64)
    u, c = np.unique(key, return_counts=True)
    per_res = np.bincount(hb.res_id, minlength=int(hb.res_id.max()) + 1)
    busy = set(np.argsort(-per_res)[:k_busy].tolist())
    res = (u >> np.uint64(32)).astype(np.int64)
    pick = [i for i in range(u.size) if res[i] in busy]
    rng = np.random.default_rng(seed)
    pick += rng.choice(u.size, size=min(k_rand, u.size), replace=False).tolist()
    pick = sorted(set(pick))
    return [(int(u[i] >> np.uint64(32)), int(u[i] & np.uint64(0xffffffff))) for i in pick]


def _run(rules, batches, cfg, pairs, res_sample, async_dev=False):
    from sentinel_amd import engine
    eng, ora = engine.FlowEngine(cfg), OracleEngine(cfg)
    try:
        eng.load_flow_rules(rules)
        ora.load_flow_rules(rules)
        for k, b in enumerate(batches):
            want = ora.submit(b)
            if async_dev:
                db = engine.DeviceBatch(eng, b)
                dv = engine.DeviceVerdicts(eng, b.n, with_wait=True, with_rule=True)
                eng.submit_device_async(db, dv)
                eng.sync()
                got = abi.HostVerdicts(b.n)
                got.status[:] = dv.status.numpy(); got.wait_ms[:] = dv.wait_ms.numpy(); got.rule_idx[:] = dv.rule_idx.numpy()
                db.free(); dv.free()
            else:
                got = eng.submit(b)
            parity.compare_verdicts(got, want, f"batch {k}")
        parity.compare_nodes(eng, ora, res_sample)
        parity.compare_entry_node(eng, ora)
        parity.compare_aux_nodes(eng, ora, origin_nodes=pairs)
        return eng.stats()
    finally:
        eng.close()
        ora.close()


def test_gpu_origin_nodes_config3_shape():
    """The config-3 mix (QPS / THREAD / WarmUp / RateLimiter, Zipf(1.1)) with a
    Zipf-drawn origin out of 64 on every entry, no origin rules: 2.1M events in
    three batches, heavy_min 512 -- long segments on the window / stream
    kernels and k_ox_hacc, short ones on the lane walks and k_ox_light."""
    R = 20_000
    hb = trace.with_origins(trace.mixed_zipf(R, 2_100_000, duration_ms=6000, seed=31), seed=32)
    rules = trace.mixed_rules(R, seed=31)
    cuts = [0, 700_000, 1_400_000, hb.n]
    batches = [hb.subset(cuts[i], cuts[i + 1]) for i in range(3)]
    cfg = abi.default_config(max_resources=R, max_batch=max(b.n for b in batches), heavy_min_events=512)
    per_res = np.bincount(hb.res_id, minlength=R)
    assert (per_res > 512 * 2).sum() > 20                    # long segments in every batch
    res_sample = np.unique(np.concatenate([np.argsort(-per_res)[:32], np.arange(0, R, 97)]))
    st = _run(rules, batches, cfg, _sample_pairs(hb), res_sample)
    ent = hb.origin != abi.ORIGIN_NONE
    n_pairs = np.unique(hb.res_id[ent].astype(np.uint64) << np.uint64(32) | hb.origin[ent].astype(np.uint64)).size
    assert st.aux_nodes == n_pairs


def test_gpu_origin_nodes_async_pipelined():
    """The same pass on HBM-resident batches through sf_submit_async."""
    R = 5000
    hb = trace.with_origins(trace.mixed_zipf(R, 600_000, duration_ms=4000, seed=33), seed=34, none_frac=0.2)
    rules = trace.mixed_rules(R, seed=33)
    batches = [hb.subset(0, 300_000), hb.subset(300_000, hb.n)]
    cfg = abi.default_config(max_resources=R, max_batch=300_000)
    per_res = np.bincount(hb.res_id, minlength=R)
    _run(rules, batches, cfg, _sample_pairs(hb), np.argsort(-per_res)[:64], async_dev=True)


def test_gpu_origin_pool_and_index_grow():
    """More (resource, origin) pairs than aux_capacity, arriving over several
    batches: the pool grows by chunks and the index table is rebuilt larger
    between batches; nothing fails, every pair is exact."""
    R = 60_000
    rng = np.random.default_rng(35)
    n = 240_000
    res = rng.integers(0, R, n).astype(np.uint32)
    ts = trace.T0 + np.sort(rng.integers(0, 8000, n)).astype(np.int64)
    org = (2 + rng.integers(0, 6, n)).astype(np.uint32)
    hb = abi.HostBatch(res, ts, np.ones(n, np.int32), np.full(n, abi.EV_IN, np.uint8), origin=org)
    rules = [abi.sf_flow_rule(resource=r, grade=abi.GRADE_QPS, count=float(1 + r % 5), strategy=0,
                              control_behavior=0, warm_up_period_sec=10, max_queueing_time_ms=500)
             for r in range(0, R, 3)]
    batches = [hb.subset(k * 60_000, (k + 1) * 60_000) for k in range(4)]
    cfg = abi.default_config(max_resources=R, max_batch=60_000)
    cfg.aux_capacity = 1000                                  # one chunk (65536 nodes) to start with
    pairs = _sample_pairs(hb, 8, 600)
    st = _run(rules, batches, cfg, pairs, np.arange(0, R, 211))
    n_pairs = np.unique(res.astype(np.uint64) << np.uint64(32) | org.astype(np.uint64)).size
    assert st.aux_nodes == n_pairs > 65536
    assert st.aux_capacity >= n_pairs
    assert st.aux_index_grows >= 1


def test_gpu_origin_with_other_rules():
    """'other' / origin-specific limitApp rules on 1% of the resources (the
    xflow walk, which updates their origin nodes in line) beside the plain
    traffic of the rest (the origin-node pass), in the same batches."""
    R = 20_000
    hb = trace.with_origins(trace.mixed_zipf(R, 1_000_000, duration_ms=4000, seed=36), n_origins=16, seed=37)
    rules = list(trace.mixed_rules(R, seed=36))
    per_res = np.bincount(hb.res_id, minlength=R)
    xres = np.argsort(-per_res)[5:5 + R // 100]              # 1%: some long segments among them
    for r in xres:
        rules.append(abi.sf_flow_rule(resource=int(r), grade=abi.GRADE_QPS, count=float(5 + r % 40), strategy=0,
                                      control_behavior=0, warm_up_period_sec=10, max_queueing_time_ms=500,
                                      limit_app=abi.APP_OTHER))
    batches = [hb.subset(0, 500_000), hb.subset(500_000, hb.n)]
    cfg = abi.default_config(max_resources=R, max_batch=500_000)
    pairs = _sample_pairs(hb) + [(int(r), o) for r in xres[:10] for o in range(2, 18)
                                 if ((hb.res_id == r) & (hb.origin == o)).any()]
    _run(rules, batches, cfg, sorted(set(pairs)), np.concatenate([xres[:50], np.argsort(-per_res)[:20]]))


def test_gpu_origin_with_system_rule():
    """Origins inside the SystemRule planner's sub-batches (each view runs the
    index pass and the origin-node pass)."""
    R = 2000
    hb = trace.with_origins(trace.mixed_zipf(R, 200_000, duration_ms=4000, seed=38), n_origins=8, seed=39)
    rules = trace.mixed_rules(R, seed=38)
    cfg = abi.default_config(max_resources=R, max_batch=hb.n)
    sysr = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=0.4 * hb.n / 4.0,
                               avg_rt=-1, max_thread=-1)]
    from sentinel_amd import engine
    eng, ora = engine.FlowEngine(cfg), OracleEngine(cfg)
    try:
        for x in (eng, ora):
            x.load_system_rules(sysr)
            x.load_flow_rules(rules)
        got, want = eng.submit(hb), ora.submit(hb)
        parity.compare_verdicts(got, want)
        assert (want.status == abi.V_BLOCK_SYSTEM).sum() > 1000
        assert eng.stats().sys_rounds > 1
        parity.compare_entry_node(eng, ora)
        parity.compare_aux_nodes(eng, ora, origin_nodes=_sample_pairs(hb, 16, 300))
    finally:
        eng.close()
        ora.close()


def test_gpu_param_table_grows_between_batches():
    """The exact ParamFlow table from 4096 slots under four batches of
    Zipf-drawn values (many new keys per batch): the engine rebuilds it larger
    before a batch that could fill it (sf_engine.cpp param_reserve), so no
    batch fails, and every verdict, wait and rule index equals the oracle's."""
    from sentinel_amd import engine
    rules, b = trace.param_zipf(300, 200_000, 1_000_000, duration_ms=8000, seed=41)
    batches = [b.subset(k * 50_000, (k + 1) * 50_000) for k in range(4)]
    cfg = abi.default_config(max_resources=300, max_batch=50_000, param_capacity=4096)
    eng, ora = engine.FlowEngine(cfg), OracleEngine(cfg)
    try:
        for x in (eng, ora):
            x.load_param_rules(rules)
        for k, bb in enumerate(batches):
            parity.compare_verdicts(eng.submit(bb), ora.submit(bb), f"batch {k}")
        st = eng.stats()
        assert st.param_table_grows >= 1
        used = eng.param_table_stats()["used"]
        assert used > 4096
    finally:
        eng.close()
        ora.close()
