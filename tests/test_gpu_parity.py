"""GPU parity: libsentinel_flow.so (HIP, gfx950) against the oracle, bit for
bit (verdicts, waits, rule indices, node windows, controller state), on every
seeded workload, through the C-ABI.  Run with -m gpu on an MI355X."""
import numpy as np
import pytest

from sentinel_amd import abi, trace
from tests import parity, workloads

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng_mod():
    from sentinel_amd import engine
    engine.lib()
    return engine


@pytest.mark.parametrize("heavy_min", [0, 8])
@pytest.mark.parametrize("name", list(workloads.ALL))
def test_workload(eng_mod, so, name, heavy_min):
    w = workloads.ALL[name]()
    w["cfg"].heavy_min_events = heavy_min
    workloads.run(eng_mod.FlowEngine, so.OracleEngine, w)


@pytest.mark.parametrize("heavy_min", [0, 64])
def test_config3_many_batches(eng_mod, so, heavy_min):
    w = workloads.config3(R=20_000, n=600_000, seed=17, split=5)
    w["cfg"].heavy_min_events = heavy_min
    workloads.run(eng_mod.FlowEngine, so.OracleEngine, w)


def test_long_run_minute_wrap(eng_mod, so):
    """70 s of config-3 traffic in 7 batches with the default split (light
    segments up to 512 events on the lane walks): nodes (minute buckets
    reused after the 60 s wrap), every rule's controller state (WarmUp tokens,
    RateLimiter latestPassedTime) and ENTRY_NODE equal the oracle's."""
    w = workloads.long_run()
    eng, ora, outs = workloads.run(eng_mod.FlowEngine, so.OracleEngine, w)
    span = int(w["batches"][-1].ts_ms[-1] - w["batches"][0].ts_ms[0])
    assert span > 60_000, span


@pytest.mark.parametrize("seed", range(4))
def test_heavy_edge_traces(eng_mod, so, seed):
    from tests.test_hostsim_parity import test_heavy_edge_traces as body
    import types
    # reuse the CPU edge-trace builder with the GPU engine
    fake_hs = types.SimpleNamespace(HostSimEngine=eng_mod.FlowEngine)
    body(fake_hs, so, seed)


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("heavy_min", [2, 512])
def test_heavy_thread_traces(eng_mod, so, seed, heavy_min):
    """THREAD-grade heavy segments: the wave kernel's Lindley fast path, the
    ballot path (in-window exits, acquireCount > 1) and the LDS pass ring."""
    from tests.test_hostsim_parity import thread_workload
    workloads.run(eng_mod.FlowEngine, so.OracleEngine, thread_workload(seed, heavy_min=heavy_min))


def test_heavy_thread_long_range(eng_mod, so):
    """Exits 0..3 s after their entries in a 600k-event single-resource
    segment: references beyond the 128 Ki-event LDS ring take the HBM path."""
    from tests.test_hostsim_parity import thread_workload
    w = thread_workload(7, R=1, n=600_000, max_rt=3000, gaps=(0,) * 99 + (1,), heavy_min=512)
    workloads.run(eng_mod.FlowEngine, so.OracleEngine, w)


def ms_block_thread_workload(seed, n_entry=200_000, duration=300, count=50.0, rt_mean=5.0):
    """One saturated THREAD-grade resource with the config-3 head's layout:
    every millisecond holds its entries, then the exits that fall due in it
    (so runs of entry-only windows end in a window whose live exits all follow
    its entries, then exit-only windows); acquireCount 1 (90 %), 2-5, and a
    few above 2^20 (the exact walk's int-wrap guard), two batches."""
    rng = np.random.default_rng(900 + seed)
    ts = np.sort(rng.integers(0, duration, n_entry)).astype(np.int64) + trace.T0
    acq = np.ones(n_entry, np.int32)
    multi = rng.random(n_entry) < 0.1
    acq[multi] = rng.integers(2, 6, int(multi.sum()))
    acq[rng.choice(n_entry, 8, replace=False)] = 1 << 21
    rt = np.floor(rng.exponential(rt_mean, n_entry)).astype(np.int64)
    ets = np.minimum(ts + rt, trace.T0 + duration - 1)
    all_ts = np.concatenate([ts, ets])
    isx = np.concatenate([np.zeros(n_entry, bool), np.ones(n_entry, bool)])
    order = np.lexsort((isx, all_ts))
    pos = np.empty(order.size, np.int64)
    pos[order] = np.arange(order.size)
    src = np.concatenate([np.arange(n_entry), np.arange(n_entry)])
    fl = np.where(isx[order], abi.EV_EXIT | abi.EV_IN, abi.EV_IN).astype(np.uint8)
    eref = np.full(order.size, -1, np.int64)
    eref[pos[n_entry:]] = pos[:n_entry]
    b = abi.HostBatch(np.zeros(order.size, np.uint32), all_ts[order], acq[src][order], fl, entry_ref=eref)
    rules = [abi.sf_flow_rule(resource=0, grade=abi.GRADE_THREAD, count=count, control_behavior=0)]
    k = b.n // 2
    return dict(cfg=abi.default_config(max_resources=1, max_batch=b.n), flow=rules,
                batches=[b.subset(0, k), b.subset(k, b.n)], nodes=[0], n_flow=1)


@pytest.mark.parametrize("seed", range(2))
def test_heavy_thread_ms_blocks(eng_mod, so, seed):
    """The saturated THREAD walk's merged step (skipped windows + a window
    whose live exits follow its entries + the exit-only run) against the
    oracle, on per-millisecond entry / exit blocks."""
    workloads.run(eng_mod.FlowEngine, so.OracleEngine, ms_block_thread_workload(seed))


@pytest.mark.parametrize("count,rt_mean,duration", [(50.0, 5.0, 300), (3.0, 2.0, 300), (5000.0, 20.0, 300),
                                                   (400.0, 0.3, 150), (80.0, 200.0, 400)])
def test_heavy_thread_runs(eng_mod, so, count, rt_mean, duration):
    """The THREAD walk's run mode (chunks of a few long runs of entries and of
    exits): saturated with a small and a tiny room, never saturated, exits in
    their entry's millisecond, and exits far beyond the LDS ring (the HBM
    live-exit bitmap) -- against the oracle, two batches."""
    workloads.run(eng_mod.FlowEngine, so.OracleEngine,
                  ms_block_thread_workload(7, n_entry=150_000, duration=duration, count=count, rt_mean=rt_mean))


def test_device_resident_batch(eng_mod, so):
    """Inputs already in HBM (the bench path): same verdicts as the host path."""
    w = workloads.config3(R=5000, n=200_000, seed=5, split=1)
    e = eng_mod.FlowEngine(w["cfg"])
    e.load_flow_rules(w["flow"])
    ora = so.OracleEngine(w["cfg"])
    ora.load_flow_rules(w["flow"])
    hb = w["batches"][0]
    db = eng_mod.DeviceBatch(e, hb)
    dv = eng_mod.DeviceVerdicts(e, hb.n, with_wait=True, with_rule=True)
    e.submit_device(db, dv)
    got = abi.HostVerdicts(hb.n)
    got.status, got.wait_ms, got.rule_idx = dv.status.numpy(), dv.wait_ms.numpy(), dv.rule_idx.numpy()
    parity.compare_verdicts(got, ora.submit(hb), "device batch")
    parity.compare_nodes(e, ora, w["nodes"])


@pytest.mark.parametrize("split", [2, 5])
def test_async_pipelined_batches(eng_mod, so, split):
    """sf_submit_async: batch k+1 is sorted while batch k is decided (two Work
    sets); every batch's verdicts, the node state and ENTRY_NODE equal the
    oracle's sequential replay."""
    w = workloads.config3(R=3000, n=240_000, seed=8, split=split)
    e = eng_mod.FlowEngine(w["cfg"])
    e.load_flow_rules(w["flow"])
    ora = so.OracleEngine(w["cfg"])
    ora.load_flow_rules(w["flow"])
    dbs = [eng_mod.DeviceBatch(e, hb) for hb in w["batches"]]
    dvs = [eng_mod.DeviceVerdicts(e, hb.n, with_wait=True, with_rule=True) for hb in w["batches"]]
    for db, dv in zip(dbs, dvs):
        e.submit_device_async(db, dv)
    e.sync()
    for k, (hb, dv) in enumerate(zip(w["batches"], dvs)):
        got = abi.HostVerdicts(hb.n)
        got.status, got.wait_ms, got.rule_idx = dv.status.numpy(), dv.wait_ms.numpy(), dv.rule_idx.numpy()
        parity.compare_verdicts(got, ora.submit(hb), f"async batch {k}")
    parity.compare_nodes(e, ora, w["nodes"])
    parity.compare_entry_node(e, ora)
    # a synchronous submit after the asynchronous ones continues the same state
    extra = workloads.config3(R=3000, n=20_000, seed=9, split=1, duration_ms=500)["batches"][0]
    shifted = abi.HostBatch(extra.res_id, extra.ts_ms + 6000, extra.count, extra.flags, entry_ref=extra.entry_ref)
    parity.compare_verdicts(e.submit(shifted), ora.submit(shifted), "sync after async")


def test_async_error_reported_at_sync(eng_mod):
    cfg = abi.default_config(max_resources=8, max_batch=16)
    e = eng_mod.FlowEngine(cfg)
    db = eng_mod.DeviceBatch(e, abi.HostBatch([9], [trace.T0], [1], [0]))   # resource outside the shard
    dv = eng_mod.DeviceVerdicts(e, 1)
    e.submit_device_async(db, dv)
    with pytest.raises(eng_mod.EngineError):
        e.sync()
    e.submit(abi.HostBatch([1], [trace.T0], [1], [0]))    # still usable


@pytest.mark.parametrize("kind", ["qps", "thread", "rt", "load", "cpu"])
def test_system_rule(eng_mod, so, kind):
    """SystemRuleManager.checkSystem on the global ENTRY_NODE (k_replay):
    verdicts (SF_V_BLOCK_SYSTEM with the reason in rule_idx), every node, the
    ENTRY_NODE and the controller states equal the oracle's."""
    w = workloads.system(kind)
    eng, ora, outs = workloads.run(eng_mod.FlowEngine, so.OracleEngine, w)
    blocked = sum(int((o[1].status == abi.V_BLOCK_SYSTEM).sum()) for o in outs)
    assert blocked > 0, "the SystemRule never fired: the workload does not exercise it"
    n = sum(b.n for b in w["batches"])
    assert 0 < eng.stats().sys_rounds < n // 4, eng.stats().sys_rounds   # planned sub-batches, not a replay


@pytest.mark.parametrize("kind", ["param", "param06", "mixed"])
def test_system_rule_large(eng_mod, so, kind):
    """SystemRules at scale through the planner: config 4's shape (2 Mi
    events, 1k resources, param rules, inbound QPS at 0.8x the offered rate)
    and config 3's traffic with QPS + thread + RT system rules over three
    batches; every verdict, the sampled nodes, ENTRY_NODE and the controller
    states equal the oracle's."""
    w = workloads.system_large(kind)
    eng, ora, outs = workloads.run(eng_mod.FlowEngine, so.OracleEngine, w)
    st = np.concatenate([o[1].status for o in outs])
    reasons = np.concatenate([o[1].rule_idx[o[1].status == abi.V_BLOCK_SYSTEM] for o in outs])
    assert (st == abi.V_BLOCK_SYSTEM).sum() > 1000, "the SystemRule barely fired"
    if kind == "mixed":
        assert set(np.unique(reasons)) >= {0, 1}, np.unique(reasons)
    n = sum(b.n for b in w["batches"])
    print(f"{kind}: {n} events, {eng.stats().sys_rounds} planner rounds, "
          f"{(st == abi.V_BLOCK_SYSTEM).sum()} system blocks, reasons {np.bincount(reasons)}")


@pytest.mark.parametrize("kind", ["qps", "thread", "rt", "load", "cpu", "mixed"])
def test_system_sharded_two_engines(eng_mod, so, kind):
    """SystemRules on a resource-sharded node (two engines on cuda:0, one per
    rank, in threads): the node-wide round protocol (system_shard.py:
    sf_system_plan / sf_submit_forced / sf_entry_node_add) gives the verdicts
    of one oracle replay of the whole node batch, and every rank's ENTRY_NODE
    equals the oracle's."""
    from tests import test_system_shard as ts
    w = workloads.system_large("mixed") if kind == "mixed" else workloads.system(kind)
    got, ens = ts.run_local_ranks(eng_mod.FlowEngine, w, w["batches"])
    ts.check_against_reference(w, w["batches"], got, ens)


def test_system_sharded_plain_submit_refused(eng_mod):
    """A sharded engine with SystemRules refuses sf_submit (ENTRY_NODE is node-wide)."""
    w = workloads.system("thread")
    cfg = abi.default_config(max_resources=w["cfg"].max_resources, max_batch=w["cfg"].max_batch,
                             shard_count=2, shard_index=0)
    e = eng_mod.FlowEngine(cfg)
    e.load_system_rules(list(w["system"]))
    b = w["batches"][0].shard(2, 0)
    with pytest.raises(RuntimeError, match="round protocol"):
        e.submit(b)


@pytest.mark.parametrize("seed,prio,heavy_min,system", [(11, 0.0, 512, False), (12, 0.2, 8, False),
                                                        (13, 0.0, 64, True), (14, 0.1, 512, True)])
def test_degrade_in_submit_chain(eng_mod, so, seed, prio, heavy_min, system):
    """DegradeSlot after FlowSlot inside sf_submit (DegradeSlot.java:42-94):
    verdicts, breaker states, nodes and ENTRY_NODE equal to the oracle's chain;
    with a SystemRule the planner's forced verdicts precede the breakers."""
    from tests import test_degrade_chain as tc
    cfg, flow, rules, b = tc.chain_workload(seed, prio=prio, n=60_000)
    cfg.heavy_min_events = heavy_min
    sysr = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=-1, avg_rt=-1,
                               max_thread=60)] if system else None
    cut = b.n // 3
    batches = [b.subset(0, cut), b.subset(cut, b.n)]
    e, got, n = tc.run_chain(eng_mod.FlowEngine, cfg, flow, rules, batches, sysr)
    o, want, n2 = tc.run_chain(so.OracleEngine, cfg, flow, rules, batches, sysr)
    assert n == n2
    for k, (g, w) in enumerate(zip(got, want)):
        parity.compare_verdicts(g, w, f"batch{k}")
    st = np.concatenate([w.status for w in want])
    assert (st == abi.V_BLOCK_DEGRADE).sum() > 0 and (st == abi.V_BLOCK_FLOW).sum() > 0
    if system:
        assert (st == abi.V_BLOCK_SYSTEM).sum() > 0
    assert np.array_equal(tc._breaker_rows(e, n), tc._breaker_rows(o, n))
    parity.compare_nodes(e, o, range(0, cfg.max_resources, 3), sample_count=cfg.sample_count)
    parity.compare_entry_node(e, o, sample_count=cfg.sample_count)


def test_config2_large_properties(eng_mod, so):
    """1M-event uniform batch: oracle parity plus the window invariant
    passes(hw) + passes(hw-1) <= count for every resource."""
    R, n = 50_000, 1_000_000
    counts = trace.uniform_rules(R, seed=31)
    rules = trace.flow_rules_from_counts(counts)
    b = trace.uniform_qps(R, n, seed=31)
    cfg = abi.default_config(max_resources=R, max_batch=n)
    e = eng_mod.FlowEngine(cfg)
    e.load_flow_rules(rules)
    v = e.submit(b)
    ora = so.OracleEngine(cfg)
    ora.load_flow_rules(rules)
    parity.compare_verdicts(v, ora.submit(b), "config2 1M")
    passed = v.status == abi.V_PASS
    hw = (b.ts_ms - trace.T0) // 500
    nh = int(hw.max()) + 1
    grid = np.zeros((R, nh), np.int64)
    np.add.at(grid, (b.res_id[passed], hw[passed]), 1)
    assert ((grid[:, 1:] + grid[:, :-1]) <= counts[:, None]).all()


def test_invalid_batches_rejected(eng_mod):
    cfg = abi.default_config(max_resources=8, max_batch=16)
    e = eng_mod.FlowEngine(cfg)
    b = abi.HostBatch([9], [trace.T0], [1], [0])           # resource outside the shard
    with pytest.raises(eng_mod.EngineError):
        e.submit(b)
    b = abi.HostBatch(np.zeros(17, np.uint32), np.full(17, trace.T0), np.ones(17), np.zeros(17))
    with pytest.raises(eng_mod.EngineError):
        e.submit(b)
    e.submit(abi.HostBatch([1], [trace.T0], [1], [0]))    # still usable


def test_entry_node_and_snapshot(eng_mod, so):
    """ENTRY_NODE (all IN traffic) and the per-second MetricNode snapshot
    (StatisticNode.metrics via MetricTimerListener), twice across batches so
    lastFetchTime and the currentWindow(now) side effect are exercised."""
    w = workloads.config3(R=3000, n=120_000, seed=23, split=3, duration_ms=9000)
    e, o = eng_mod.FlowEngine(w["cfg"]), so.OracleEngine(w["cfg"])
    for x in (e, o):
        x.load_flow_rules(w["flow"])
    for k, b in enumerate(w["batches"]):
        parity.compare_verdicts(e.submit(b), o.submit(b), f"batch {k}")
        parity.compare_entry_node(e, o, what=f"batch {k}")
        now = int(b.ts_ms[-1]) + 1
        got, want = parity.metric_rows(e.snapshot(now)), parity.metric_rows(o.snapshot(now))
        assert got == want, f"snapshot after batch {k}: {len(got)} vs {len(want)} rows"
    parity.compare_nodes(e, o, w["nodes"])


def test_entry_node_rccl_single_rank(eng_mod, so):
    """The RCCL node-wide merge on a one-rank communicator is the identity."""
    w = workloads.config3(R=2000, n=60_000, seed=29, split=2)
    e = eng_mod.FlowEngine(w["cfg"])
    e.load_flow_rules(w["flow"])
    for b in w["batches"]:
        e.submit(b)
    e.comm_init(1, 0, eng_mod.comm_unique_id())
    got = abi.node_state_to_dict(e.entry_node_allreduce())
    want = abi.node_state_to_dict(e.read_entry_node())
    assert got == want


def test_metric_log_matches_oracle(eng_mod, so):
    """metrics.log on the GPU (sf_metric_log: MetricTimerListener.run ->
    MetricWriter.write -> MetricNode.toFatString) byte for byte against the
    oracle: several fetches across batches (lastFetchTime, the current-second
    exclusion, ENTRY_NODE last in each second), names with '|', resource types,
    a resource without a name, UTC+8 dates."""
    w = workloads.config3(R=3000, n=120_000, seed=31, split=3, duration_ms=9000)
    e, o = eng_mod.FlowEngine(w["cfg"]), so.OracleEngine(w["cfg"])
    R = w["cfg"].max_resources
    names = [f"/svc/{r}|op" if r % 7 == 0 else f"res-{r}" for r in range(R - 5)]   # the last 5 unnamed
    types = [r % 5 for r in range(R - 5)]
    e.load_resource_names(names, types)
    tz = 8 * 3600 * 1000
    for x in (e, o):
        x.load_flow_rules(w["flow"])
    for k, b in enumerate(w["batches"]):
        parity.compare_verdicts(e.submit(b), o.submit(b), f"batch {k}")
        for now in (int(b.ts_ms[-1]) + 1, int(b.ts_ms[-1]) + 1700):
            got = e.metric_log(now, tz_offset_ms=tz)
            want = o.metric_log(now, names=names, types=types, tz_offset_ms=tz)
            assert got == want, f"metric log after batch {k} at {now}: {len(got)} vs {len(want)} bytes"
            assert k > 0 or len(got) > 0
    assert e.metric_log(int(w["batches"][-1].ts_ms[-1]) + 1700, tz_offset_ms=tz) == b""   # nothing new
    parity.compare_nodes(e, o, w["nodes"])


def test_node_wide_metric_log_two_shards(eng_mod, so):
    """Two resource shards (two engines on cuda:0): every shard's ENTRY_NODE
    merged on the host (sentinel_amd.dist.merge_entry_nodes, the merge the
    RCCL all-reduce does), set as the reported ENTRY_NODE of shard 0
    (sf_set_report_entry_node); the merged metrics.log of the two shards
    (lines per second, ENTRY_NODE last, MetricTimerListener.java:40-69) equals
    one oracle engine's over the whole batch."""
    from sentinel_amd import dist as sd
    R = 3000
    rules = trace.mixed_rules(R, seed=33)
    full = trace.mixed_zipf(R, 120_000, duration_ms=6000, seed=33)
    engs = []
    for k in range(2):
        sub = full.shard(2, k)
        e = eng_mod.FlowEngine(abi.default_config(max_resources=R // 2, max_batch=sub.n, shard_count=2, shard_index=k))
        e.load_flow_rules([r for r in rules if r.resource % 2 == k])
        e.submit(sub)
        engs.append(e)
    ref = so.OracleEngine(abi.default_config(max_resources=R, max_batch=full.n))
    ref.load_flow_rules(rules)
    ref.submit(full)
    t_end = int(full.ts_ms[-1])
    for now in (t_end - 2500, t_end + 1500):
        merged = sd.merge_entry_nodes([e.read_entry_node() for e in engs])
        engs[0].set_report_entry_node(merged)
        parts = [engs[0].metric_log(now, entry_node=True), engs[1].metric_log(now, entry_node=False)]
        got = sd.merge_metric_logs(parts)
        want = ref.metric_log(now, entry_node=True)
        g, w = {}, {}
        for log, d in ((got, g), (want, w)):
            for line in log.split(b"\n"):
                if line:
                    d.setdefault(int(line.split(b"|")[0]), []).append(line)
        assert sorted(g) == sorted(w) and len(w) > 0
        for sec in w:
            assert g[sec][-1] == w[sec][-1] and b"__total_inbound_traffic__" in w[sec][-1]
            assert sorted(g[sec]) == sorted(w[sec])
        engs[0].set_report_entry_node(None)


def test_format_metric_rows_kat(eng_mod, so):
    """MetricNodeTest.java:29-36 fat line, formatted by the GPU kernel, and
    the formatter on edge values against the oracle's."""
    from sentinel_amd import abi as A
    e = eng_mod.FlowEngine(abi.default_config(max_resources=16))
    e.load_resource_names(["/foo/*", "a|b"], [1, 2])
    r = A.sf_metric_row(resource=0, concurrency=2, timestamp=1564382218000, pass_qps=1, success_qps=1)
    assert e.format_metric_rows([r], tz_offset_ms=8 * 3600 * 1000) == \
        b"1564382218000|2019-07-29 14:36:58|/foo/*|1|0|1|0|0|0|2|1\n"
    rows = [A.sf_metric_row(resource=res, timestamp=ts, pass_qps=p, block_qps=-p, rt=(1 << 63) - 1 - p)
            for res, ts, p in [(1, -1, 0), (0, 951868799999, 7), (A.RES_ENTRY_NODE, 253402300799000, -3),
                               (12, 0, 1 << 40), (1, -2208988800000, 9)]]
    got = e.format_metric_rows(rows, tz_offset_ms=-5 * 3600 * 1000)
    want = so.format_fat(rows, names=["/foo/*", "a|b"], types=[1, 2], tz_offset_ms=-5 * 3600 * 1000)
    assert got == want


@pytest.mark.parametrize("n", [1_500_007, 5_000_011])
def test_bucketed_verdict_scatter(eng_mod, so, n):
    """Batches above the direct-scatter size (2^20): the statuses go from
    sorted order to submission order in bucketed passes (A + C at 1.5M
    events, A + B + C above 2^22); every verdict, wait and rule index equals
    the oracle's, and so do the nodes."""
    w = workloads.config3(R=100_000, n=n, seed=41, split=1)
    workloads.run(eng_mod.FlowEngine, so.OracleEngine, w)
