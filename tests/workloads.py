"""Seeded parity workloads shared by the CPU (hostsim) and GPU parity suites.

Each builder returns a dict: cfg, flow (rules), param (rules), items, batches,
nodes (resources whose full node state is compared) and n_flow.
"""
import numpy as np

from sentinel_amd import abi, trace


def config1(duration_ms=20_000):
    rules, batch = trace.flow_qps_demo(duration_ms=duration_ms)
    return dict(cfg=abi.default_config(max_resources=4, max_batch=batch.n), flow=rules, batches=[batch],
                nodes=[0])


def config2(R=500, n=60_000, seed=2):
    rules = trace.flow_rules_from_counts(trace.uniform_rules(R, seed=seed))
    batch = trace.uniform_qps(R, n, seed=seed)
    return dict(cfg=abi.default_config(max_resources=R, max_batch=batch.n), flow=rules, batches=[batch],
                nodes=list(range(0, R, 7)))


def config3(R=2000, n=80_000, seed=3, split=2, duration_ms=6000):
    rules = trace.mixed_rules(R, seed=seed)
    full = trace.mixed_zipf(R, n, duration_ms=duration_ms, seed=seed)
    cuts = np.linspace(0, full.n, split + 1).astype(int)
    batches = [full.subset(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:])]
    hot = np.argsort(-np.bincount(full.res_id, minlength=R))[:50]
    return dict(cfg=abi.default_config(max_resources=R, max_batch=full.n), flow=rules, batches=batches,
                nodes=sorted(set(int(x) for x in hot) | set(range(0, R, 37))), n_flow=len(rules))


def config4(R=40, n=50_000, keys=5000, seed=4):
    rules, batch = trace.param_zipf(R, n, keys, seed=seed)
    return dict(cfg=abi.default_config(max_resources=R, max_batch=batch.n, param_capacity=1 << 17),
                param=rules, batches=[batch], nodes=list(range(R)))


def prioritized(seed=9, R=20, n=20000):
    rng = np.random.default_rng(seed)
    rules = trace.flow_rules_from_counts(rng.integers(2, 8, R))
    ts = np.sort(rng.integers(0, 5000, n)) + trace.T0
    res = rng.integers(0, R, n).astype(np.uint32)
    flags = np.where(rng.random(n) < 0.5, abi.EV_PRIO, 0).astype(np.uint8) | abi.EV_IN
    cnt = rng.integers(1, 3, n).astype(np.int32)
    ent = np.arange(0, n, 3)
    ex_ts = ts[ent] + rng.integers(0, 30, ent.size)
    all_ts = np.concatenate([ts, ex_ts])
    key = np.lexsort((np.concatenate([np.zeros(n), np.ones(ent.size)]), all_ts))
    pos = np.empty(key.size, np.int64)
    pos[key] = np.arange(key.size)
    src = np.concatenate([np.arange(n), ent])
    err = np.where(rng.random(ent.size) < 0.2, abi.EV_ERROR, 0)
    fl = np.concatenate([flags, (abi.EV_EXIT | abi.EV_IN | err).astype(np.uint8)])
    eref = np.full(key.size, -1, np.int64)
    eref[pos[n:]] = pos[ent]
    b = abi.HostBatch(res[src][key], all_ts[key], cnt[src][key], fl[key], entry_ref=eref)
    return dict(cfg=abi.default_config(max_resources=R, max_batch=b.n), flow=rules, batches=[b],
                nodes=list(range(R)))


def multi_rule(seed=12, R=30, n=30000):
    rng = np.random.default_rng(seed)
    rules = []
    for r in range(R):
        for _ in range(int(rng.integers(1, 4))):
            beh = int(rng.integers(0, 4))
            grade = abi.GRADE_THREAD if (beh == 0 and rng.random() < 0.3) else abi.GRADE_QPS
            rules.append(abi.sf_flow_rule(resource=r, grade=grade, count=float(rng.integers(1, 40)), strategy=0,
                                          control_behavior=beh if grade == abi.GRADE_QPS else 0,
                                          warm_up_period_sec=int(rng.integers(1, 6)),
                                          max_queueing_time_ms=int(rng.integers(1, 800))))
    ts = np.sort(rng.integers(0, 8000, n)) + trace.T0
    res = rng.integers(0, R, n).astype(np.uint32)
    b = abi.HostBatch(res, ts, rng.integers(1, 4, n).astype(np.int32), np.full(n, abi.EV_IN, np.uint8))
    return dict(cfg=abi.default_config(max_resources=R, max_batch=n), flow=rules, batches=[b],
                nodes=list(range(R)), n_flow=len(rules))


def geometry(sample_count, interval, R=50, n=20_000):
    rules = trace.flow_rules_from_counts(trace.uniform_rules(R, seed=7))
    batch = trace.uniform_qps(R, n, seed=7)
    return dict(cfg=abi.default_config(max_resources=R, max_batch=batch.n, sample_count=sample_count,
                                       interval_ms=interval), flow=rules, batches=[batch], nodes=list(range(R)))


def param_mixed(seed=21, R=12, n=30000):
    """Param rules: QPS default with burst/duration/hot items, throttle, THREAD grade
    with exits, several args, negative paramIdx, null values."""
    rng = np.random.default_rng(seed)
    items, prules = [], []
    for r in range(R):
        kinds = rng.choice(4, size=int(rng.integers(1, 3)), replace=False)
        for k in kinds:
            off = len(items)
            for v in rng.choice(50, size=2, replace=False):
                items.append(abi.sf_hot_item(tag=abi.TAG_LONG, count=int(rng.integers(0, 6)), bits=int(v)))
            pidx = int(rng.choice([0, 1, -1]))
            if k == 0:
                prules.append(abi.sf_param_rule(resource=r, grade=abi.GRADE_QPS, param_idx=pidx, control_behavior=0,
                                                count=float(rng.integers(1, 10)), burst_count=int(rng.integers(0, 4)),
                                                duration_in_sec=int(rng.integers(1, 3)), item_offset=off, item_count=2))
            elif k == 1:
                prules.append(abi.sf_param_rule(resource=r, grade=abi.GRADE_QPS, param_idx=pidx, control_behavior=2,
                                                count=float(rng.integers(1, 20)), max_queueing_time_ms=int(rng.integers(0, 300)),
                                                duration_in_sec=1, item_offset=off, item_count=2))
            else:
                prules.append(abi.sf_param_rule(resource=r, grade=abi.GRADE_THREAD, param_idx=pidx, control_behavior=0,
                                                count=float(rng.integers(1, 5)), duration_in_sec=1,
                                                item_offset=off, item_count=2))
    flow = [abi.sf_flow_rule(resource=r, grade=abi.GRADE_QPS, count=float(rng.integers(3, 30)), strategy=0,
                             control_behavior=0, warm_up_period_sec=10, max_queueing_time_ms=500) for r in range(0, R, 2)]
    ts = np.sort(rng.integers(0, 6000, n)) + trace.T0
    res = rng.integers(0, R, n).astype(np.uint32)
    tag = np.full((2, n), abi.TAG_LONG, np.uint8)
    tag[rng.random((2, n)) < 0.05] = abi.TAG_NULL
    bits = rng.integers(0, 50, (2, n)).astype(np.uint64)
    nargs = rng.integers(0, 3, n).astype(np.uint8)
    ent = np.arange(0, n, 2)
    ex_ts = ts[ent] + rng.integers(0, 100, ent.size)
    all_ts = np.concatenate([ts, ex_ts])
    key = np.lexsort((np.concatenate([np.zeros(n), np.ones(ent.size)]), all_ts))
    pos = np.empty(key.size, np.int64)
    pos[key] = np.arange(key.size)
    src = np.concatenate([np.arange(n), ent])
    fl = np.concatenate([np.full(n, abi.EV_IN, np.uint8), np.full(ent.size, abi.EV_EXIT | abi.EV_IN, np.uint8)])
    eref = np.full(key.size, -1, np.int64)
    eref[pos[n:]] = pos[ent]
    b = abi.HostBatch(res[src][key], all_ts[key], np.ones(key.size, np.int32), fl[key], entry_ref=eref,
                      arg_tag=tag[:, src][:, key], arg_bits=bits[:, src][:, key], n_args=nargs[src][key])
    return dict(cfg=abi.default_config(max_resources=R, max_batch=b.n, param_capacity=1 << 14), flow=flow,
                param=prules, items=items, batches=[b], nodes=list(range(R)), n_flow=len(flow))


def param_collections(seed=31, R=10, n=20000):
    """Param rules (QPS default with burst / hot items, throttle, THREAD grade)
    over arguments that are scalars, nulls, or Collections / arrays of 0-4
    elements (some null); exits carry their entry's arguments."""
    rng = np.random.default_rng(seed)
    items, prules = [], []
    for r in range(R):
        for k in rng.choice(3, size=int(rng.integers(1, 3)), replace=False):
            off = len(items)
            for v in rng.choice(30, size=2, replace=False):
                items.append(abi.sf_hot_item(tag=abi.TAG_LONG, count=int(rng.integers(0, 6)), bits=int(v)))
            pidx = int(rng.choice([0, 1]))
            if k == 0:
                prules.append(abi.sf_param_rule(resource=r, grade=abi.GRADE_QPS, param_idx=pidx, control_behavior=0,
                                                count=float(rng.integers(1, 12)), burst_count=int(rng.integers(0, 3)),
                                                duration_in_sec=1, item_offset=off, item_count=2))
            elif k == 1:
                prules.append(abi.sf_param_rule(resource=r, grade=abi.GRADE_QPS, param_idx=pidx, control_behavior=2,
                                                count=float(rng.integers(2, 30)),
                                                max_queueing_time_ms=int(rng.integers(0, 200)),
                                                duration_in_sec=1, item_offset=off, item_count=2))
            else:
                prules.append(abi.sf_param_rule(resource=r, grade=abi.GRADE_THREAD, param_idx=pidx, control_behavior=0,
                                                count=float(rng.integers(1, 6)), duration_in_sec=1,
                                                item_offset=off, item_count=2))
    flow = [abi.sf_flow_rule(resource=r, grade=abi.GRADE_QPS, count=float(rng.integers(20, 60)), strategy=0,
                             control_behavior=0, warm_up_period_sec=10, max_queueing_time_ms=500) for r in range(0, R, 3)]
    ts = np.sort(rng.integers(0, 5000, n)) + trace.T0
    res = rng.integers(0, R, n).astype(np.uint32)

    def value():
        u = rng.random()
        if u < 0.05:
            return None
        if u < 0.7:
            return (abi.TAG_LONG, int(rng.integers(0, 30)))
        return [None if rng.random() < 0.05 else (abi.TAG_LONG, int(rng.integers(0, 30)))
                for _ in range(int(rng.integers(0, 5)))]
    vals = [[value() for _ in range(n)] for _ in range(2)]
    ent = np.arange(0, n, 2)                               # half of the entries exit after 0-80 ms
    ex_ts = ts[ent] + rng.integers(0, 80, ent.size)
    all_ts = np.concatenate([ts, ex_ts])
    key = np.lexsort((np.concatenate([np.zeros(n), np.ones(ent.size)]), all_ts))
    pos = np.empty(key.size, np.int64)
    pos[key] = np.arange(key.size)
    src = np.concatenate([np.arange(n), ent])[key]
    m = key.size
    at, ab, off, et, eb = abi.HostBatch.collections(2, m, [[vals[a][int(s)] for s in src] for a in range(2)])
    fl = np.concatenate([np.full(n, abi.EV_IN, np.uint8), np.full(ent.size, abi.EV_EXIT | abi.EV_IN, np.uint8)])[key]
    eref = np.full(m, -1, np.int64)
    eref[pos[n:]] = pos[ent]
    nargs = rng.integers(1, 3, n).astype(np.uint8)[src]
    b = abi.HostBatch(res[src], all_ts[key], np.ones(m, np.int32), fl, entry_ref=eref, arg_tag=at, arg_bits=ab,
                      n_args=nargs, elem_off=off, elem_tag=et, elem_bits=eb)
    cuts = [0, m // 2, m]
    return dict(cfg=abi.default_config(max_resources=R, max_batch=m, param_capacity=1 << 14), flow=flow,
                param=prules, items=items, batches=[b.subset(cuts[0], cuts[1]), b.subset(cuts[1], cuts[2])],
                nodes=list(range(R)), n_flow=len(flow))


def system(kind, seed=41):
    """SystemRule over mixed traffic (SystemRuleManager.checkSystem, global
    ENTRY_NODE): config 4's inbound-QPS rule at 0.8x the offered rate, or the
    thread / RT / load (BBR) / cpu thresholds over THREAD-grade traffic with
    exits.  Decided on the GPU as planned safe sub-batches (sf_system.h)."""
    rng = np.random.default_rng(seed)
    if kind == "qps":
        rules, batch = trace.param_zipf(30, 40_000, 3000, duration_ms=4000, seed=seed)
        offered = batch.n / 4.0                             # inbound events per second
        sysr = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=0.8 * offered,
                                   avg_rt=-1, max_thread=-1)]
        return dict(cfg=abi.default_config(max_resources=30, max_batch=batch.n, param_capacity=1 << 16),
                    param=rules, batches=[batch], nodes=list(range(30)), system=sysr, status=(0.0, 0.0))
    R = 60
    full = trace.mixed_zipf(R, 30_000, duration_ms=3000, seed=seed)
    rules = trace.mixed_rules(R, seed=seed)
    thr = {"thread": (-1.0, -1.0, -1.0, -1, 4000), "rt": (-1.0, -1.0, -1.0, 15, -1),
           "load": (0.5, -1.0, -1.0, -1, -1), "cpu": (-1.0, 0.6, -1.0, -1, -1)}[kind]
    status = {"load": (2.0, 0.1), "cpu": (0.3, 0.9)}.get(kind, (0.0, 0.0))
    sysr = [abi.sf_system_rule(highest_system_load=thr[0], highest_cpu_usage=thr[1], qps=thr[2],
                               avg_rt=thr[3], max_thread=thr[4])]
    cuts = np.linspace(0, full.n, 3).astype(int)
    batches = [full.subset(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:])]
    return dict(cfg=abi.default_config(max_resources=R, max_batch=full.n), flow=rules, batches=batches,
                nodes=list(range(R)), n_flow=len(rules), system=sysr, status=status)


def system_large(kind, seed=43):
    """SystemRule at scale: "param" = config 4's shape (uniform resources with
    QPS / throttle ParamFlowRules, Zipf(1.1) keys) with the inbound-QPS rule at
    ``frac`` x the offered rate; "mixed" = config 3's traffic (flow rules of all
    four controllers, THREAD exits, acquireCount 1-5) with an inbound-QPS rule
    and a thread rule that both fire; three batches."""
    if kind in ("param", "param06"):
        # param06: the inbound-QPS rule at 0.6x, where it fires between the
        # ParamFlow blocks (the planner's inert entries, sf_system.h)
        R, n = 1000, 1 << 21
        rules, batch = trace.param_zipf(R, n, 200_000, duration_ms=4000, seed=seed)
        frac = 0.8 if kind == "param" else 0.6
        sysr = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=frac * n / 4.0,
                                   avg_rt=-1, max_thread=-1)]
        return dict(cfg=abi.default_config(max_resources=R, max_batch=batch.n, param_capacity=1 << 22),
                    param=rules, batches=[batch], nodes=list(range(0, R, 9)), system=sysr, status=(0.0, 0.0))
    R = 5000
    full = trace.mixed_zipf(R, 600_000, duration_ms=6000, seed=seed)
    rules = trace.mixed_rules(R, seed=seed)
    sysr = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=0.35 * full.n / 6.0,
                               avg_rt=-1, max_thread=60_000),
            abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=-1, avg_rt=21, max_thread=-1)]
    cuts = np.linspace(0, full.n, 4).astype(int)
    batches = [full.subset(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:])]
    hot = np.argsort(-np.bincount(full.res_id, minlength=R))[:40]
    return dict(cfg=abi.default_config(max_resources=R, max_batch=full.n), flow=rules, batches=batches,
                nodes=sorted(set(int(x) for x in hot) | set(range(0, R, 97))), n_flow=len(rules), system=sysr,
                status=(0.0, 0.0))


def xflow(seed=51, R=400, n=60_000, origins=6, contexts=4, duration_ms=6000, zipf=1.1, split=2):
    """Flow rules that read other nodes (FlowRuleChecker.selectNodeByRequesterAndStrategy):
    origin-specific and "other" limitApps (origin nodes), RELATE (another
    resource's ClusterNode, chains and self references included), CHAIN
    (the DefaultNode of a context), cluster rules with / without fallback,
    beside plain rules.  Events carry origins (some "", some the strings
    "default" / "other") and context names; prioritized entries; THREAD exits
    carry their entry's context."""
    rng = np.random.default_rng(seed)
    O0 = 2                                                   # origin ids >= 2 are names
    rules = []

    def rule(r, **kw):
        beh = int(kw.pop("beh", rng.choice([0, 0, 1, 2, 3])))
        grade = kw.pop("grade", abi.GRADE_THREAD if (beh == 0 and rng.random() < 0.25) else abi.GRADE_QPS)
        rules.append(abi.sf_flow_rule(resource=r, grade=grade, count=float(kw.pop("count", rng.integers(1, 30))),
                                      strategy=kw.pop("strategy", 0),
                                      control_behavior=beh if grade == abi.GRADE_QPS else 0,
                                      warm_up_period_sec=int(rng.integers(1, 5)),
                                      max_queueing_time_ms=int(rng.integers(1, 600)), **kw))
    for r in range(R):
        u = rng.random()
        if u < 0.4:
            rule(r)
        elif u < 0.55:                                       # origin-specific (+ a default rule)
            for _ in range(int(rng.integers(1, 3))):
                rule(r, limit_app=int(rng.integers(O0, O0 + origins)))
            if rng.random() < 0.5:
                rule(r)
        elif u < 0.65:                                       # "other" beside a specific origin
            rule(r, limit_app=int(rng.integers(O0, O0 + origins)))
            rule(r, limit_app=abi.APP_OTHER)
        elif u < 0.78:                                       # RELATE
            refs = [r, int(rng.integers(0, R)), int(rng.integers(0, R)), R + 5, abi.REF_NONE]
            rule(r, strategy=abi.STRATEGY_RELATE, ref_resource=refs[int(rng.integers(0, len(refs)))],
                 limit_app=int(rng.choice([abi.APP_DEFAULT, abi.APP_DEFAULT, O0])))
        elif u < 0.88:                                       # CHAIN on a context
            rule(r, strategy=abi.STRATEGY_CHAIN, ref_resource=int(rng.integers(0, contexts)))
            if rng.random() < 0.4:
                rule(r)
        elif u < 0.94:                                       # cluster rule, ClusterStateManager not started
            rule(r, cluster_mode=1, cluster_fallback=int(rng.random() < 0.5))
        # else: no rule (may still be a RELATE target)
    # events: Zipf resources, contexts, origins; THREAD exits
    w = 1.0 / np.arange(1, R + 1) ** zipf
    perm_r = rng.permutation(R)
    res = perm_r[rng.choice(R, size=n, p=w / w.sum())].astype(np.uint32)
    ts = np.sort(rng.integers(0, duration_ms, n)) + trace.T0
    og = rng.integers(0, O0 + origins + 1, n).astype(np.uint32)
    og[rng.random(n) < 0.3] = abi.ORIGIN_NONE
    cx = rng.integers(0, contexts, n).astype(np.uint32)
    cnt = np.where(rng.random(n) < 0.85, 1, rng.integers(2, 4, n)).astype(np.int32)
    flags = (np.where(rng.random(n) < 0.1, abi.EV_PRIO, 0) | abi.EV_IN).astype(np.uint8)
    ent = np.nonzero(rng.random(n) < 0.4)[0]
    ex_ts = ts[ent] + rng.integers(0, 60, ent.size)
    all_ts = np.concatenate([ts, ex_ts])
    key = np.lexsort((np.concatenate([np.zeros(n), np.ones(ent.size)]), all_ts))
    pos = np.empty(key.size, np.int64)
    pos[key] = np.arange(key.size)
    src = np.concatenate([np.arange(n), ent])
    err = np.where(rng.random(ent.size) < 0.2, abi.EV_ERROR, 0)
    fl = np.concatenate([flags, (abi.EV_EXIT | abi.EV_IN | err).astype(np.uint8)])
    eref = np.full(key.size, -1, np.int64)
    eref[pos[n:]] = pos[ent]
    full = abi.HostBatch(res[src][key], all_ts[key], cnt[src][key], fl[key], entry_ref=eref,
                         origin=og[src][key], context=cx[src][key])
    cuts = np.linspace(0, full.n, split + 1).astype(int)
    batches = [full.subset(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:])]
    # every entry with an origin has its origin node (ClusterBuilderSlot.java:107-110);
    # context nodes are kept for the CHAIN rules that read them
    has_o = full.origin != abi.ORIGIN_NONE
    pairs = np.unique(full.res_id[has_o].astype(np.uint64) << np.uint64(32) | full.origin[has_o].astype(np.uint64))
    on = {(int(p >> np.uint64(32)), int(p & np.uint64(0xffffffff))) for p in pairs}
    dn = set()
    for r in rules:
        sel = full.res_id == r.resource
        if r.strategy == abi.STRATEGY_CHAIN and np.any(full.context[sel] == r.ref_resource):
            dn.add((int(r.ref_resource), int(r.resource)))
    n_valid = sum(1 for r in rules if not (r.grade == abi.GRADE_QPS and r.strategy in (1, 2) and
                                            r.ref_resource == abi.REF_NONE))   # checkStrategyField
    return dict(cfg=abi.default_config(max_resources=R, max_batch=full.n, aux_capacity=max(4096, 2 * (len(on) + len(dn)))),
                flow=rules, batches=batches, nodes=list(range(R)), n_flow=n_valid, origin_nodes=sorted(on),
                context_nodes=sorted(dn))


def long_run(R=20_000, n=1_400_000, duration_ms=70_000, batches=7, seed=61):
    """Config 3's traffic over 70 s of trace time in 7 batches: light lane
    walks (most resources see tens of events) across the minute-window wrap
    (buckets reused after 60 s), WarmUp token state, RateLimiter
    latestPassedTime and THREAD exits carried across batches."""
    rules = trace.mixed_rules(R, seed=seed)
    full = trace.mixed_zipf(R, n, duration_ms=duration_ms, seed=seed)
    cuts = np.linspace(0, full.n, batches + 1).astype(int)
    bl = [full.subset(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:])]
    hot = np.argsort(-np.bincount(full.res_id, minlength=R))[:40]
    return dict(cfg=abi.default_config(max_resources=R, max_batch=max(b.n for b in bl)), flow=rules, batches=bl,
                nodes=sorted(set(int(x) for x in hot) | set(range(0, R, 53))), n_flow=len(rules))


def preblocked(w, frac=0.05, seed=0):
    """The workload with a fraction of its entries flagged SF_EV_BLOCKED: blocked
    by AuthoritySlot, which StatisticSlot wraps (StatisticSlot.java:102-124)
    but the engine does not run.  Each such entry is a block on its resource's
    ClusterNode and ENTRY_NODE that no rule sees; its exit records nothing.
    Entries are picked by a hash of (resource, time), so an exit in a later
    batch (entry_ref -1, create_ts) knows its entry was blocked and carries
    entry_ref -2 as a caller would."""
    thr = np.uint64(int(frac * (1 << 20)))

    def pick(res, ts):
        h = (res.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15) ^ ts.astype(np.uint64) * np.uint64(0xC2B2AE3D27D4EB4F)
             ^ np.uint64((seed * 0x165667B19E3779F9 + 1) % (1 << 64)))
        h ^= h >> np.uint64(29)
        h *= np.uint64(0xBF58476D1CE4E5B9)
        h ^= h >> np.uint64(32)
        return (h & np.uint64((1 << 20) - 1)) < thr

    for b in w["batches"]:
        b.flags = b.flags.copy()
        ent = (b.flags & abi.EV_EXIT) == 0
        b.flags[ent & pick(b.res_id, b.ts_ms)] |= abi.EV_BLOCKED
        if b.entry_ref is not None and b.create_ts is not None:
            early = ~ent & (b.entry_ref == -1)
            dead = early & pick(b.res_id, b.create_ts)
            if dead.any():
                b.entry_ref = b.entry_ref.copy()
                b.entry_ref[dead] = -2
    return w


ALL = {
    "config1": config1, "config2": config2, "config3": config3, "config4": config4,
    "prioritized": prioritized, "multi_rule": multi_rule, "param_mixed": param_mixed,
    "param_collections": param_collections,
    "geom_S1": lambda: geometry(1, 1000), "geom_S4": lambda: geometry(4, 1000), "geom_S10": lambda: geometry(10, 2000),
}


def run(make_engine, make_oracle, w):
    from tests import parity
    eng, ora, outs = parity.run_both(make_engine, make_oracle, w["cfg"], flow_rules=w.get("flow", ()),
                                     param_rules=w.get("param", ()), items=w.get("items", ()),
                                     batches=w["batches"], system=w.get("system", ()),
                                     status=w.get("status"))
    for k, (a, b) in enumerate(outs):
        parity.compare_verdicts(a, b, f"batch{k}")
    parity.compare_nodes(eng, ora, w["nodes"], sample_count=w["cfg"].sample_count)
    if hasattr(eng, "node_digests"):           # every row, not only the sampled ones
        parity.compare_all_nodes(eng, ora, w["cfg"].max_resources, sample_count=w["cfg"].sample_count)
        if w.get("n_flow"):
            parity.compare_all_rule_states(eng, ora, w["n_flow"])
    if getattr(eng, "has_entry_node", False):
        parity.compare_entry_node(eng, ora, sample_count=w["cfg"].sample_count)
    if w.get("n_flow"):
        parity.compare_rule_states(eng, ora, w["n_flow"])
    parity.compare_aux_nodes(eng, ora, w.get("origin_nodes", ()), w.get("context_nodes", ()),
                             sample_count=w["cfg"].sample_count)
    return eng, ora, outs
