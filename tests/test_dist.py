"""Node-wide ENTRY_NODE over resource shards (sentinel_amd.dist): two ranks
on the gloo backend, each replaying its shard of a config-3 batch with the
oracle (the GPU engine's ENTRY_NODE is pinned to the oracle by the GPU parity
suite); the all-reduced node must equal the ENTRY_NODE of one replay of the
whole batch.  CPU only (world size 2, 127.0.0.1)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from sentinel_amd import abi, trace


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from oracle import oracle as so
    from sentinel_amd import dist as sd
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R = 1500
    rules = trace.mixed_rules(R, seed=31)
    full = trace.mixed_zipf(R, 60_000, duration_ms=7000, seed=31)
    sub = full.shard(world, rank)
    cfg = abi.default_config(max_resources=(R + world - 1) // world, max_batch=max(sub.n, 1), shard_count=world,
                             shard_index=rank)
    o = so.OracleEngine(cfg)
    o.load_flow_rules([r for r in rules if r.resource % world == rank])
    half = sub.n // 2
    o.submit(sub.subset(0, half))
    o.submit(sub.subset(half, sub.n))
    merged = sd.entry_node_allreduce(o.read_entry_node())
    rows = sd.gather_snapshot(o.snapshot(int(full.ts_ms[-1]) + 1))
    if rank == 0:
        ref = so.OracleEngine(abi.default_config(max_resources=R, max_batch=full.n))
        ref.load_flow_rules(rules)
        h = full.n // 2
        ref.submit(full.subset(0, h))
        ref.submit(full.subset(h, full.n))
        from tests import parity
        want_rows = parity.metric_rows(ref.snapshot(int(full.ts_ms[-1]) + 1))
        q.put((abi.node_state_to_dict(merged), abi.node_state_to_dict(ref.read_entry_node()), rows, want_rows))
    dist.destroy_process_group()


def test_entry_node_allreduce_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, want, rows, want_rows = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k in want:
        assert got[k] == want[k], f"ENTRY_NODE field {k}:\n merged={got[k]}\n single={want[k]}"
    assert rows == want_rows


def _metric_worker(rank, world, port, q):
    """Node-wide metrics.log: every rank's engine holds its shard; the
    all-reduced ENTRY_NODE is set as the reported one on rank 0
    (sf_set_report_entry_node), every rank writes its shard's lines, and the
    merged log (lines per second, ENTRY_NODE last) equals one engine's log over
    the whole batch."""
    import torch.distributed as dist
    from oracle import oracle as so
    from sentinel_amd import dist as sd
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R = 1200
    rules = trace.mixed_rules(R, seed=37)
    full = trace.mixed_zipf(R, 50_000, duration_ms=5000, seed=37)
    sub = full.shard(world, rank)
    cfg = abi.default_config(max_resources=(R + world - 1) // world, max_batch=max(sub.n, 1), shard_count=world,
                             shard_index=rank)
    o = so.OracleEngine(cfg)
    o.load_flow_rules([r for r in rules if r.resource % world == rank])
    o.submit(sub)
    logs = []
    t_end = int(full.ts_ms[-1])
    for now in (t_end - 2500, t_end + 1500):           # two MetricTimerListener runs (lastFetchTime advances)
        merged = sd.entry_node_allreduce(o.read_entry_node())
        if rank == 0:
            o.set_report_entry_node(merged)
        part = o.metric_log(now, entry_node=(rank == 0))
        parts = [None] * world
        dist.all_gather_object(parts, part)
        logs.append(sd.merge_metric_logs(parts))
    if rank == 0:
        ref = so.OracleEngine(abi.default_config(max_resources=R, max_batch=full.n))
        ref.load_flow_rules(rules)
        ref.submit(full)
        want = [ref.metric_log(now, entry_node=True) for now in (t_end - 2500, t_end + 1500)]
        q.put((logs, want))
    dist.destroy_process_group()


def _sec_groups(log):
    g = {}
    for line in log.split(b"\n"):
        if line:
            g.setdefault(int(line.split(b"|")[0]), []).append(line)
    return g


def test_node_wide_metric_log_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_metric_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    logs, want = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for got, ref in zip(logs, want):
        assert got.count(b"\n") == ref.count(b"\n") > 0
        gg, rr = _sec_groups(got), _sec_groups(ref)
        assert sorted(gg) == sorted(rr)
        for sec in rr:
            # the ENTRY_NODE line (last in its second) is the node-wide one
            assert gg[sec][-1] == rr[sec][-1] and b"__total_inbound_traffic__" in rr[sec][-1]
            assert sorted(gg[sec]) == sorted(rr[sec])


def _degrade_worker(rank, world, port, q):
    """DegradeSlot over resource shards: each rank replays its shard with the
    degrade oracle; rank 0 gathers the verdicts (gloo all_gather of the
    submission positions and statuses) and compares them with one replay of
    the whole batch.  Breaker state is per resource, so the decision path has
    no exchange step."""
    import torch
    import torch.distributed as dist
    from oracle import degrade as od
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R = 400
    rules = trace.degrade_rules(R, seed=41)
    full = trace.degrade_workload(R, 30_000, duration_ms=5000, seed=41, err_p=0.2)
    sel = np.nonzero(full.res_id % world == rank)[0]
    sub = full.shard(world, rank)
    o = od.DegradeOracle()
    o.load_rules([r for r in rules if r["resource"] % world == rank])
    # both replays split at the same event (by submission position), so the
    # same exits cross the batch boundary (entry_ref -1 + create_ts)
    cut = full.n // 2
    half = int(np.searchsorted(sel, cut))
    st = np.concatenate([o.submit(*_cols(sub.subset(0, half)))[0], o.submit(*_cols(sub.subset(half, sub.n)))[0]])
    n_max = torch.tensor([sel.size])
    dist.all_reduce(n_max, op=dist.ReduceOp.MAX)
    pos = torch.full((int(n_max),), -1, dtype=torch.int64)
    pos[:sel.size] = torch.from_numpy(sel)
    val = torch.zeros(int(n_max), dtype=torch.int64)
    val[:sel.size] = torch.from_numpy(st.astype(np.int64))
    all_pos = [torch.empty_like(pos) for _ in range(world)]
    all_val = [torch.empty_like(val) for _ in range(world)]
    dist.all_gather(all_pos, pos)
    dist.all_gather(all_val, val)
    if rank == 0:
        got = np.full(full.n, 255, np.int64)
        for p, v in zip(all_pos, all_val):
            m = p >= 0
            got[p[m].numpy()] = v[m].numpy()
        ref = od.DegradeOracle()
        ref.load_rules(rules)
        want = np.concatenate([ref.submit(*_cols(full.subset(0, cut)))[0],
                               ref.submit(*_cols(full.subset(cut, full.n)))[0]])
        q.put((got, want))
    dist.destroy_process_group()


def _cols(b):
    return b.res_id, b.ts_ms, b.flags, b.entry_ref, b.create_ts


def test_degrade_sharded_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_degrade_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, want = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert np.array_equal(got, want)
    assert (want == 8).sum() > 0


def _token_worker(rank, world, port, q):
    """Cluster token server sharded by flowId: the library's
    sf_token_shard routes every request (a namespace with a
    GlobalRequestLimiter pinned to one shard); each rank decides its requests
    with the token service of its own engine (the oracle here: the CPU
    stand-in of the GPU engine, which the GPU suite pins to it); rank 0 gathers
    the results and compares them with one token server deciding every request."""
    import torch
    import torch.distributed as dist
    from oracle import oracle as so
    from sentinel_amd import engine
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ns, flow, param, items, b = trace.token_workload(20_000, seed=33, max_qps=1500.0, n_flow=60, n_param=20)
    owner = engine.token_shard(flow, param, ns, world, b)
    sel = np.nonzero(owner == rank)[0]
    cfg = abi.default_config(max_resources=4, max_batch=b.n, param_capacity=1 << 16, shard_count=world,
                             shard_index=rank)
    o = so.OracleEngine(cfg)
    o.load_namespaces(ns)
    o.load_cluster_rules(flow, param, items)
    r = o.request_tokens(b.take(sel))
    n_max = torch.tensor([sel.size])
    dist.all_reduce(n_max, op=dist.ReduceOp.MAX)
    pack = torch.full((int(n_max), 3), -99, dtype=torch.int64)
    pos = torch.full((int(n_max),), -1, dtype=torch.int64)
    pos[:sel.size] = torch.from_numpy(sel)
    pack[:sel.size, 0] = torch.from_numpy(r.status.astype(np.int64))
    pack[:sel.size, 1] = torch.from_numpy(r.remaining.astype(np.int64))
    pack[:sel.size, 2] = torch.from_numpy(r.wait_ms.astype(np.int64))
    all_pos = [torch.empty_like(pos) for _ in range(world)]
    all_pack = [torch.empty_like(pack) for _ in range(world)]
    dist.all_gather(all_pos, pos)
    dist.all_gather(all_pack, pack)
    if rank == 0:
        got = np.full((b.n, 3), -99, np.int64)
        for p_, v in zip(all_pos, all_pack):
            m = p_ >= 0
            got[p_[m].numpy()] = v[m].numpy()
        ref = so.OracleEngine(abi.default_config(max_resources=4, max_batch=b.n, param_capacity=1 << 16))
        ref.load_namespaces(ns)
        ref.load_cluster_rules(flow, param, items)
        w = ref.request_tokens(b)
        want = np.stack([w.status.astype(np.int64), w.remaining.astype(np.int64), w.wait_ms.astype(np.int64)], 1)
        q.put((got, want, np.bincount(owner, minlength=world)))
    dist.destroy_process_group()


def test_token_server_sharded_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_token_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, want, per_shard = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert (per_shard > 1000).all(), per_shard
    assert np.array_equal(got, want)
    assert (want[:, 0] == abi.TOKEN_TOO_MANY_REQUEST).sum() > 0        # the pinned namespace limiter fired


def _hostsim_worker(rank, world, port, q):
    """Resource-sharded flow engine: each rank runs the engine's own decision
    code (tests/hostsim: sf_decide.h / sf_heavy.h built for the CPU) with
    shard_count = 2 on its shard of a config-3 batch (two batches, exits
    crossing them); rank 0 gathers the verdicts and compares them with one
    oracle replay of the whole batch."""
    import torch
    import torch.distributed as dist
    from oracle import oracle as so
    from tests.hostsim import hostsim
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R = 3000
    rules = trace.mixed_rules(R, seed=35)
    full = trace.mixed_zipf(R, 120_000, duration_ms=6000, seed=35)
    sel = np.nonzero(full.res_id % world == rank)[0]
    sub = full.shard(world, rank)
    cfg = abi.default_config(max_resources=(R + world - 1) // world, max_batch=max(sub.n, 1), shard_count=world,
                             shard_index=rank, heavy_min_events=64)
    h = hostsim.HostSimEngine(cfg)
    h.load_flow_rules([r for r in rules if r.resource % world == rank])
    cut = full.n // 2
    half = int(np.searchsorted(sel, cut))
    outs = [h.submit(sub.subset(0, half)), h.submit(sub.subset(half, sub.n))]
    st = np.concatenate([o.status for o in outs]).astype(np.int64)
    wt = np.concatenate([o.wait_ms for o in outs]).astype(np.int64)
    n_max = torch.tensor([sel.size])
    dist.all_reduce(n_max, op=dist.ReduceOp.MAX)
    pos = torch.full((int(n_max),), -1, dtype=torch.int64)
    pos[:sel.size] = torch.from_numpy(sel)
    val = torch.zeros((int(n_max), 2), dtype=torch.int64)
    val[:sel.size, 0] = torch.from_numpy(st)
    val[:sel.size, 1] = torch.from_numpy(wt)
    all_pos = [torch.empty_like(pos) for _ in range(world)]
    all_val = [torch.empty_like(val) for _ in range(world)]
    dist.all_gather(all_pos, pos)
    dist.all_gather(all_val, val)
    if rank == 0:
        got = np.full((full.n, 2), -1, np.int64)
        for p_, v in zip(all_pos, all_val):
            m = p_ >= 0
            got[p_[m].numpy()] = v[m].numpy()
        ref = so.OracleEngine(abi.default_config(max_resources=R, max_batch=full.n))
        ref.load_flow_rules(rules)
        ws = [ref.submit(full.subset(0, cut)), ref.submit(full.subset(cut, full.n))]
        want = np.stack([np.concatenate([w.status for w in ws]), np.concatenate([w.wait_ms for w in ws])], 1)
        q.put((got, want.astype(np.int64)))
    dist.destroy_process_group()


def test_flow_engine_hostsim_sharded_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hostsim_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, want = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(got, want)


def _node_trace_worker(rank, world, port, q):
    import torch.distributed as dist
    import bench
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hb, pl = bench.node_trace(5000, 200_000, world, rank, dist)
    assert pl is None
    q.put((rank, hb.res_id, hb.ts_ms, hb.count, hb.flags, hb.entry_ref))
    dist.destroy_process_group()


def test_node_trace_two_ranks():
    """bench.py's node-wide trace for N > 1: rank r holds exactly the events of
    res % N == r of the superposed components (mixed_zipf seeds 3, 4), in
    time order (a millisecond in component order), exits pointing at their
    entries -- the same as building the node's trace on one host."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_node_trace_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((x[0], x[1:]) for x in (q.get(timeout=240), q.get(timeout=240)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    comps = [trace.mixed_zipf(5000, 200_000, duration_ms=4000, seed=3 + c) for c in range(2)]
    for r in range(2):
        res, ts, cnt, fl, er = got[r]
        parts = []
        for c, b in enumerate(comps):
            sel = np.nonzero(b.res_id % 2 == r)[0]
            parts.append((b.ts_ms[sel], np.full(sel.size, c), b.res_id[sel], b.count[sel], b.flags[sel]))
        wts = np.concatenate([p[0] for p in parts])
        wc = np.concatenate([p[1] for p in parts])
        o = np.lexsort((wc, wts))
        assert np.array_equal(ts, wts[o])
        assert np.array_equal(res, np.concatenate([p[2] for p in parts])[o])
        assert np.array_equal(cnt, np.concatenate([p[3] for p in parts])[o])
        assert np.array_equal(fl, np.concatenate([p[4] for p in parts])[o])
        assert np.all(res % 2 == r)
        ex = np.nonzero(fl & abi.EV_EXIT)[0]
        assert ex.size > 0 and np.all(er[ex] >= 0) and np.all(er[ex] < ex)
        assert np.all(res[er[ex]] == res[ex]) and np.all((fl[er[ex]] & abi.EV_EXIT) == 0)
    assert got[0][0].size + got[1][0].size == 400_000


def _placement_worker(rank, world, port, q):
    """bench.py's N > 1 trace with the placement: this rank's shard (engine
    ids) decided by an oracle engine holding its placed resources' rules."""
    import torch.distributed as dist
    import bench
    from oracle import oracle as so
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R = 5000
    hb, pl = bench.node_trace(R, 200_000, world, rank, dist, placement_k=64)
    grade, beh, count = trace.mixed_rule_table(R, seed=3)
    mine = np.nonzero(pl.owner(np.arange(R)) == rank)[0]
    o = so.OracleEngine(abi.default_config(max_resources=pl.local_rows(), max_batch=hb.n, shard_count=world,
                                           shard_index=rank))
    o.load_flow_rules(abi.flow_rules_np(pl.engine_id(mine).astype(np.uint32), grade[mine], count[mine], beh[mine]))
    v = o.submit(hb)
    inv = np.full(pl.R_pad + world * pl.extra, -1, np.int64)
    inv[pl.eid] = np.arange(R)
    q.put((rank, inv[hb.res_id], hb.ts_ms, hb.flags, v.status, v.wait_ms, pl.loads(np.bincount(
        inv[hb.res_id], minlength=R)), int(pl.moved.size)))
    dist.destroy_process_group()


def test_node_trace_placement_two_ranks():
    """The placement of bench.py's N > 1 mode (sentinel_amd/placement.py: the
    top-K resources by the node's counts spread LPT-greedy, renamed to fresh
    engine ids) keeps every verdict: the two ranks' oracle replays of their
    shards equal one replay of the whole node trace (original ids), and the
    ranks' event counts are balanced."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_placement_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((x[0], x[1:]) for x in (q.get(timeout=300), q.get(timeout=300)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle import oracle as so
    R = 5000
    comps = [trace.mixed_zipf(R, 200_000, duration_ms=4000, seed=3 + c) for c in range(2)]
    # the node trace on one host: components merged in time order (a millisecond in component order)
    ts = np.concatenate([b.ts_ms for b in comps])
    cid = np.concatenate([np.full(b.n, c) for c, b in enumerate(comps)])
    o = np.lexsort((cid, ts))
    pos = np.empty(o.size, np.int64)
    pos[o] = np.arange(o.size)
    off = np.array([0, comps[0].n])
    er = np.concatenate([np.where(b.entry_ref >= 0, b.entry_ref + off[c], -1) for c, b in enumerate(comps)])[o]
    er = np.where(er >= 0, pos[np.clip(er, 0, None)], -1)
    node = abi.HostBatch(np.concatenate([b.res_id for b in comps])[o], ts[o],
                         np.concatenate([b.count for b in comps])[o], np.concatenate([b.flags for b in comps])[o],
                         entry_ref=er)
    grade, beh, count = trace.mixed_rule_table(R, seed=3)
    ref = so.OracleEngine(abi.default_config(max_resources=R, max_batch=node.n))
    ref.load_flow_rules(abi.flow_rules_np(np.arange(R, dtype=np.uint32), grade, count, beh))
    want = ref.submit(node)
    for r in range(2):
        res, ts_r, fl_r, st, wt, loads, k = got[r]
        sel = np.nonzero(np.isin(node.res_id, np.unique(res)))[0]
        # this rank's events are exactly the node's events of its resources, in node order
        assert np.array_equal(node.res_id[sel], res) and np.array_equal(node.ts_ms[sel], ts_r)
        assert np.array_equal(st, want.status[sel]) and np.array_equal(wt, want.wait_ms[sel])
        assert k == 64
    sizes = np.array([got[0][0].size, got[1][0].size])
    assert sizes.sum() == node.n and sizes.max() / sizes.mean() < 1.02
