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
