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
