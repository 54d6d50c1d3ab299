"""SystemRules on a resource-sharded node: the node-wide round protocol of
sentinel_amd/system_shard.py driven over oracle engines (their
so_system_plan / so_submit_forced / so_entry_node_add restate the engine's
sf_system_plan / sf_submit_forced / sf_entry_node_add one IN event per round).
Two ranks, each holding the resources ``res % 2 == rank``: the merged
verdicts and every rank's ENTRY_NODE must equal one replay of the whole
batch.  In-process ranks (LocalComm, threads) and a gloo world of two
processes (TorchComm, 127.0.0.1).  The GPU engines run the same protocol in
tests/test_gpu_parity.py::test_system_sharded_two_engines."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from sentinel_amd import abi, system_shard
from tests import workloads


def _workload(kind, n_max=6000):
    w = workloads.system(kind)
    full = w["batches"][0]
    n = min(full.n, n_max)
    full = full.subset(0, n)
    # thresholds for the shortened traffic (about 0.6 s of it) so the rule fires
    if kind == "qps":
        w["system"] = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=3000.0, avg_rt=-1,
                                          max_thread=-1)]
    elif kind == "thread":
        w["system"] = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=-1, avg_rt=-1,
                                          max_thread=600)]
    return w, [full.subset(0, n // 2), full.subset(n // 2, n)]


def _load(e, w, world=1, rank=0):
    if w.get("status") is not None:
        e.set_system_status(*w["status"])
    e.load_system_rules(list(w["system"]))
    if w.get("flow"):
        e.load_flow_rules([r for r in w["flow"] if r.resource % world == rank])
    if w.get("param"):
        e.load_param_rules([r for r in w["param"] if r.resource % world == rank], list(w.get("items", ())))


def _rank_run(make, w, batches, world, rank, comm):
    """One rank: its shard of every batch through the protocol; returns
    (batch positions, verdict columns, ENTRY_NODE dict)."""
    R = w["cfg"].max_resources
    cfg = abi.default_config(max_resources=(R + world - 1) // world, max_batch=max(b.n for b in batches),
                             shard_count=world, shard_index=rank, param_capacity=w["cfg"].param_capacity)
    e = make(cfg)
    _load(e, w, world, rank)
    pos, cols, off = [], [], 0
    for b in batches:
        sel = np.nonzero(b.res_id % world == rank)[0]
        v = system_shard.submit_node(e, b.shard(world, rank), sel, comm)
        pos.append(sel + off)
        cols.append(np.stack([v.status, v.wait_ms, v.rule_idx]).astype(np.int64))
        off += b.n
    en = abi.node_state_to_dict(e.read_entry_node(), cfg.sample_count)
    return np.concatenate(pos), np.concatenate(cols, axis=1), en


def _reference(w, batches):
    from oracle import oracle as so
    cfg = abi.default_config(max_resources=w["cfg"].max_resources, max_batch=max(b.n for b in batches),
                             param_capacity=w["cfg"].param_capacity)
    o = so.OracleEngine(cfg)
    _load(o, w)
    vs = [o.submit(b) for b in batches]
    want = np.concatenate([np.stack([v.status, v.wait_ms, v.rule_idx]).astype(np.int64) for v in vs], axis=1)
    return want, abi.node_state_to_dict(o.read_entry_node(), cfg.sample_count)


def _merge(parts, n):
    got = np.full((3, n), -1, np.int64)
    for pos, cols, _ in parts:
        got[:, pos] = cols
    return got


def run_local_ranks(make, w, batches, world=2):
    """Every rank in a thread of this process (LocalComm); returns the merged
    verdict columns and the ranks' ENTRY_NODEs."""
    import threading
    comms = system_shard.LocalComm.group(world)
    parts = [None] * world
    errs = []

    def run(r):
        try:
            parts[r] = _rank_run(make, w, batches, world, r, comms[r])
        except BaseException as ex:          # noqa: BLE001 -- re-raised below
            errs.append(ex)
            comms[r].s["bar"].abort()

    ths = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errs:
        raise errs[0]
    return _merge(parts, sum(b.n for b in batches)), [p[2] for p in parts]


def check_against_reference(w, batches, got, ens):
    want, want_en = _reference(w, batches)
    bad = np.nonzero((got != want).any(axis=0))[0]
    assert bad.size == 0, f"{bad.size} verdicts differ; first {bad[0]}: got {got[:, bad[0]]} want {want[:, bad[0]]}"
    assert (want[0] == abi.V_BLOCK_SYSTEM).sum() > 0, "the SystemRule never fired"
    for en in ens:
        assert en == want_en


@pytest.mark.parametrize("kind", ["qps", "thread", "rt", "load", "cpu"])
def test_system_rounds_local_ranks(kind):
    from oracle import oracle as so
    w, batches = _workload(kind)
    got, ens = run_local_ranks(so.OracleEngine, w, batches)
    check_against_reference(w, batches, got, ens)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, kind, q):
    import torch.distributed as dist
    from oracle import oracle as so
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w, batches = _workload(kind, 3000)
    q.put((rank, _rank_run(so.OracleEngine, w, batches, world, rank, system_shard.TorchComm())))
    dist.destroy_process_group()


def test_system_rounds_gloo_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, "thread", q)) for r in range(2)]
    for p in procs:
        p.start()
    parts = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w, batches = _workload("thread", 3000)
    got = _merge([parts[0], parts[1]], sum(b.n for b in batches))
    check_against_reference(w, batches, got, [parts[0][2], parts[1][2]])

