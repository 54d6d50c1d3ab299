"""The sharded SystemRule protocols (sentinel_amd/system_shard.py) timed
with two ranks on one GPU: the per-window exchange (sf_submit_node, the
default) or, with --gather, the event all-gather round protocol: two processes (gloo on 127.0.0.1), each an engine
on cuda:0 holding the resources ``res % 2 == rank`` of a config-4-shaped batch
(ParamFlow rules, Zipf keys, inbound-QPS SystemRule at 0.6x the offered
rate).  Rank 0 prints one JSON line: wall time, planner rounds, bytes and
milliseconds of each collective per round, and the verdicts against one
engine deciding the whole batch (the same GPU, after the two ranks finish).

    python tools/system_two_ranks.py [--events 2097152] [--resources 1000] [--out profiles/r05_system_two_ranks.json]
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def workload(R, n, frac):
    from sentinel_amd import abi, trace
    rules, b = trace.param_zipf(R, n, 1_000_000, duration_ms=4000, seed=4)
    sysr = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=frac * n / 4.0, avg_rt=-1,
                               max_thread=-1)]
    return rules, b, sysr


class CountingComm:
    """TorchComm with the bytes and time of every collective recorded."""

    def __init__(self, inner):
        self.inner, self.log = inner, []

    def allgather_i64(self, x):
        t = time.perf_counter()
        r = self.inner.allgather_i64(x)
        self.log.append(("allgather_i64", int(r.nbytes), time.perf_counter() - t))
        return r

    def allreduce_max_i32(self, x):
        t = time.perf_counter()
        r = self.inner.allreduce_max_i32(x)
        self.log.append(("allreduce_max_i32", int(r.nbytes), time.perf_counter() - t))
        return r

    def allgather_bytes(self, x):
        t = time.perf_counter()
        r = self.inner.allgather_bytes(x)
        self.log.append(("allgather_bytes", int(x.nbytes), time.perf_counter() - t))
        return r


def worker(rank, world, port, a, q):
    import numpy as np
    import torch.distributed as dist
    from sentinel_amd import abi, engine, system_shard
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rules, b, sysr = workload(a.resources, a.events, a.frac)
    cfg = abi.default_config(max_resources=(a.resources + world - 1) // world, max_batch=b.n, shard_count=world,
                             shard_index=rank, param_capacity=1 << 24)
    e = engine.FlowEngine(cfg)
    e.load_system_rules(sysr)
    e.load_param_rules([r for r in rules if r.resource % world == rank])
    sel = np.nonzero(b.res_id % world == rank)[0]
    part = b.shard(world, rank)
    comm = CountingComm(system_shard.TorchComm())
    dist.barrier()
    t = time.perf_counter()
    if a.gather:
        v = system_shard.submit_node_gather(e, part, sel, comm)
    else:
        v = system_shard.submit_node(e, part, sel, comm)
    dist.barrier()
    wall = time.perf_counter() - t
    rounds = int(e.stats().sys_rounds)
    e.close()
    q.put((rank, sel, v.status, v.wait_ms, v.rule_idx, wall, comm.log, rounds))
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1 << 21)
    ap.add_argument("--resources", type=int, default=1000)
    ap.add_argument("--frac", type=float, default=0.6)
    ap.add_argument("--gather", action="store_true", help="the event all-gather protocol instead of the exchange")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import numpy as np
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, 2, port, a, q)) for r in range(2)]
    for p in procs:
        p.start()
    parts = dict((x[0], x[1:]) for x in (q.get(timeout=900) for _ in range(2)))
    # (parts[r]: sel, status, wait, rule, wall, log, rounds)
    for p in procs:
        p.join(timeout=120)
    from sentinel_amd import abi, engine
    rules, b, sysr = workload(a.resources, a.events, a.frac)
    got = np.full((3, b.n), -1, np.int64)
    for r in range(2):
        sel, st, wt, ri = parts[r][:4]
        got[:, sel] = np.stack([st, wt, ri])
    cfg = abi.default_config(max_resources=a.resources, max_batch=b.n, param_capacity=1 << 24)
    e = engine.FlowEngine(cfg)
    e.load_system_rules(sysr)
    e.load_param_rules(rules)
    t = time.perf_counter()
    v = e.submit(b)
    one_ms = 1e3 * (time.perf_counter() - t)
    e.close()
    want = np.stack([v.status, v.wait_ms, v.rule_idx]).astype(np.int64)
    log = parts[0][5]
    ag = [x for x in log if x[0] == "allgather_i64"]
    ar = [x for x in log if x[0] == "allreduce_max_i32"]
    xb = [x for x in log if x[0] == "allgather_bytes"]
    proto = ("event all-gather round protocol (system_shard.submit_node_gather)" if a.gather else
             "per-window exchange (sf_submit_node via system_shard.submit_node)")
    res = {"what": f"sharded SystemRule, {proto}, 2 ranks (gloo) on one GPU, "
                   f"config-4 shape: {a.resources} resources with ParamFlow rules, Zipf keys, "
                   f"inbound QPS at {a.frac}x offered", "events": int(b.n),
           "wall_ms_max_over_ranks": round(1e3 * max(parts[r][4] for r in range(2)), 3),
           "planner_rounds": parts[0][6] if not a.gather else len(ar),
           "exchange": {"calls": len(xb), "bytes_sent_per_rank": int(sum(x[1] for x in xb)),
                        "bytes_per_call_max": int(max((x[1] for x in xb), default=0)),
                        "ms": round(1e3 * sum(x[2] for x in xb), 3)},
           "allgather": {"calls": len(ag), "bytes": int(sum(x[1] for x in ag)),
                         "ms": round(1e3 * sum(x[2] for x in ag), 3)},
           "allreduce_per_round": {"calls": len(ar), "bytes_mean": round(float(np.mean([x[1] for x in ar])), 1)
                                   if ar else 0, "ms_mean": round(1e3 * float(np.mean([x[2] for x in ar])), 3)
                                   if ar else 0},
           "one_engine_whole_batch_ms": round(one_ms, 3),
           "system_blocks": int((want[0] == abi.V_BLOCK_SYSTEM).sum()),
           "parity": {"what": "merged verdicts of the two ranks vs one engine deciding the whole batch",
                      "mismatches": int((got != want).any(axis=0).sum()),
                      "exact": bool((got == want).all())}}
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
