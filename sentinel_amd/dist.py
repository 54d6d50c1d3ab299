"""Node-wide aggregates over resource shards (one process per GPU).

Resources are hash-sharded over the GPUs of a node (``res % N == rank``) and
the decision path exchanges nothing.  The one exchange step is the node-wide
``Constants.ENTRY_NODE`` (Constants.java:66): every rank's engine keeps the
ENTRY_NODE windows of its own shard's inbound traffic, and the node-wide node
is their merge.  Java's LeapArray keeps, per bucket slot, the latest window
that saw traffic (LeapArray.currentWindow, LeapArray.java:128-225), so the
merge is:

1. all-reduce MAX of each slot's window start;
2. every rank drops its slots that hold an older window;
3. all-reduce SUM of the counters, MIN of minRt, SUM of curThreadNum.

With ``torch.distributed`` on the ``nccl`` backend (RCCL on ROCm) these are
three small all-reduces over xGMI (< 8 KB); with ``gloo`` they run on the CPU
(tests).  The metric snapshot rows (MetricTimerListener) are gathered to
rank 0 off the decision path.
"""
from __future__ import annotations

import numpy as np

from . import abi

FIELDS = ("pass_", "block", "exception", "success", "rt", "occupied_pass")
I64_MIN = np.iinfo(np.int64).min


def _state_arrays(st: abi.sf_node_state, sample_count: int):
    buckets = [st.second[i] for i in range(sample_count)] + [st.minute[i] for i in range(abi.SF_MINUTE_BUCKETS)]
    ws = np.array([b.window_start for b in buckets], np.int64)
    cnt = np.array([[getattr(b, f) for f in FIELDS] for b in buckets], np.int64)
    minrt = np.array([b.min_rt for b in buckets], np.int64)
    return ws, cnt, minrt


def entry_node_allreduce(state: abi.sf_node_state, sample_count: int = 2, device=None, group=None,
                         statistic_max_rt: int = 5000) -> abi.sf_node_state:
    """Merge this rank's ENTRY_NODE with every other rank's; returns the
    node-wide ENTRY_NODE (same layout as ``sf_read_entry_node``)."""
    import torch
    import torch.distributed as dist

    ws, cnt, minrt = _state_arrays(state, sample_count)
    absent = ws == abi.SF_WS_ABSENT
    t_ws = torch.tensor(np.where(absent, I64_MIN, ws), dtype=torch.int64, device=device)
    dist.all_reduce(t_ws, op=dist.ReduceOp.MAX, group=group)
    gws = t_ws.cpu().numpy()
    keep = (~absent) & (ws == gws)
    t_cnt = torch.tensor(np.where(keep[:, None], cnt, 0), dtype=torch.int64, device=device)
    t_min = torch.tensor(np.where(keep, minrt, np.iinfo(np.int64).max), dtype=torch.int64, device=device)
    t_thr = torch.tensor([state.cur_thread_num], dtype=torch.int64, device=device)
    dist.all_reduce(t_cnt, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(t_min, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(t_thr, op=dist.ReduceOp.SUM, group=group)
    gcnt, gmin = t_cnt.cpu().numpy(), t_min.cpu().numpy()
    out = abi.sf_node_state()
    for i in range(abi.SF_MAX_SAMPLE_COUNT):
        out.second[i].window_start = abi.SF_WS_ABSENT
        out.borrow_ws[i] = abi.SF_WS_ABSENT
    buckets = [out.second[i] for i in range(sample_count)] + [out.minute[i] for i in range(abi.SF_MINUTE_BUCKETS)]
    for k, b in enumerate(buckets):
        if gws[k] == I64_MIN:
            b.window_start = abi.SF_WS_ABSENT
            continue
        b.window_start = int(gws[k])
        for j, f in enumerate(FIELDS):
            setattr(b, f, int(gcnt[k, j]))
        b.min_rt = int(gmin[k]) if gmin[k] != np.iinfo(np.int64).max else statistic_max_rt
    out.cur_thread_num = int(t_thr.item())
    return out


def merge_entry_nodes(states, sample_count: int = 2, statistic_max_rt: int = 5000) -> abi.sf_node_state:
    """The same merge over host copies of every shard's ENTRY_NODE (no
    process group): per slot the latest window, SUM of its counters, MIN of
    minRt, SUM of curThreadNum."""
    arrs = [_state_arrays(st, sample_count) for st in states]
    ws = np.stack([np.where(a[0] == abi.SF_WS_ABSENT, I64_MIN, a[0]) for a in arrs])
    gws = ws.max(axis=0)
    keep = (ws == gws[None, :]) & (ws != I64_MIN)
    gcnt = sum(np.where(keep[k][:, None], arrs[k][1], 0) for k in range(len(arrs)))
    gmin = np.min(np.stack([np.where(keep[k], arrs[k][2], np.iinfo(np.int64).max) for k in range(len(arrs))]), axis=0)
    out = abi.sf_node_state()
    for i in range(abi.SF_MAX_SAMPLE_COUNT):
        out.second[i].window_start = abi.SF_WS_ABSENT
        out.borrow_ws[i] = abi.SF_WS_ABSENT
    buckets = [out.second[i] for i in range(sample_count)] + [out.minute[i] for i in range(abi.SF_MINUTE_BUCKETS)]
    for k, b in enumerate(buckets):
        if gws[k] == I64_MIN:
            b.window_start = abi.SF_WS_ABSENT
            continue
        b.window_start = int(gws[k])
        for j, f in enumerate(FIELDS):
            setattr(b, f, int(gcnt[k, j]))
        b.min_rt = int(gmin[k]) if gmin[k] != np.iinfo(np.int64).max else statistic_max_rt
    out.cur_thread_num = int(sum(st.cur_thread_num for st in states))
    return out


def gather_snapshot(rows, group=None):
    """Gather every rank's MetricNode rows to rank 0 (object gather, off the decision path)."""
    import torch.distributed as dist
    packed = [(r.resource, r.timestamp, r.pass_qps, r.block_qps, r.success_qps, r.exception_qps, r.rt,
               r.occupied_pass_qps) for r in rows]
    world = dist.get_world_size(group)
    out = [None] * world if dist.get_rank(group) == 0 else None
    dist.gather_object(packed, out, dst=0, group=group)
    if out is None:
        return None
    return sorted(x for part in out for x in part)


def rccl_join(eng, group=None):
    """Join ``eng`` to an RCCL communicator of all ranks of ``group`` (the
    unique id travels over the host process group, e.g. gloo)."""
    import torch.distributed as dist
    from . import engine as _engine
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    box = [_engine.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0, group=group)
    eng.comm_init(world, rank, box[0])


ENTRY_NODE_NAME = b"__total_inbound_traffic__"


def merge_metric_logs(parts):
    """metrics.log of a resource-sharded node from every rank's sf_metric_log
    bytes (rank 0's carries the node-wide ENTRY_NODE line, set with
    sf_set_report_entry_node): lines grouped by second ascending as
    MetricTimerListener's TreeMap does (MetricTimerListener.java:40-69), each
    second's resource lines in rank order and the ENTRY_NODE line last."""
    by_sec = {}
    for part in parts:
        for line in part.split(b"\n"):
            if not line:
                continue
            f = line.split(b"|")
            sec = int(f[0])
            ent = by_sec.setdefault(sec, ([], []))
            (ent[1] if f[2] == ENTRY_NODE_NAME else ent[0]).append(line)
    out = []
    for sec in sorted(by_sec):
        res, en = by_sec[sec]
        out += res + en
    return b"".join(x + b"\n" for x in out)
