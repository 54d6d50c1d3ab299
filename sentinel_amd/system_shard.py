"""SystemRules on a resource-sharded node.

Two protocols.  ``submit_node`` uses the engine's per-window exchange
(sf_submit_node, sentinel_amd/csrc/sf_sysx.h): the ranks all-gather per-window
aggregates (each rank's ENTRY_NODE contribution and a 128-bin histogram of its
undecided IN entries, 4.2 KB per rank and level) over RCCL or the ``comm``
callback, for SystemRules that read only the inbound-QPS (and CPU) check.
Every other SystemRule (thread, average RT, BBR) and batches with a negative
acquireCount fall back to ``submit_node_gather``, the event all-gather round
protocol below.

The event all-gather round protocol.

SystemRuleManager.checkSystem (SystemRuleManager.java:291-348) reads
Constants.ENTRY_NODE, the one ClusterNode every EntryType.IN event of every
resource updates (StatisticSlot.java:64-123 entry, :139-165 exit).  With
resources sharded over ranks (``res % world == rank``, one engine per GPU) an IN
entry's SystemRule verdict therefore depends on the verdicts of every earlier
IN event of the node, whichever rank decides it.  A single engine resolves
this with its safe-prefix planner (sf_system.h): the SystemRule verdicts of a
prefix [p, q) of the IN stream are fixed by the ENTRY_NODE at p alone.  Here
the same planner runs on every rank over the node's merged IN stream:

1. all-gather the IN events of the batch (global submission sequence numbers
   order them; an exit's entry is found by its sequence number): 24 B per IN
   event, plus the exits' entry references and create times;
2. ``sf_system_plan`` on the merged stream -> q and the forced SystemRule
   verdicts of merged[p, q) -- identical on every rank (same stream, same
   ENTRY_NODE, same rules);
3. each rank decides its own events before merged[q] with ``sf_submit_forced``;
4. all-reduce the verdicts of merged[p, q) (each event has one owner) and
   every rank adds them to its ENTRY_NODE with ``sf_entry_node_add``.

The exchange per round is one all-reduce of the round's verdicts; the event
gather happens once per batch.  The verdicts equal those of one engine over
the whole batch (tests/test_gpu_system_shard.py)."""
from __future__ import annotations

import numpy as np

from . import abi

SYS_NONE = 0xFF
_BLOCKED = (abi.V_BLOCK_FLOW, abi.V_BLOCK_PARAM, abi.V_BLOCK_SYSTEM, abi.V_BLOCK_DEGRADE, abi.V_BLOCK_OTHER)


def _blocked(v: np.ndarray) -> np.ndarray:
    return np.isin(v, _BLOCKED)


class TorchComm:
    """The protocol's two collectives over torch.distributed (gloo on host
    tensors, or nccl = RCCL with ``device`` a GPU)."""

    def __init__(self, group=None, device="cpu"):
        self.group, self.device = group, device

    def allgather_i64(self, x: np.ndarray) -> np.ndarray:
        """Concatenation over ranks (rank order) of a [k, n_r] int64 array."""
        import torch
        import torch.distributed as dist
        world = dist.get_world_size(self.group)
        n = torch.tensor([x.shape[1]], dtype=torch.int64, device=self.device)
        ns = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(ns, n, group=self.group)
        ns = [int(v.item()) for v in ns]
        if max(ns) == 0:                                  # (every rank knows: no second collective)
            return np.zeros((x.shape[0], 0), np.int64)
        pad = np.zeros((x.shape[0], max(ns)), np.int64)
        pad[:, :x.shape[1]] = x
        t = torch.from_numpy(pad).to(self.device)
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t, group=self.group)
        return np.concatenate([p.cpu().numpy()[:, :k] for p, k in zip(parts, ns)], axis=1)

    def allreduce_max_i32(self, x: np.ndarray) -> np.ndarray:
        import torch
        import torch.distributed as dist
        t = torch.from_numpy(np.ascontiguousarray(x, np.int32)).to(self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t.cpu().numpy()

    def allgather_bytes(self, x: np.ndarray):
        """Every rank's equal-sized byte message, rank order (the engine's
        sf_allgather_fn)."""
        import torch
        import torch.distributed as dist
        t = torch.from_numpy(np.ascontiguousarray(x, np.uint8)).to(self.device)
        parts = [torch.empty_like(t) for _ in range(dist.get_world_size(self.group))]
        dist.all_gather(parts, t, group=self.group)
        return [p.cpu().numpy() for p in parts]


class LocalComm:
    """The same collectives between engines of one process, one thread per
    rank (LocalComm.group(world) -> the ranks' comms)."""

    def __init__(self, shared, rank):
        self.s, self.rank = shared, rank

    @staticmethod
    def group(world: int):
        import threading
        shared = {"bar": threading.Barrier(world), "slots": [None] * world}
        return [LocalComm(shared, r) for r in range(world)]

    def _exchange(self, x):
        s = self.s
        s["slots"][self.rank] = x
        s["bar"].wait()
        parts = list(s["slots"])
        s["bar"].wait()                                   # every rank read the slots before reuse
        return parts

    def allgather_i64(self, x: np.ndarray) -> np.ndarray:
        return np.concatenate(self._exchange(np.asarray(x, np.int64)), axis=1)

    def allreduce_max_i32(self, x: np.ndarray) -> np.ndarray:
        return np.maximum.reduce(self._exchange(np.asarray(x, np.int32)))

    def allgather_bytes(self, x: np.ndarray):
        # (x may be a view of the engine's send buffer: the slot holds a copy)
        return self._exchange(np.array(x, np.uint8, copy=True))


def _sub(b: abi.HostBatch, lo: int, hi: int, eref, cts) -> abi.HostBatch:
    """Events [lo, hi) of b with the given entry refs / create timestamps."""
    kw = {}
    if b.arg_tag is not None:
        if b.elem_off is not None:
            raise NotImplementedError("collection arguments under the sharded SystemRule protocol")
        kw = dict(arg_tag=b.arg_tag[:, lo:hi], arg_bits=b.arg_bits[:, lo:hi],
                  n_args=None if b.n_args is None else b.n_args[lo:hi])
    return abi.HostBatch(b.res_id[lo:hi], b.ts_ms[lo:hi], b.count[lo:hi], b.flags[lo:hi],
                         entry_ref=eref, create_ts=cts, **kw)


def submit_node(eng, batch: abi.HostBatch, seq: np.ndarray, comm=None) -> abi.HostVerdicts:
    """This rank's ``batch`` (its shard's events in submission order, ``seq``
    their increasing sequence numbers in the node's stream) with the node-wide
    SystemRule semantics: the engine's per-window exchange when the engine has
    one and its rules allow it, else the event all-gather protocol.  ``comm``
    None: a TorchComm over the default process group."""
    comm = comm or TorchComm()
    if hasattr(eng, "submit_node"):
        from .engine import EngineError
        try:
            return eng.submit_node(batch, seq, comm)
        except EngineError as ex:
            if ex.code != abi.SF_ERR_UNSUPPORTED:
                raise
    return submit_node_gather(eng, batch, seq, comm)


def submit_node_gather(eng, batch: abi.HostBatch, seq: np.ndarray, comm=None) -> abi.HostVerdicts:
    """Decides this rank's ``batch`` (its shard's events, in submission order;
    ``seq`` = their increasing sequence numbers in the node's stream) with the
    node-wide SystemRule semantics.  Every rank of ``comm`` (default: a
    TorchComm over the default process group) calls it with its part of the
    same node batch.  ``entry_ref`` indexes ``batch`` (-1: entry
    passed in an earlier batch, create_ts given; -2: it was blocked)."""
    comm = comm or TorchComm()
    n = batch.n
    seq = np.ascontiguousarray(seq, np.int64)
    assert seq.shape == (n,) and (n < 2 or (np.diff(seq) > 0).all())
    fl = batch.flags
    is_in = (fl & abi.EV_IN) != 0
    li = np.nonzero(is_in)[0]
    # IN events with their entry's sequence number (or the raw -1 / -2 ref)
    eref = batch.entry_ref
    ref_seq = np.full(li.size, -1, np.int64)
    cts = np.zeros(li.size, np.int64) if batch.create_ts is None else batch.create_ts[li].copy()
    if eref is not None:
        r = eref[li]
        ref_seq = np.where(r >= 0, seq[np.clip(r, 0, None)], r)
    # every IN event as 3 words (sequence number, time, acquireCount | flags << 32);
    # the exits' entry sequence numbers and create times in a second gather of
    # the exits alone (24 B per IN entry instead of 48)
    cnt_fl = (batch.count[li].astype(np.int64) & 0xFFFFFFFF) | (fl[li].astype(np.int64) << 32)
    allv = comm.allgather_i64(np.stack([seq[li], batch.ts_ms[li], cnt_fl]))
    xi = np.nonzero(fl[li] & abi.EV_EXIT)[0]
    allx = comm.allgather_i64(np.stack([seq[li][xi], ref_seq[xi], cts[xi]]))
    order = np.argsort(allv[0], kind="stable")
    allv = allv[:, order]
    mseq = allv[0]
    m = mseq.size
    m_cnt = (allv[2] & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
    m_fl = ((allv[2] >> 32) & 0xFF).astype(np.uint8)
    rs = np.full(m, -1, np.int64)
    m_cts = np.zeros(m, np.int64)
    if allx.shape[1]:
        xp = np.searchsorted(mseq, allx[0])
        rs[xp] = allx[1]
        m_cts[xp] = allx[2]
    pos = np.searchsorted(mseq, np.clip(rs, 0, None))
    m_eref = np.where(rs >= 0, pos, rs)
    if m and (rs >= 0).any():
        assert (mseq[pos[rs >= 0]] == rs[rs >= 0]).all(), "exit of an IN entry that no rank holds"
    merged = abi.HostBatch(np.zeros(m, np.uint32), allv[1], m_cnt, m_fl, entry_ref=m_eref, create_ts=m_cts)
    # where this rank's IN events sit in the merged stream
    my_m = np.searchsorted(mseq, seq[li]) if li.size else np.zeros(0, np.int64)
    m_status = np.zeros(m, np.uint8)
    m_mask = np.full(m, SYS_NONE, np.uint8)
    out = abi.HostVerdicts(n)
    lp = 0                                                   # this rank's events before lp are decided

    def decide_local(lq: int, mask: np.ndarray):
        nonlocal lp
        if lq <= lp:
            return
        er = ct = None
        if eref is not None:
            r = eref[lp:lq]
            c0 = np.zeros(lq - lp, np.int64) if batch.create_ts is None else batch.create_ts[lp:lq].copy()
            early = (r >= 0) & (r < lp)
            rr = np.clip(r, 0, None)
            er = np.where(r >= lp, r - lp, r)
            er = np.where(early, np.where(_blocked(out.status[rr]), -2, -1), er).astype(np.int64)
            ct = np.where(early, batch.ts_ms[rr], c0).astype(np.int64)
        v = eng.submit_forced(_sub(batch, lp, lq, er, ct), mask)
        out.status[lp:lq] = v.status
        out.wait_ms[lp:lq] = v.wait_ms
        out.rule_idx[lp:lq] = v.rule_idx
        lp = lq

    p = 0
    while p < m:
        q = eng.system_plan(merged, m_status, p, m_mask)
        # this rank's events before merged[q] (all remaining ones after the last round)
        lq = n if q == m else int(np.searchsorted(seq, mseq[q]))
        mask = np.full(lq - lp, SYS_NONE, np.uint8)
        a, z = np.searchsorted(li, [lp, lq])                # (li and my_m are increasing: ranges, not masks)
        mask[li[a:z] - lp] = m_mask[my_m[a:z]]
        decide_local(lq, mask)
        # verdicts of merged[p, q): owner's value, max over ranks
        vals = np.zeros(q - p, np.int32)
        a, z = np.searchsorted(my_m, [p, q])
        vals[my_m[a:z] - p] = out.status[li[a:z]]
        m_status[p:q] = comm.allreduce_max_i32(vals).astype(np.uint8)
        seg = abi.HostBatch(np.zeros(q - p, np.uint32), merged.ts_ms[p:q], merged.count[p:q], merged.flags[p:q],
                            entry_ref=np.where(m_eref[p:q] >= p, m_eref[p:q] - p,
                                               np.where(m_eref[p:q] >= 0,
                                                        np.where(_blocked(m_status[np.clip(m_eref[p:q], 0, None)]),
                                                                 -2, -1), m_eref[p:q])),
                            create_ts=np.where((m_eref[p:q] >= 0) & (m_eref[p:q] < p),
                                               merged.ts_ms[np.clip(m_eref[p:q], 0, None)], merged.create_ts[p:q]))
        eng.entry_node_add(seg, m_status[p:q])
        p = q
    decide_local(n, np.full(n - lp, SYS_NONE, np.uint8))    # no IN event on the node: nothing to plan
    return out
