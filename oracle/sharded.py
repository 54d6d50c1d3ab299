"""TEST INFRASTRUCTURE / CPU BASELINE ONLY -- the C oracle replayed on several
host cores: the batch is split by resource (res % T, local id res // T, the
engine's own shard map), each shard replays on its own OracleEngine in its own
thread (the ctypes call releases the GIL), and the verdicts are merged back
into batch order.  Without SystemRules (node-wide ENTRY_NODE) the shards are
independent, so the merged verdicts equal one replay of the whole batch
(SURVEY.md §6 / BASELINE.md: the multi-core CPU baseline, resource-sharded).
Used by bench.py's cpu_baseline leg and tests/test_oracle_sharded.py."""
import threading

import numpy as np

from sentinel_amd import abi


def split(hb: abi.HostBatch, T: int):
    """Per-shard HostBatch (local resource ids, entry refs remapped) and the
    batch positions of each shard's events."""
    res = hb.res_id.astype(np.int64)
    shard = (res % T).astype(np.uint8 if T <= 255 else np.int32)   # uint8: numpy sorts it by radix
    order = np.argsort(shard, kind="stable")
    counts = np.bincount(shard, minlength=T)
    starts = np.concatenate([[0], np.cumsum(counts)])
    pos = np.empty(hb.n, np.int64)                          # batch index -> index inside its shard
    for k in range(T):
        idx = order[starts[k]:starts[k + 1]]
        pos[idx] = np.arange(idx.size)
    out = []
    for k in range(T):
        idx = order[starts[k]:starts[k + 1]]
        eref = None
        if hb.entry_ref is not None:
            r = hb.entry_ref[idx]
            eref = np.where(r >= 0, pos[np.clip(r, 0, None)], r).astype(np.int64)
        b = abi.HostBatch((res[idx] // T).astype(np.uint32), hb.ts_ms[idx], hb.count[idx], hb.flags[idx],
                          entry_ref=eref, create_ts=None if hb.create_ts is None else hb.create_ts[idx],
                          origin=None if hb.origin is None else hb.origin[idx],
                          context=None if hb.context is None else hb.context[idx])
        out.append((idx, b))
    return out


def shard_rules(rules, T: int, k: int):
    """Flow rules of shard k with local resource ids (list order kept); rules is
    a list of abi.sf_flow_rule or an abi.FLOW_RULE_DTYPE array.  A RELATE
    reference (same shard by construction) gets its local id too."""
    if isinstance(rules, np.ndarray):
        out = rules[rules["resource"] % T == k].copy()
        out["resource"] //= T
        rel = (out["strategy"] == abi.STRATEGY_RELATE) & (out["ref_resource"] != abi.REF_NONE)
        out["ref_resource"][rel] //= T
        return out
    out = []
    for r in rules:
        if r.resource % T == k:
            c = abi.sf_flow_rule.from_buffer_copy(r)
            c.resource = r.resource // T
            if c.strategy == abi.STRATEGY_RELATE and c.ref_resource != abi.REF_NONE:
                c.ref_resource //= T
            out.append(c)
    return out


def replay(rules, hb: abi.HostBatch, R: int, T: int):
    """Replays hb on T threads; returns (verdicts in batch order, seconds of
    the parallel replay, excluding the split and the rule loads)."""
    from oracle import oracle as so
    parts = split(hb, T)
    engines = []
    for k in range(T):
        e = so.OracleEngine(abi.default_config(max_resources=R // T + 1, max_batch=max(1, parts[k][1].n)))
        e.load_flow_rules(shard_rules(rules, T, k))
        engines.append(e)
    outs = [None] * T

    def run(k):
        outs[k] = engines[k].submit(parts[k][1])

    import time
    ths = [threading.Thread(target=run, args=(k,)) for k in range(T)]
    t = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t
    for e in engines:
        e.close()
    v = abi.HostVerdicts(hb.n)
    for k in range(T):
        idx = parts[k][0]
        v.status[idx] = outs[k].status
        v.wait_ms[idx] = outs[k].wait_ms
        v.rule_idx[idx] = outs[k].rule_idx
    return v, dt


class ShardedOracle:
    """The C oracle over T host threads for a sequence of batches of the same
    resource set: one OracleEngine per resource shard (res % T) keeps its
    state across batches.  ``split_like`` reuses one batch's partition for
    batches that differ only in their timestamps (bench.py's time-shifted
    steps)."""

    def __init__(self, rules, R: int, T: int, max_batch: int):
        from oracle import oracle as so
        self.T = T
        self.engines = []
        for k in range(T):
            e = so.OracleEngine(abi.default_config(max_resources=R // T + 1, max_batch=max(1, max_batch // T * 2 + 64)))
            e.load_flow_rules(shard_rules(rules, T, k))
            self.engines.append(e)
        self.parts = None

    def split_like(self, hb: abi.HostBatch):
        self.parts = split(hb, self.T)

    def submit(self, hb: abi.HostBatch, ts_shift: int = 0):
        """Replays hb (partitioned like the split_like batch, timestamps +
        ts_shift); returns (verdicts in batch order, seconds)."""
        import time
        if self.parts is None:
            self.split_like(hb)
        outs = [None] * self.T

        def run(k):
            idx, b = self.parts[k]
            if ts_shift:
                b = abi.HostBatch(b.res_id, b.ts_ms + ts_shift, b.count, b.flags, entry_ref=b.entry_ref,
                                  create_ts=None if b.create_ts is None else b.create_ts + ts_shift,
                                  origin=b.origin, context=b.context)
            outs[k] = self.engines[k].submit(b)

        ths = [threading.Thread(target=run, args=(k,)) for k in range(self.T)]
        t = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t
        v = abi.HostVerdicts(hb.n)
        for k in range(self.T):
            idx = self.parts[k][0]
            v.status[idx] = outs[k].status
            v.wait_ms[idx] = outs[k].wait_ms
            v.rule_idx[idx] = outs[k].rule_idx
        return v, dt

    def read_node(self, res: int):
        return self.engines[res % self.T].read_node(res // self.T)

    def read_origin_node(self, res: int, origin: int):
        return self.engines[res % self.T].read_origin_node(res // self.T, origin)

    def read_rule_state(self, res_rule: int):
        """Rule state of the resource's single rule (one rule per resource)."""
        return self.engines[res_rule % self.T].read_rule_state(res_rule // self.T)

    def node_digests(self, R: int):
        """so_node_digests of every resource 0..R-1 (shard res % T, row res // T)."""
        parts = [None] * self.T

        def run(k):
            n = (R - k + self.T - 1) // self.T
            parts[k] = self.engines[k].node_digests(n) if n > 0 else None

        ths = [threading.Thread(target=run, args=(k,)) for k in range(self.T)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        out = np.empty(R, np.uint64)
        for k in range(self.T):
            if parts[k] is not None:
                out[k::self.T] = parts[k]
        return out

    def rule_states(self, R: int):
        """(R, 3) controller states of rules 0..R-1, rule r being resource r's single rule."""
        out = np.empty((R, 3), np.int64)
        for k, e in enumerate(self.engines):
            n = (R - k + self.T - 1) // self.T
            if n > 0:
                out[k::self.T] = e.rule_states(0, n)
        return out

    def entry_nodes(self):
        return [e.read_entry_node() for e in self.engines]

    def close(self):
        for e in self.engines:
            e.close()
