"""TEST-ONLY restatement of the per-window SystemRule exchange of a sharded
node (sentinel_amd/csrc/sf_sysx.h, sf_engine.cpp ``sf_submit_node``) driven
over oracle engines, so the CPU suite checks the protocol itself -- plan
windows, the binned upper bounds, the level refinement, q -- against one
replay of the whole node batch.

Differences from the product, all outside the plan: every IN entry counts in
u (the product leaves out entries its first ParamFlow rule certainly blocks,
an optimisation that only tightens the bound), and ENTRY_NODE is brought up to
date by all-gathering the decided IN events of the round (the product
all-gathers each rank's 16-word sum of them; the adds of one bucket window
commute, so both give the same node).  ``sx_reduce`` below is the same
function as the product's, line for line; tests/test_system_exchange.py also
checks it against the product's host build (tests/hostsim ``hs_sx_reduce``)."""
from __future__ import annotations

from math import gcd

import numpy as np

from sentinel_amd import abi

SX_B = 128
SX_DELTA = 16
SX_WORDS = SX_DELTA + 4 * SX_B
I64_MAX, I64_MIN = np.iinfo(np.int64).max, np.iinfo(np.int64).min
_BLOCKED = (abi.V_BLOCK_FLOW, abi.V_BLOCK_PARAM, abi.V_BLOCK_SYSTEM, abi.V_BLOCK_DEGRADE, abi.V_BLOCK_OTHER)


def _sat(a, b):
    return I64_MAX if a > I64_MAX - b else a + b


def sx_reduce(msgs: np.ndarray, plan: dict, qps: float, interval_sec: float) -> None:
    """One level over the ranks' messages [N, SX_WORDS] (sf_sysx.h sx_reduce)."""
    if plan["done"]:
        return
    G = plan["ub"]
    base = plan["P"] / interval_sec
    u, n = msgs[:, SX_DELTA:SX_DELTA + SX_B], msgs[:, SX_DELTA + SX_B:SX_DELTA + 2 * SX_B]
    cmin, cmax = msgs[:, SX_DELTA + 2 * SX_B:SX_DELTA + 3 * SX_B], msgs[:, SX_DELTA + 3 * SX_B:]
    for b in range(SX_B):
        lo_b = plan["lo"] + b * plan["w"]
        if lo_b >= plan["hi"]:
            break
        U = 0
        for k in range(msgs.shape[0]):
            U = _sat(U, int(u[k, b]))
        nn = int(n[:, b].sum())
        if nn == 0:
            continue
        cmn, cmx = int(cmin[:, b].min()), int(cmax[:, b].max())
        fire_all = base + float(cmn) > qps
        if not fire_all:
            top = _sat(_sat(max(plan["P"], 0), G), 0 if plan["w"] == 1 else U)
            if (float(top) / interval_sec + float(cmx)) > qps:
                if plan["w"] == 1:
                    plan.update(q=lo_b, done=1)
                    return
                hi = min(lo_b + plan["w"], plan["hi"])
                plan.update(ub=G, lo=lo_b, hi=hi, w=(hi - lo_b + SX_B - 1) // SX_B, level=plan["level"] + 1)
                return
        G = _sat(G, U)
    plan.update(q=plan["hi"], done=1)


def begin(lo, hi):
    return dict(lo=lo, hi=hi, w=(hi - lo + SX_B - 1) // SX_B if hi > lo else 1, ub=0, P=0, q=hi,
                done=1 if hi <= lo else 0, level=0)


def stats(batch: abi.HostBatch, seq: np.ndarray, lp: int, plan: dict) -> np.ndarray:
    """This rank's bins of its undecided IN entries in [lo, hi) (k_sx_stats)."""
    m = np.zeros(SX_WORDS, np.int64)
    m[SX_DELTA + 2 * SX_B:SX_DELTA + 3 * SX_B] = I64_MAX
    m[SX_DELTA + 3 * SX_B:] = I64_MIN
    if plan["done"]:
        return m
    i0 = lp + int(np.searchsorted(seq[lp:], plan["lo"]))
    i1 = lp + int(np.searchsorted(seq[lp:], plan["hi"]))
    fl = batch.flags[i0:i1]
    ok = ((fl & abi.EV_IN) != 0) & ((fl & (abi.EV_EXIT | abi.EV_BLOCKED)) == 0)
    c = batch.count[i0:i1][ok].astype(np.int64)
    k = (seq[i0:i1][ok] - plan["lo"]) // plan["w"]
    m[SX_DELTA:SX_DELTA + SX_B] = np.bincount(k, weights=np.maximum(c, 0), minlength=SX_B)[:SX_B].astype(np.int64)
    m[SX_DELTA + SX_B:SX_DELTA + 2 * SX_B] = np.bincount(k, minlength=SX_B)[:SX_B]
    for b in np.unique(k):
        sel = k == b
        m[SX_DELTA + 2 * SX_B + b] = c[sel].min()
        m[SX_DELTA + 3 * SX_B + b] = c[sel].max()
    return m


def base_P(en: abi.sf_node_state, S: int, wl: int, interval: int, t: int) -> int:
    """ENTRY_NODE's pass sum over the buckets valid at t (sf_system.h sys_base)."""
    W = t - t % wl
    idx = (t // wl) % S
    P = 0
    for i in range(S):
        b = en.second[i]
        if i == idx:
            if b.window_start == W:
                P += b.pass_
            continue
        if b.window_start == abi.SF_WS_ABSENT or t - b.window_start > interval:
            continue
        P += b.pass_
    return P


def _allgather_i64(comm, x) -> np.ndarray:
    x = np.ascontiguousarray(x, np.int64)
    return np.stack([np.asarray(p, np.uint8).view(np.int64) for p in comm.allgather_bytes(x.view(np.uint8))])


def submit_node_windows(o, batch: abi.HostBatch, seq: np.ndarray, comm, *, S: int, interval: int, qps: float,
                        cpu_fires: bool = False, stats_out: dict | None = None) -> abi.HostVerdicts:
    """One rank of the exchange (sf_submit_node) over oracle engine ``o``."""
    n = batch.n
    seq = np.ascontiguousarray(seq, np.int64)
    wl = interval // S
    g = gcd(wl, 1000)
    isec = interval / 1000.0
    fl = batch.flags
    is_ent = ((fl & abi.EV_IN) != 0) & ((fl & (abi.EV_EXIT | abi.EV_BLOCKED)) == 0)
    hdr = np.array([batch.ts_ms[0] // g if n else I64_MAX, batch.ts_ms[-1] // g if n else I64_MIN,
                    seq[-1] + 1 if n else I64_MIN, int((is_ent & (batch.count < 0)).any()), n], np.int64)
    H = _allgather_i64(comm, hdr)
    live = H[:, 4] > 0
    assert not H[:, 3].any(), "negative acquireCount: the gather protocol"
    out = abi.HostVerdicts(n)
    if not live.any():
        return out
    C0, C1, seq_end = int(H[live, 0].min()), int(H[live, 1].max()), int(H[live, 2].max())
    nw = C1 - C0 + 1
    wf = np.full(nw, I64_MAX, np.int64)
    if n:
        cell = batch.ts_ms // g - C0
        first = np.r_[True, cell[1:] != cell[:-1]]
        wf[cell[first]] = seq[first]
    Wf = _allgather_i64(comm, wf).min(axis=0)
    wkey = np.nonzero(Wf != I64_MAX)[0]
    wseq = Wf[wkey]
    lp, sp, j, rounds, levels = 0, int(wseq[0]), 0, 0, 0
    pending = np.zeros((5, 0), np.int64)          # decided IN events of the last sub-batch: ts, c, flags, status, cts
    while True:
        fin = sp >= seq_end
        while not fin and j + 1 < wseq.size and wseq[j + 1] <= sp:
            j += 1
        # ENTRY_NODE += the node's IN events of the last sub-batch
        cnt = _allgather_i64(comm, np.array([pending.shape[1]], np.int64))[:, 0]
        pad = np.zeros((5, int(cnt.max())), np.int64)
        pad[:, :pending.shape[1]] = pending
        allp = _allgather_i64(comm, pad.reshape(-1)).reshape(len(cnt), 5, -1)
        ev = np.concatenate([allp[k][:, :cnt[k]] for k in range(len(cnt))], axis=1)
        if ev.shape[1]:
            m = ev.shape[1]
            o.entry_node_add(abi.HostBatch(np.zeros(m, np.uint32), ev[0], ev[1].astype(np.int32),
                                           ev[2].astype(np.uint8), entry_ref=np.full(m, -1, np.int64),
                                           create_ts=ev[4]), ev[3].astype(np.uint8))
        if fin:
            break
        lo, hi = sp, int(wseq[j + 1]) if j + 1 < wseq.size else seq_end
        wstart = (C0 + int(wkey[j])) * g
        plan = begin(lo, hi)
        plan["P"] = base_P(o.read_entry_node(), S, wl, interval, wstart)
        while not plan["done"]:
            sx_reduce(_allgather_i64(comm, stats(batch, seq, lp, plan)), plan, qps, isec)
            levels += 1
        q = plan["q"]
        assert sp < q <= hi
        lq = lp + int(np.searchsorted(seq[lp:], q))
        if lq > lp:
            c = batch.count[lp:lq].astype(np.float64)
            fire = plan["P"] / isec + c > qps
            mask = np.where(fire, 0, 4 if cpu_fires else 0xFF).astype(np.uint8)
            mask[~is_ent[lp:lq]] = 0xFF
            er = ct = None
            if batch.entry_ref is not None:
                r = batch.entry_ref[lp:lq]
                c0 = np.zeros(lq - lp, np.int64) if batch.create_ts is None else batch.create_ts[lp:lq].copy()
                early = (r >= 0) & (r < lp)
                rr = np.clip(r, 0, None)
                er = np.where(r >= lp, r - lp, r)
                er = np.where(early, np.where(np.isin(out.status[rr], _BLOCKED), -2, -1), er).astype(np.int64)
                ct = np.where(early, batch.ts_ms[rr], c0).astype(np.int64)
            kw = {}
            if batch.arg_tag is not None:
                kw = dict(arg_tag=batch.arg_tag[:, lp:lq], arg_bits=batch.arg_bits[:, lp:lq],
                          n_args=None if batch.n_args is None else batch.n_args[lp:lq])
            sub = abi.HostBatch(batch.res_id[lp:lq], batch.ts_ms[lp:lq], batch.count[lp:lq], batch.flags[lp:lq],
                                entry_ref=er, create_ts=ct, **kw)
            v = o.submit_forced(sub, mask)
            out.status[lp:lq], out.wait_ms[lp:lq], out.rule_idx[lp:lq] = v.status, v.wait_ms, v.rule_idx
            # the round's IN events for ENTRY_NODE (exits: their entry's create time)
            idx = np.nonzero((fl[lp:lq] & abi.EV_IN) != 0)[0] + lp
            cts = np.zeros(idx.size, np.int64)
            if batch.entry_ref is not None:
                r = batch.entry_ref[idx]
                cts = np.where(r >= 0, batch.ts_ms[np.clip(r, 0, None)],
                               batch.create_ts[idx] if batch.create_ts is not None else batch.ts_ms[idx])
            pending = np.stack([batch.ts_ms[idx], batch.count[idx].astype(np.int64), fl[idx].astype(np.int64),
                                out.status[idx].astype(np.int64), cts])
        else:
            pending = np.zeros((5, 0), np.int64)
        lp, sp = lq, q
        rounds += 1
    assert lp == n
    if stats_out is not None:
        stats_out.update(rounds=rounds, levels=levels)
    return out
