"""Diagnostics: the THREAD-grade head chain (k_heavy_stream) alone.

One resource with a THREAD rule (count 242, the busiest THREAD resource of
config 3) and C superposed components of its config-3 traffic: per component
E entries per 4 s (acquireCount 1 for 90 %, else 2-5), every entry followed by
its exit after floor(Exp(20 ms)); each millisecond holds component 0's entries
then its exits, then component 1's, ... as bench.py's N-rank node trace merges
them.  C = 1 is the single-GPU head segment (4.87M events), C = 8 what the rank
owning it decides at N = 8.  Prints the segment's device time (heavy profile)
and the decide phase's stream time; --check compares the verdicts with the
oracle on a prefix."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from sentinel_amd import abi, engine, trace  # noqa: E402


def chain_trace(C, entries, count_ms=4000, rt_mean=20.0, seed=11):
    rng = np.random.default_rng(seed)
    ts_l, ex_l, cnt_l, comp_l = [], [], [], []
    for c in range(C):
        ts = np.sort(rng.integers(0, count_ms, size=entries)).astype(np.int64)
        rt = np.floor(rng.exponential(rt_mean, size=entries)).astype(np.int64)
        cnt = np.where(rng.random(entries) < 0.9, 1, rng.integers(2, 6, size=entries)).astype(np.int32)
        ts_l.append(ts); ex_l.append(np.minimum(ts + rt, count_ms - 1)); cnt_l.append(cnt)
        comp_l.append(np.full(entries, c, np.int64))
    ts = np.concatenate(ts_l); ex = np.concatenate(ex_l); cnt = np.concatenate(cnt_l); comp = np.concatenate(comp_l)
    n_e = ts.size
    all_ts = np.concatenate([ts, ex])
    is_exit = np.concatenate([np.zeros(n_e, np.int64), np.ones(n_e, np.int64)])
    comp2 = np.concatenate([comp, comp])
    key = all_ts * (2 * C) + comp2 * 2 + is_exit
    order = np.argsort(key, kind="stable")
    pos = np.empty(2 * n_e, np.int64)
    pos[order] = np.arange(2 * n_e)
    flags = np.full(2 * n_e, abi.EV_IN, np.uint8)
    flags[is_exit[order] == 1] = abi.EV_IN | abi.EV_EXIT
    eref = np.full(2 * n_e, -1, np.int64)
    eref[pos[n_e:]] = pos[:n_e]
    count = np.concatenate([cnt, np.ones(n_e, np.int32)])[order]
    return abi.HostBatch(np.zeros(2 * n_e, np.uint32), trace.T0 + all_ts[order], count, flags, entry_ref=eref)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--comps", default="1,8")
    ap.add_argument("--entries", type=int, default=2_433_762)     # 4.87M events per component
    ap.add_argument("--count", type=float, default=242.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--check", type=int, default=0, help="oracle check on the first N events")
    a = ap.parse_args()
    rules = [abi.sf_flow_rule(resource=0, grade=abi.GRADE_THREAD, count=a.count, control_behavior=0)]
    for C in [int(x) for x in a.comps.split(",")]:
        t = time.time()
        hb = chain_trace(C, a.entries)
        print(f"[chain] C={C}: {hb.n} events built in {time.time() - t:.1f}s", flush=True)
        eng = engine.FlowEngine(abi.default_config(max_resources=64, max_batch=hb.n))
        eng.load_flow_rules(rules)
        span = 4000
        bs = [engine.DeviceBatch(eng, abi.HostBatch(hb.res_id, hb.ts_ms + k * span, hb.count, hb.flags,
                                                    entry_ref=hb.entry_ref)) for k in range(a.reps + 1)]
        out = engine.DeviceVerdicts(eng, hb.n)
        eng.submit_device(bs[0], out)
        eng.sync()
        seg_us, stream_ms, wall = [], [], []
        for r in range(a.reps):
            eng.set_timing(True)
            t = time.perf_counter()
            eng.submit_device(bs[r + 1], out)
            eng.sync()
            wall.append((time.perf_counter() - t) * 1e3)
            st = eng.stats()
            stream_ms.append(st.stream_ms)
            prof = eng.heavy_profile()
            seg_us.append(max((p[3] for p in prof), default=0.0))
            eng.set_timing(False)
        passes = int((out.status.numpy() == abi.V_PASS).sum())
        print(f"[chain] C={C}: segment {np.median(seg_us) / 1e3:.3f} ms, stream {np.median(stream_ms):.3f} ms, "
              f"submit wall {np.median(wall):.2f} ms, passes {passes}", flush=True)
        if a.check:
            from oracle import oracle as so
            n = a.check
            sub = hb.subset(0, n)
            e2 = engine.FlowEngine(abi.default_config(max_resources=64, max_batch=n))
            e2.load_flow_rules(rules)
            o = so.OracleEngine(abi.default_config(max_resources=64, max_batch=n))
            o.load_flow_rules(rules)
            g, w = e2.submit(sub), o.submit(sub)
            bad = int((g.status != w.status).sum())
            print(f"[chain] C={C}: oracle check on {n} events: {bad} mismatches", flush=True)
            e2.close(); o.close()
        for b in bs:
            b.free()
        eng.close()


if __name__ == "__main__":
    main()
