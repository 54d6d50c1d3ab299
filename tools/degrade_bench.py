"""DegradeSlot bench: sf_degrade_submit over an HBM-resident batch.

Workload: R resources, one circuit breaker on half of them (RT / exception
ratio / exception count 1:1:1), entries on a Zipf(s) mix each followed by its
EXIT after an Exp(20 ms) response time, 15% of exits with a business error.
Prints one JSON line: events/s (wall clock around the synchronous submit,
inputs already in HBM) and the CPU oracle (pure Python, one core) on a
bounded sample of the same batch.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from sentinel_amd import abi, engine, trace  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--resources", type=int, default=1_000_000)
    ap.add_argument("--entries", type=int, default=1 << 22)
    ap.add_argument("--zipf", type=float, default=1.1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-sample", type=int, default=200_000)
    ap.add_argument("--check", action="store_true", help="compare every verdict with the oracle (slow)")
    a = ap.parse_args()
    R = a.resources
    rules = trace.degrade_rules_array(R, seed=5)
    b = trace.degrade_workload(R, a.entries, duration_ms=4000, seed=6, s=a.zipf)
    e = engine.FlowEngine(abi.default_config(max_resources=R, max_batch=b.n))
    n_cb = e.load_degrade_rules(rules)
    db = engine.DeviceBatch(e, b)
    dv = engine.DeviceVerdicts(e, b.n, with_wait=False, with_rule=True)
    # every step replays the same trace from fresh breakers (an empty load drops
    # them), shifted by a multiple of every stat interval: the clock moves forward
    span = (int(b.ts_ms[-1] - b.ts_ms[0]) // 60_000 + 2) * 60_000
    shifted = [engine.DeviceBatch.with_ts(e, db, b.ts_ms + k * span) for k in range(1, a.warmup + a.steps + 1)]
    wall = []
    for k, x in enumerate(shifted):
        e.load_degrade_rules([])
        e.load_degrade_rules(rules)
        t = time.perf_counter()
        e.degrade_submit_device(x, dv)
        if k >= a.warmup:
            wall.append(time.perf_counter() - t)
    st = dv.status.numpy() if hasattr(dv, "status") else None
    ms = 1e3 * float(np.median(wall))
    counts = np.bincount(np.asarray(b.res_id, np.int64), minlength=R)
    out = {"metric": "degrade-check events/s", "value": b.n / (ms / 1e3), "unit": "events/s",
           "ms_per_step": round(ms, 3), "steps": a.steps, "events": int(b.n), "resources": R,
           "breakers": int(n_cb), "zipf": a.zipf, "max_events_per_resource": int(counts.max()),
           "alg_bytes_per_event": 24}
    if st is not None:
        out["blocked"] = int((st == abi.V_BLOCK_DEGRADE).sum())
    if a.check:
        from oracle import degrade as od
        o = od.DegradeOracle()
        o.load_rules([{k: (v.item() if hasattr(v, "item") else v) for k, v in zip(rules.dtype.names, r)}
                      for r in rules])
        want, want_rule = o.submit(b.res_id, b.ts_ms, b.flags, b.entry_ref, b.create_ts)
        ri = dv.rule_idx.numpy()
        blk = want == abi.V_BLOCK_DEGRADE
        out["parity"] = {"events": int(b.n), "status_mismatches": int((st != want).sum()),
                         "rule_idx_mismatches": int((ri[blk] != want_rule[blk]).sum())}
    if a.cpu_sample:
        from oracle import degrade as od
        o = od.DegradeOracle()
        o.load_rules([{k: (v.item() if hasattr(v, "item") else v) for k, v in zip(rules.dtype.names, r)}
                      for r in rules[np.isin(rules["resource"], np.unique(b.res_id[:a.cpu_sample]))]])
        sub = b.subset(0, a.cpu_sample)
        t = time.perf_counter()
        o.submit(sub.res_id, sub.ts_ms, sub.flags, sub.entry_ref, sub.create_ts)
        dt = time.perf_counter() - t
        out["cpu_baseline"] = {"value": a.cpu_sample / dt, "unit": "events/s", "cores": 1, "kind": "port",
                               "sample": f"first {a.cpu_sample} events, pure-Python oracle/degrade.py"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
