"""Config 4 with its SystemRule (BASELINE.json configs[3]): hot-parameter
limiting over 1k resources (one QPS ParamFlowRule each, +10 % with a throttle
rule), keys Zipf(1.1) over 100M distinct values, every event EntryType.IN, and
the inbound-QPS SystemRule at 0.8x the offered rate.

One sf_submit of an HBM-resident batch from a fresh engine is timed (the
planner cuts it into safe sub-batches, sf_system.h); the oracle replays the
same batch from fresh state (verdict parity + the CPU baseline).  Prints one
JSON line with the exact table's load factor and longest probe.

    python tools/system_bench.py [--events 16777216] [--keys 100000000] [--no-check]
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


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--resources", type=int, default=1000)
    ap.add_argument("--events", type=int, default=1 << 24)
    ap.add_argument("--keys", type=int, default=100_000_000)
    ap.add_argument("--duration-ms", type=int, default=4000)
    ap.add_argument("--qps-frac", type=float, default=0.8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    engine.lib()
    t0 = time.time()
    rules, b = trace.param_zipf(a.resources, a.events, a.keys, duration_ms=a.duration_ms, seed=4)
    offered = b.n / (a.duration_ms / 1000.0)
    sysr = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=a.qps_frac * offered,
                               avg_rt=-1, max_thread=-1)]
    pairs = np.unique(b.res_id.astype(np.uint64) << np.uint64(40) ^ (b.arg_bits[0] & np.uint64((1 << 40) - 1))).size
    cap = 1 << int(np.ceil(np.log2(max(2.5 * pairs * 1.1, 1 << 16))))
    cfg = abi.default_config(max_resources=a.resources, max_batch=b.n, param_capacity=cap)
    log(f"trace {b.n} events, ~{pairs} (resource, key) pairs, table {cap} slots, {time.time() - t0:.1f}s")

    walls, st = [], None
    for rep in range(a.reps):
        e = engine.FlowEngine(cfg)
        e.load_system_rules(sysr)
        e.load_param_rules(rules)
        db = engine.DeviceBatch(e, b)
        dv = engine.DeviceVerdicts(e, b.n, with_wait=True, with_rule=True)
        e.sync()
        t = time.perf_counter()
        e.submit_device(db, dv)
        walls.append(time.perf_counter() - t)
        if rep == a.reps - 1:
            st = (dv.status.numpy(), dv.wait_ms.numpy(), dv.rule_idx.numpy())
            tab = e.param_table_stats()
            rounds = e.stats().sys_rounds
        db.free()
        dv.free()
        e.close()
    ms = 1e3 * float(np.median(walls))
    ent = int(((b.flags & abi.EV_EXIT) == 0).sum())
    out = {"metric": "config4 flow-check decisions/s (ParamFlow 100M-key Zipf + SystemRule qps 0.8x offered)",
           "value": round(ent / (ms / 1e3), 1), "unit": "decisions/s", "ms_per_batch": round(ms, 3),
           "events": int(b.n), "resources": a.resources, "key_space": a.keys, "distinct_pairs": int(pairs),
           "planner_rounds": int(rounds), "param_table": tab,
           "system_blocks": int((st[0] == abi.V_BLOCK_SYSTEM).sum()),
           "param_blocks": int((st[0] == abi.V_BLOCK_PARAM).sum()),
           "passed": int(np.isin(st[0], abi.PASSED).sum()), "reps_ms": [round(1e3 * w, 3) for w in walls]}
    if not a.no_check:
        from oracle import oracle as so
        o = so.OracleEngine(cfg)
        o.load_system_rules(sysr)
        o.load_param_rules(rules)
        t = time.perf_counter()
        want = o.submit(b)
        dt = time.perf_counter() - t
        o.close()
        mism = {"status": int((st[0] != want.status).sum()), "wait_ms": int((st[1] != want.wait_ms).sum()),
                "rule_idx": int((st[2] != want.rule_idx).sum())}
        out["parity"] = {"events": int(b.n), "mismatches": mism, "exact": not any(mism.values())}
        out["cpu_baseline"] = {"value": round(ent / dt, 1), "unit": "decisions/s", "cores": 1, "kind": "port",
                               "sample": "the same batch from fresh state, single-threaded C oracle",
                               "seconds": round(dt, 2)}
        out["speedup_vs_oracle"] = round(dt / (ms / 1e3), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
