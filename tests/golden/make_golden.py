"""Writes the committed golden vectors of tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

The reference is Java and cannot run here (no JDK), so the golden outputs are
produced by the C restatement in oracle/, which is itself pinned by the
reference's own JUnit known-answer assertions (tests/test_oracle_kat.py).
Seeds are fixed; inputs are the shapes of BASELINE.json's configs at test size:

  flowqps_demo   config 1: FlowQpsDemo, one resource, QPS count 20 (10 s)
  mixed_1k       config 3 shape: 1k resources Zipf(1.1), QPS / THREAD / WarmUp /
                 RateLimiter rules, exits, two batches; verdicts + node states
  param_40       config 4 shape: ParamFlow QPS / throttle, Zipf keys
  param_mixed    ParamFlow QPS / throttle / THREAD grade, hot items, null values
  token_5k       config 5 shape: requestToken / requestParamToken, namespace limiter
  degrade_3k     DegradeSlot: RT / exception-ratio / exception-count breakers on
                 3k resources, Zipf entries + exits, two batches (cross-batch
                 exits); verdicts, breaker indices, final breaker states.  Made by
                 oracle/degrade.py, which the reference's circuit-breaker tests
                 pin (tests/test_degrade.py)
"""
import os
import sys

import ctypes as C

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from sentinel_amd import abi, trace  # noqa: E402
from oracle import oracle as so  # noqa: E402
from tests import workloads  # noqa: E402


def batch_arrays(prefix, b):
    d = {f"{prefix}res": b.res_id, f"{prefix}ts": b.ts_ms, f"{prefix}cnt": b.count, f"{prefix}flags": b.flags}
    for k, v in (("eref", b.entry_ref), ("cts", b.create_ts), ("atag", b.arg_tag), ("abits", b.arg_bits),
                 ("nargs", b.n_args)):
        if v is not None:
            d[f"{prefix}{k}"] = v
    return d


def rules_array(rules):
    return np.frombuffer(bytes(abi.rules_array(type(rules[0]), list(rules))), np.uint8) if rules else np.zeros(0, np.uint8)


def node_array(st):
    return np.frombuffer(bytes(st), np.uint8)


def flow_case(name, w):
    cfg = w["cfg"]
    o = so.OracleEngine(cfg)
    if w.get("flow"):
        o.load_flow_rules(w["flow"])
    if w.get("param"):
        o.load_param_rules(w["param"], w.get("items", ()))
    out = {"cfg": np.frombuffer(bytes(cfg), np.uint8), "flow": rules_array(w.get("flow", ())),
           "param": rules_array(w.get("param", ())), "items": rules_array(list(w.get("items", ()))),
           "n_batches": np.array(len(w["batches"])),
           "flow_rec": np.array(C.sizeof(abi.sf_flow_rule))}
    for k, b in enumerate(w["batches"]):
        v = o.submit(b)
        out.update(batch_arrays(f"b{k}_", b))
        out[f"b{k}_status"], out[f"b{k}_wait"], out[f"b{k}_rule"] = v.status, v.wait_ms, v.rule_idx
    nodes = np.array(w["nodes"], np.uint32)
    out["nodes"] = nodes
    out["node_states"] = np.stack([node_array(o.read_node(int(r))) for r in nodes])
    out["entry_node"] = node_array(o.read_entry_node())
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, sum(b.n for b in w["batches"]), "events")


def token_case(name, n):
    ns, flow, param, items, b = trace.token_workload(n, seed=41, max_qps=600.0)
    cfg = abi.default_config(max_resources=4, max_batch=b.n, param_capacity=1 << 14)
    o = so.OracleEngine(cfg)
    o.load_namespaces(ns)
    o.load_cluster_rules(flow, param, items)
    r = o.request_tokens(b)
    now = int(b.ts_ms[-1])
    sums = np.array([[o.cluster_sum(f.flow_id, ev, now) for ev in range(7)] for f in flow], np.int64)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), cfg=np.frombuffer(bytes(cfg), np.uint8),
                        ns=rules_array(ns), cflow=rules_array(flow), cparam=rules_array(param),
                        citems=rules_array(items), flow_id=b.flow_id, count=b.count, flags=b.flags, ts=b.ts_ms,
                        ptag=b.param_tag, pbits=b.param_bits, status=r.status, remaining=r.remaining,
                        wait=r.wait_ms, sums=sums)
    print(name, b.n, "requests")


def degrade_case(name="degrade_3k"):
    from oracle import degrade as od
    R = 3000
    rules = trace.degrade_rules(R, seed=81)
    arr = np.zeros(len(rules), abi.DEGRADE_RULE_DTYPE)
    for i, r in enumerate(rules):
        for k, v in r.items():
            arr[i][k] = v
    full = trace.degrade_workload(R, 40_000, duration_ms=6000, seed=81, err_p=0.2)
    cut = full.n // 2
    o = od.DegradeOracle()
    n = o.load_rules(rules)
    out = {"rules": arr, "R": np.array([R])}
    for k, b in enumerate((full.subset(0, cut), full.subset(cut, full.n))):
        st, ri = o.submit(b.res_id, b.ts_ms, b.flags, b.entry_ref, b.create_ts)
        out.update(batch_arrays(f"b{k}_", b))
        out[f"b{k}_status"], out[f"b{k}_rule"] = st, ri
    states = [o.state(i) for i in range(n)]
    out["breakers"] = np.array([[s["state"], s["next_retry_ms"],
                                 abi.WS_ABSENT if s["window_start"] is None else s["window_start"],
                                 s["hit_count"], s["total_count"]] for s in states], np.int64)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, full.n, "events,", n, "breakers")


if __name__ == "__main__":
    flow_case("flowqps_demo", workloads.config1(duration_ms=10_000))
    flow_case("mixed_1k", workloads.config3(R=1000, n=50_000, seed=77, split=2, duration_ms=5000))
    flow_case("param_40", workloads.config4(R=40, n=30_000, keys=3000, seed=78))
    flow_case("param_mixed", workloads.param_mixed(seed=79, R=10, n=15_000))
    token_case("token_5k", 5000)
    degrade_case()
