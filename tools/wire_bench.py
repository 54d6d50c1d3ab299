"""Throughput of the token-server wire path (sf_serve_frames), config 5 shape:
500 client connections of namespace 1, 10k flowIds + 1k param flowIds (Zipf
values over 1M), 10 % prioritized, maxAllowedQps 1e12 (limiter open).  The
request frames are written by the reference client layout (sentinel_amd.wire)
with numpy, one call = one batch of all connections' inbound bytes.

Prints one JSON line: requests/s from the engine's device clock (framing to
encoded responses, inputs already in HBM), the bytes read and written, and the
CPU oracle on a bounded sample.  TEST/MEASUREMENT TOOL: the oracle leg only."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sentinel_amd import abi, trace  # noqa: E402


def frames(n_req, n_streams, seed):
    rng = np.random.default_rng(seed)
    n_flow, n_param, n_values = 10000, 1000, 1 << 20
    ns = [abi.sf_namespace(namespace_id=1, connected_count=n_streams, max_allowed_qps=1e12)]
    flow = [abi.sf_cluster_flow_rule(flow_id=k + 1, count=float(rng.integers(1, 21)),
                                     threshold_type=abi.THRESHOLD_AVG_LOCAL, namespace_id=1, sample_count=10,
                                     window_interval_ms=1000) for k in range(n_flow)]
    param = [abi.sf_cluster_param_rule(flow_id=n_flow + k + 1, count=float(rng.integers(1, 30)),
                                       threshold_type=abi.THRESHOLD_AVG_LOCAL, namespace_id=1, sample_count=10,
                                       window_interval_ms=1000, item_offset=0, item_count=0) for k in range(n_param)]
    is_param = rng.random(n_req) < 0.2
    conn = rng.integers(0, n_streams, n_req)
    fid = np.where(is_param, n_flow + 1 + rng.integers(0, n_param, n_req), 1 + rng.integers(0, n_flow, n_req))
    cnt = rng.integers(1, 4, n_req).astype(np.int32)
    prio = rng.random(n_req) < 0.1
    vals = trace.scramble(trace.zipf_bounded(rng, 1.1, n_values, n_req) - 1, n_values).astype(np.int64)
    order = np.argsort(conn, kind="stable")
    size = np.where(is_param, 32, 20)[order]
    start = np.zeros(n_req + 1, np.int64)
    start[1:] = np.cumsum(size)
    buf = np.zeros(int(start[-1]), np.uint8)
    xid = np.arange(n_req, dtype=np.int64)
    for kind, L in ((False, 20), (True, 32)):
        sel = order[is_param[order] == kind]
        pos = start[:-1][is_param[order] == kind]
        rec = np.zeros((sel.size, L), np.uint8)
        rec[:, 0:2] = np.frombuffer(np.full(sel.size, L - 2, ">u2").tobytes(), np.uint8).reshape(-1, 2)
        rec[:, 2:6] = np.frombuffer(xid[sel].astype(">i4").tobytes(), np.uint8).reshape(-1, 4)
        rec[:, 6] = 2 if kind else 1
        rec[:, 7:15] = np.frombuffer(fid[sel].astype(">i8").tobytes(), np.uint8).reshape(-1, 8)
        rec[:, 15:19] = np.frombuffer(cnt[sel].astype(">i4").tobytes(), np.uint8).reshape(-1, 4)
        if kind:
            rec[:, 19:23] = np.frombuffer(np.ones(sel.size, ">i4").tobytes(), np.uint8).reshape(-1, 4)
            rec[:, 23] = 1                                            # PARAM_TYPE_LONG
            rec[:, 24:32] = np.frombuffer(vals[sel].astype(">i8").tobytes(), np.uint8).reshape(-1, 8)
        else:
            rec[:, 19] = prio[sel]
        buf[pos[:, None] + np.arange(L)] = rec
    soff = np.zeros(n_streams + 1, np.int64)
    soff[1:] = np.cumsum(np.bincount(conn, weights=np.where(is_param, 32, 20), minlength=n_streams)).astype(np.int64)
    streams = [buf[soff[s]:soff[s + 1]].tobytes() for s in range(n_streams)]
    return ns, flow, param, streams


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=1 << 22)
    ap.add_argument("--streams", type=int, default=500)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-sample", type=int, default=1 << 20)
    a = ap.parse_args()
    from sentinel_amd import engine
    ns, flow, param, streams = frames(a.requests, a.streams, 7)
    cfg = abi.default_config(max_resources=4, max_batch=a.requests, param_capacity=1 << 22)
    cfg.max_flow_ids = 1 << 15
    e = engine.FlowEngine(cfg)
    e.load_namespaces(ns)
    e.load_cluster_rules(flow, param, [])
    n_bytes = sum(len(s) for s in streams)
    for k in range(a.warmup):
        e.serve_frames(streams, trace.T0 + 1000 * k)
    e.set_timing(True)
    dev = []
    wall = []
    for k in range(a.steps):
        t = time.perf_counter()
        r = e.serve_frames(streams, trace.T0 + 1000 * (a.warmup + k))
        wall.append(time.perf_counter() - t)
        dev.append(e.stats().wire_ms)
    assert r.n_requests == a.requests, (r.n_requests, a.requests)
    ms = float(np.median(dev))
    out = {"what": "sf_serve_frames: C1 frames in -> token decisions -> response frames out",
           "requests": a.requests, "connections": a.streams, "in_bytes": n_bytes, "out_bytes": int(r.n_responses) * 16,
           "device_ms": round(ms, 3), "requests_per_s": round(a.requests / (ms / 1e3), 1),
           "wall_ms_incl_pcie": round(float(np.median(wall)) * 1e3, 2),
           "frame_bytes_GBs": round((n_bytes + r.n_responses * 16) / (ms / 1e3) / 1e9, 2)}
    if a.cpu_sample:
        from oracle import oracle as so
        k = max(1, a.cpu_sample * a.streams // a.requests)
        o = so.OracleEngine(cfg)
        o.load_namespaces(ns)
        o.load_cluster_rules(flow, param, [])
        sub = streams[:k]
        t = time.perf_counter()
        ro = o.serve_frames(sub, trace.T0)
        dt = time.perf_counter() - t
        out["cpu_baseline"] = {"value": round(ro.n_requests / dt, 1), "unit": "requests/s", "cores": 1, "kind": "port",
                               "sample": f"{k} of {a.streams} connections ({ro.n_requests} requests), oracle so_serve_frames"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
