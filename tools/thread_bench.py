"""Diagnostics: one heavy THREAD-grade resource alone on the GPU (k_heavy_stream
SM_THREAD path), at several densities and thresholds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from sentinel_amd import abi, engine, trace  # noqa: E402

engine.lib()
CHECK = os.environ.get("CHECK", "1") == "1"


def one(n_entry, count, rt_mean=20.0, duration=4000, seed=1, exits=True):
    rng = np.random.default_rng(seed)
    ts = np.sort(rng.integers(0, duration, n_entry)).astype(np.int64) + trace.T0
    acq = np.ones(n_entry, np.int32)
    multi = rng.random(n_entry) < 0.1
    acq[multi] = rng.integers(2, 6, int(multi.sum()))
    if exits:
        rt = np.floor(rng.exponential(rt_mean, n_entry)).astype(np.int64)
        ets = np.minimum(ts + rt, trace.T0 + duration - 1)
        all_ts = np.concatenate([ts, ets])
        isx = np.concatenate([np.zeros(n_entry, bool), np.ones(n_entry, bool)])
        order = np.lexsort((isx, all_ts))
        pos = np.empty(order.size, np.int64)
        pos[order] = np.arange(order.size)
        src = np.concatenate([np.arange(n_entry), np.arange(n_entry)])
        fl = np.where(isx[order], abi.EV_EXIT | abi.EV_IN, abi.EV_IN).astype(np.uint8)
        eref = np.full(order.size, -1, np.int64)
        eref[pos[n_entry:]] = pos[:n_entry]
        b = abi.HostBatch(np.zeros(order.size, np.uint32), all_ts[order], acq[src][order], fl, entry_ref=eref)
    else:
        b = abi.HostBatch(np.zeros(n_entry, np.uint32), ts, acq, np.full(n_entry, abi.EV_IN, np.uint8))
    rules = [abi.sf_flow_rule(resource=0, grade=abi.GRADE_THREAD, count=float(count), control_behavior=0)]
    cfg = abi.default_config(max_resources=1, max_batch=b.n)
    e = engine.FlowEngine(cfg)
    e.load_flow_rules(rules)
    db = engine.DeviceBatch(e, b)
    out = engine.DeviceVerdicts(e, b.n)
    e.set_timing(True)
    e.submit_device(db, out)
    e.sync()
    st = e.stats()
    prof = e.heavy_profile()
    us = prof[0][3] if prof else -1
    npass = int((out.status.numpy() == abi.V_PASS).sum())
    if CHECK and b.n <= 6_000_000:
        from oracle import oracle as so
        o = so.OracleEngine(cfg)
        o.load_flow_rules(rules)
        want = o.submit(b)
        o.close()
        assert (want.status == out.status.numpy()).all(), "verdicts differ from the oracle"
    print(f"entries {n_entry:9d} events {b.n:9d} count {count:5d} exits {exits}: stream {st.stream_ms:8.3f} ms "
          f"segment {us:9.0f} us  {us * 1e3 / b.n:7.2f} ns/event  passes {npass}", flush=True)


if len(sys.argv) > 2:                      # one case: entries count [noexit]
    one(int(sys.argv[1]), int(sys.argv[2]), exits=len(sys.argv) < 4)
else:
    for n, cnt in [(2_430_000, 242), (150_000, 525), (2_430_000, 100000), (150_000, 100000)]:
        one(n, cnt)
    one(2_430_000, 242, exits=False)
    one(150_000, 525, rt_mean=200.0)
