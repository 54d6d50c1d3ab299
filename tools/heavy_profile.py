"""Diagnostics: time every heavy segment of a config-3 batch on the GPU and
print the slowest ones with their algorithm (SM_* in sf_heavy.h)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from sentinel_amd import abi, engine, trace  # noqa: E402

engine.lib()
MODES = {1: "GENERIC", 2: "QPS", 3: "WARM", 4: "RL", 5: "NORULE", 6: "THREAD"}

ap = argparse.ArgumentParser()
ap.add_argument("--resources", type=int, default=10_000_000)
ap.add_argument("--events", type=int, default=1 << 27)
ap.add_argument("--top", type=int, default=25)
a = ap.parse_args()
grade, beh, count = trace.mixed_rule_table(a.resources, seed=3)
rules = abi.flow_rules_np(np.arange(a.resources, dtype=np.uint32), grade, count, beh)
hb = trace.mixed_zipf(a.resources, a.events, duration_ms=4000, seed=3)
eng = engine.FlowEngine(abi.default_config(max_resources=a.resources, max_batch=hb.n))
eng.load_flow_rules(rules)
b0 = engine.DeviceBatch(eng, hb)
b1 = engine.DeviceBatch(eng, abi.HostBatch(hb.res_id, hb.ts_ms + 4000, hb.count, hb.flags, entry_ref=hb.entry_ref))
out = engine.DeviceVerdicts(eng, hb.n)
eng.submit_device(b0, out)
eng.set_timing(True)
eng.submit_device(b1, out)
eng.sync()
st = eng.stats()
print(f"light {st.light_ms:.2f} ms  heavy_decide {st.heavy_decide_ms:.2f} ms  stream {st.stream_ms:.2f} ms  fill {st.heavy_fill_ms:.2f} ms  "
      f"sort {st.sort_ms:.2f} ms  scatter {st.scatter_ms:.2f} ms")
prof = eng.heavy_profile()
prof.sort(key=lambda x: -x[3])
by_mode = {}
for r, n, m, us in prof:
    d = by_mode.setdefault(MODES.get(m, m), [0, 0, 0.0, 0.0])
    d[0] += 1; d[1] += n; d[2] += us; d[3] = max(d[3], us)
print("mode       segs     events    sum_us     max_us")
for k, (c, n, s, mx) in sorted(by_mode.items()):
    print(f"{k:8s} {c:6d} {n:10d} {s:10.0f} {mx:10.0f}")
print("slowest segments: resource events mode us ns/event rule(grade,behavior,count)")
for r, n, m, us in prof[:a.top]:
    print(f"{r:9d} {n:9d} {MODES.get(m, m):8s} {us:9.0f} {us*1e3/max(n,1):7.2f}  ({grade[r]},{beh[r]},{count[r]})")
