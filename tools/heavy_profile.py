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
for r, n, m, us, _ in prof:
    d = by_mode.setdefault(MODES.get(m, m), [0, 0, 0.0, 0.0])
    d[0] += 1; d[1] += n; d[2] += us; d[3] = max(d[3], us)
print("mode       segs     events    sum_us     max_us")
for k, (c, n, s, mx) in sorted(by_mode.items()):
    print(f"{k:8s} {c:6d} {n:10d} {s:10.0f} {mx:10.0f}")
print("slowest segments: resource events mode us ns/event start_us end_us rule(grade,behavior,count)")
for r, n, m, us, t0 in prof[:a.top]:
    print(f"{r:9d} {n:9d} {MODES.get(m, m):8s} {us:9.0f} {us*1e3/max(n,1):7.2f} {t0:8.0f} {t0+us:8.0f}  "
          f"({grade[r]},{beh[r]},{count[r]})")
st_ = [(t0 + us, t0, n, MODES.get(m, m)) for r, n, m, us, t0 in prof if m in (4, 6)]
st_.sort(reverse=True)
print("latest-ending stream segments: end_us start_us events mode")
for e_, t0, n, m in st_[:10]:
    print(f"{e_:9.0f} {t0:9.0f} {n:9d} {m}")
# concurrency of k_heavy_stream segments over time (1 ms bins)
if st_:
    end = max(e_ for e_, _, _, _ in st_)
    nb = int(end // 1000) + 1
    started = [0] * nb; active = [0.0] * nb
    for e_, t0, n, m in st_:
        started[int(t0 // 1000)] += 1
        for b in range(int(t0 // 1000), int(e_ // 1000) + 1):
            lo_, hi_ = max(t0, b * 1000), min(e_, (b + 1) * 1000)
            active[b] += max(0.0, hi_ - lo_) / 1000
    print("ms  started  mean_active  (k_heavy_stream segments)")
    for b in range(nb):
        print(f"{b:3d} {started[b]:8d} {active[b]:10.1f}")
