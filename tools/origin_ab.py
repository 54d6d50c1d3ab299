"""A/B of the config3_origin leg (no parity) for one engine library
(SENTINEL_FLOW_LIB): python tools/origin_ab.py [variant,...] [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import bench  # noqa: E402
from sentinel_amd import abi, trace  # noqa: E402

variants = (sys.argv[1] if len(sys.argv) > 1 else "other_rules_1pct").split(",")
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
R = 10_000_000
t0 = time.time()
g, b, c = trace.mixed_rule_table(R, seed=3)
rules = abi.flow_rules_np(np.arange(R, dtype=np.uint32), g, c, b)
hb = trace.mixed_zipf(R, 1 << 27, duration_ms=bench.DURATION_MS, seed=3)
print(f"trace {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
out = bench.config3_origin_leg(hb, rules, R, 15.5, steps=steps, warmup=1, parity=False, variants=variants)
print(json.dumps({"lib": os.environ.get("SENTINEL_FLOW_LIB", "default"),
                  **{k: {kk: v[kk] for kk in ("ms_per_step", "batch0_ms", "wave_walk") if kk in v}
                     for k, v in out.items() if isinstance(v, dict)}}), flush=True)
