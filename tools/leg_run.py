"""Run one of bench.py's legs alone (profiling / A-B): python tools/leg_run.py config2|config4|config5"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

leg = sys.argv[1]
kw = {}
for a in sys.argv[2:]:
    k, v = a.split("=")
    kw[k] = int(v) if v.lstrip("-").isdigit() else float(v)
print(json.dumps(getattr(bench, leg + "_leg")(**kw)))
