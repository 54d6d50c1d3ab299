"""Summarise rocprofv3 output databases into the files committed under profiles/.

Usage:
  python tools/prof_summary.py --kt gpurun_out/prof/kt/kt_results.db \
      [--fetch .../fetch_results.db] [--write .../write_results.db] --out profiles/r01_config3

Writes <out>_kernels.txt (per-kernel dispatch count, average / total duration,
the --kernel-trace --stats view) and <out>_summary.json (the same plus HBM
traffic per launch from the FETCH_SIZE / WRITE_SIZE passes).

HBM traffic follows MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are
reported in KiB; on gfx950 FETCH_SIZE counts half the bytes of wide coalesced
streaming reads, so the fetch figure is doubled (``fetch_bytes_corrected``) and
the raw value is kept next to it.
"""
import argparse
import json
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0]
    for p in ("void ", "sf::"):
        n = n.replace(p, "")
    if "rocprim" in n:
        n = "rocprim::" + name.split("::")[-1].split("(")[0][:60]
    return n


def kernel_stats(db):
    c = sqlite3.connect(db)
    out = defaultdict(lambda: {"count": 0, "total_ns": 0})
    for name, dur in c.execute("select name, end - start from kernels"):
        d = out[short(name)]
        d["count"] += 1
        d["total_ns"] += dur
    return out


def pmc(db, counter):
    c = sqlite3.connect(db)
    out = defaultdict(list)
    for name, v in c.execute("select name, counter_value from pmc_events where counter_name = ?", (counter,)):
        out[short(name)].append(float(v) * 1024.0)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kt", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--out", required=True)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    ks = kernel_stats(a.kt)
    fetch = pmc(a.fetch, "FETCH_SIZE") if a.fetch else {}
    write = pmc(a.write, "WRITE_SIZE") if a.write else {}
    rows = []
    for k, d in sorted(ks.items(), key=lambda kv: -kv[1]["total_ns"]):
        r = {"kernel": k, "count": d["count"], "avg_ms": d["total_ns"] / d["count"] / 1e6,
             "total_ms": d["total_ns"] / 1e6}
        if k in fetch:
            f = sum(fetch[k]) / len(fetch[k])
            r["fetch_bytes_raw"] = f
            r["fetch_bytes_corrected"] = 2 * f
        if k in write:
            r["write_bytes"] = sum(write[k]) / len(write[k])
        if "fetch_bytes_corrected" in r and "write_bytes" in r:
            r["hbm_bytes_per_launch"] = r["fetch_bytes_corrected"] + r["write_bytes"]
        rows.append(r)
    with open(a.out + "_summary.json", "w") as f:
        json.dump({"note": a.note, "kernels": rows}, f, indent=1)
    with open(a.out + "_kernels.txt", "w") as f:
        if a.note:
            f.write(a.note + "\n")
        f.write(f"{'kernel':60s} {'count':>5s} {'avg_ms':>9s} {'total_ms':>9s} {'fetch_MB(x2)':>12s} {'write_MB':>9s}\n")
        for r in rows:
            fb = r.get("fetch_bytes_corrected")
            wb = r.get("write_bytes")
            f.write(f"{r['kernel'][:60]:60s} {r['count']:5d} {r['avg_ms']:9.3f} {r['total_ms']:9.3f} "
                    f"{(fb / 1e6 if fb is not None else float('nan')):12.1f} "
                    f"{(wb / 1e6 if wb is not None else float('nan')):9.1f}\n")
    print(open(a.out + "_kernels.txt").read())


if __name__ == "__main__":
    main()
