"""Per-kernel SQ counters from a rocprofv3 --pmc database (tools/gpu_sq.sh).

Prints, per kernel (averaged over its dispatches): waves, wave-cycles per wave,
and the split of wave time into active / waiting at s_waitcnt (memory) /
issue-stalled, VALU instructions per wave and vector-memory reads per wave.
SQ_WAVE_CYCLES, SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles
(MI355X_MICROARCH.md, rocprofv3 PMC slots).
"""
import sqlite3
import sys
from collections import defaultdict

from prof_summary import short


def main(db):
    c = sqlite3.connect(db)
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for name, cn, v, did in c.execute("select name, counter_name, counter_value, dispatch_id from pmc_events"):
        k = short(name)
        acc[k][cn] += float(v)
        disp[k].add(did)
    rows = []
    for k, d in acc.items():
        n = max(1, len(disp[k]))
        w = d.get("SQ_WAVES", 0) / n
        cyc = d.get("SQ_WAVE_CYCLES", 0)
        f = (lambda x: d.get(x, 0) / cyc if cyc else 0.0)
        rows.append((cyc / n, k, w, (cyc / n) / w if w else 0, f("SQ_ACTIVE_INST_ANY"), f("SQ_WAIT_ANY"),
                     f("SQ_WAIT_INST_ANY"), f("SQ_ACTIVE_INST_VALU"),
                     d.get("SQ_INSTS_VALU", 0) / n / w if w else 0, d.get("SQ_INSTS_VMEM_RD", 0) / n / w if w else 0))
    print(f"{'kernel':52s} {'waves':>8s} {'qcyc/wave':>10s} {'active':>7s} {'waitmem':>7s} {'waitiss':>7s} "
          f"{'valu':>6s} {'valu/w':>8s} {'vmrd/w':>7s}")
    for r in sorted(rows, reverse=True)[:40]:
        print(f"{r[1][:52]:52s} {r[2]:8.0f} {r[3]:10.0f} {r[4]:7.2f} {r[5]:7.2f} {r[6]:7.2f} {r[7]:6.2f} {r[8]:8.0f} {r[9]:7.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
