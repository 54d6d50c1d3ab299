"""Kernel timeline of the last two batches of a rocprofv3 rocpd database (diagnostics)."""
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
rows = [r for r in rows if 'copyBuffer' not in r[0] and 'fillBuffer' not in r[0]]
# a batch starts with its sort's first kernel (the hand-written sort's batch-source count, or k_keys_packed)
idx = [i for i, r in enumerate(rows) if 'k_keys_packed' in r[0] or ('k_rs_count' in r[0] and 'RsBatchSrc' in r[0])]
sel = rows[idx[-2]:]
t0 = sel[0][1]
for n, s, e, sid in sel:
    short = re.sub(r'\(.*', '', n)
    short = re.sub(r'rocprim::ROCPRIM_\w+::detail::', 'rp::', short)[:90]
    print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f} s{sid} {short}")
