# GPU box: kernel timeline (per-kernel totals) of one config-4 batch with its SystemRule
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && OUT=gpurun_out/c4tl; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/kt -o kt -- python3 tools/system_bench.py --reps 1 --no-check --qps-frac ${QF:-0.6} > $OUT/c4.json 2> $OUT/c4.err || { echo FAILED; tail $OUT/c4.err; exit 1; }
python3 - $(find $OUT/kt -name '*.db' | head -1) <<'PY'
import re, sqlite3, sys
from collections import defaultdict
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels order by start").fetchall()
tot = defaultdict(lambda: [0, 0.0])
for n, s, e in rows:
    k = re.sub(r'\(.*', '', n)[:70]
    tot[k][0] += 1; tot[k][1] += (e - s) / 1e6
span = (rows[-1][2] - rows[0][1]) / 1e6
print(f"span {span:.1f} ms, {len(rows)} kernels")
for k, (cnt, ms) in sorted(tot.items(), key=lambda x: -x[1][1])[:18]:
    print(f"{ms:9.3f} ms {cnt:6d}  {k}")
PY
