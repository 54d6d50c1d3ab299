# GPU box: one bench leg per library variant (sentinel_amd/variants/*.so + the main one) under a kernel trace
#   LEG=config2 LEG_ARGS=... VARIANTS="qc4 qc16" bash tools/gpu_variants.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NAME=${NAME:-variants}; OUT=gpurun_out/$NAME; rm -rf $OUT; mkdir -p $OUT
for v in main $VARIANTS; do
  if [ $v = main ]; then lib=$PWD/sentinel_amd/libsentinel_flow.so; else lib=$PWD/sentinel_amd/variants/$v.so; fi
  echo "== $v"
  SENTINEL_FLOW_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o kt -- python3 tools/leg_run.py ${LEG:-config2} $LEG_ARGS > $OUT/$v.json 2> $OUT/$v.err || { echo "RUN_FAILED $v"; tail $OUT/$v.err; exit 1; }
  cat $OUT/$v.json
  f=$(find $OUT/$v -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:10]:
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1e6:9.3f} ms avg {float(r["TotalDurationNs"])/1e6:9.3f} ms tot')
PY
done
