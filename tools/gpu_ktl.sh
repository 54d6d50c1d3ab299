# GPU box: rocprofv3 kernel trace of a short bench (env passed through, e.g. SF_SERIAL_STREAMS=1),
# then the kernel timeline of the last batch (tools/timeline.py); VARIANTS="new old" A/B of the sort
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NAME=${NAME:-ktl}
for v in ${VARIANTS:-cur}; do
  OUT=gpurun_out/$NAME/$v; rm -rf $OUT; mkdir -p $OUT
  if [ $v = old ]; then export SF_SORT_ROCPRIM=1; else unset SF_SORT_ROCPRIM; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/kt -o kt -- python3 bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu --no-metric-log --no-degrade --no-legs} > $OUT/bench.json 2> $OUT/bench.err || { echo KT_FAILED; tail $OUT/bench.err; exit 1; }
  python3 tools/timeline.py $(find $OUT/kt -name '*.db' | head -1) > $OUT/timeline.txt
  echo "== $v"; head -40 $OUT/timeline.txt
done
