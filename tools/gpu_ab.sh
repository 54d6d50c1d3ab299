# GPU box: GPU parity tests, one leg under a kernel trace, then the default bench (A/B of a kernel change)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NAME=${NAME:-ab}; OUT=gpurun_out/$NAME; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
if [ -n "$LEG" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd -d $OUT/kt -o kt -- python3 tools/leg_run.py $LEG $LEG_ARGS > $OUT/leg.json 2> $OUT/leg.err || { echo KT_FAILED; tail $OUT/leg.err; exit 1; }
  cat $OUT/leg.json
  python3 tools/prof_summary.py --kt $(find $OUT/kt -name '*.db' | head -1) --out $OUT/summary && head -25 $OUT/summary_kernels.txt
fi
timeout -k 10 600 python3 -u bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
