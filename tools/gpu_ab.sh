# GPU box: GPU parity tests, then an A/B of an environment switch on the default bench
# (VAR=<env name>; variants "new" = unset, "old" = VAR=1), and optionally a leg (LEG=config2) per variant
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NAME=${NAME:-ab}; OUT=gpurun_out/$NAME; rm -rf $OUT; mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
i=0
for v in ${VARIANTS:-new old new old}; do
  i=$((i+1))
  if [ $v = old ]; then export $VAR=${VAR_VALUE:-1}; else unset $VAR; fi
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-legs --no-degrade --no-metric-log ${BENCH_ARGS} > $OUT/b_${v}_$i.json 2> $OUT/b_${v}_$i.err || { echo BENCH_FAILED $v; tail -20 $OUT/b_${v}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/b_${v}_$i.json')); p=d.get('parity') or {}; print('$v', d['ms_per_step'], d['roofline']['kernels_ms'], p.get('exact'), (p.get('steady_state') or {}).get('exact'))"
  if [ -n "$LEG" ]; then
    timeout -k 10 300 python3 tools/leg_run.py $LEG $LEG_ARGS > $OUT/leg_$v.json 2> $OUT/leg_$v.err || { echo LEG_FAILED $v; tail -20 $OUT/leg_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/leg_$v.json')); print('$v leg', d.get('ms_per_step', d.get('ms_per_batch')), d.get('parity'))"
  fi
done
