# GPU box: A/B of the sort phase -- microbench, GPU tests on the new sort, config-3 step with each sort
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${NAME:-sortab}; rm -rf $OUT; mkdir -p $OUT
for bin in tools/micro/rsb_*; do [ -x $bin ] && { timeout -k 10 60 $bin >> $OUT/rs.txt 2>&1 || exit 1; }; done
[ -f $OUT/rs.txt ] && cat $OUT/rs.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in ${VARIANTS:-new old new old}; do
  if [ $v = old ]; then export SF_SORT_ROCPRIM=1; else unset SF_SORT_ROCPRIM; fi
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-legs --no-degrade --no-metric-log ${BENCH_ARGS} > $OUT/b_$v.json 2> $OUT/b_$v.err || { echo BENCH_FAILED $v; tail -20 $OUT/b_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/b_$v.json')); print('$v', d['ms_per_step'], d.get('parity',{}).get('exact'), d.get('parity',{}).get('steady_state',{}).get('exact'))"
done
