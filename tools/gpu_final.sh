# GPU box: the round's final evidence -- GPU tests, the driver's default bench
# line, and the config-3 profile (kernel trace + FETCH_SIZE / WRITE_SIZE passes)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${NAME:-final}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 900 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['value'], d.get('parity',{}).get('exact'))"
if [ -n "$PROF" ]; then NAME=${NAME:-final}/prof PMC=1 BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-legs --no-degrade --no-metric-log" bash tools/gpu_profile.sh > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail $OUT/prof.log; exit 1; }; head -30 $OUT/prof/summary_kernels.txt; fi
