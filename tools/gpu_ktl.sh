# GPU box: rocprofv3 kernel trace of a short bench (env passed through, e.g. SF_SERIAL_STREAMS=1),
# then the kernel timeline of the last batch (tools/timeline.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NAME=${NAME:-ktl}; OUT=gpurun_out/$NAME; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/kt -o kt -- python3 bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu --no-metric-log --no-degrade} > $OUT/bench.json 2> $OUT/bench.err || { echo KT_FAILED; tail $OUT/bench.err; exit 1; }
python3 tools/timeline.py $(find $OUT/kt -name '*.db' | head -1)
