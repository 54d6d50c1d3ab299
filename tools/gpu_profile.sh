# rocprofv3 passes over the default bench (run on the GPU box from the repo root):
#   NAME=<dir under gpurun_out>  PMC=1 (add FETCH_SIZE / WRITE_SIZE passes)
#   BENCH_ARGS (default "--steps 3 --warmup 1 --no-cpu")
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NAME=${NAME:-prof}; OUT=gpurun_out/$NAME; mkdir -p $OUT
ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd -d $OUT/kt -o kt -- python3 bench.py $ARGS \
    > $OUT/bench.json 2> $OUT/bench.err || { echo KT_FAILED; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
KT=$(find $OUT/kt -name '*.db' | head -1)
if [ -n "$PMC" ]; then
    timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format rocpd -d $OUT/fetch -o fetch -- python3 bench.py $ARGS \
        > $OUT/fetch.log 2>&1 || { echo FETCH_FAILED; tail $OUT/fetch.log; exit 1; }
    timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format rocpd -d $OUT/write -o write -- python3 bench.py $ARGS \
        > $OUT/write.log 2>&1 || { echo WRITE_FAILED; tail $OUT/write.log; exit 1; }
    python3 tools/prof_summary.py --kt $KT --fetch $(find $OUT/fetch -name '*.db' | head -1) \
        --write $(find $OUT/write -name '*.db' | head -1) --out $OUT/summary
else
    python3 tools/prof_summary.py --kt $KT --out $OUT/summary
fi
cat $OUT/summary_kernels.txt
