# DegradeSlot bench + rocprofv3 kernel trace (run on the GPU box from the repo root).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/degrade; mkdir -p $OUT
timeout -k 10 300 python3 tools/degrade_bench.py ${DG_ARGS:-} --check > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 200 python3 tools/degrade_bench.py ${DG_ARGS:-} --zipf 0.6 --cpu-sample 0 --check > $OUT/bench_mild.json 2> $OUT/bench_mild.err || { echo BENCH2_FAILED; tail $OUT/bench_mild.err; exit 1; }
cat $OUT/bench_mild.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd -d $OUT/kt -o kt -- python3 tools/degrade_bench.py \
    ${DG_ARGS:-} --steps 3 --warmup 1 --cpu-sample 0 > $OUT/kt_bench.json 2> $OUT/kt.err || { echo KT_FAILED; tail $OUT/kt.err; exit 1; }
KT=$(find $OUT/kt -name '*.db' | head -1)
if [ -n "$PMC" ]; then
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format rocpd -d $OUT/fetch -o fetch -- python3 tools/degrade_bench.py \
        ${DG_ARGS:-} --steps 3 --warmup 1 --cpu-sample 0 > $OUT/fetch.log 2>&1 || { echo FETCH_FAILED; tail $OUT/fetch.log; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format rocpd -d $OUT/write -o write -- python3 tools/degrade_bench.py \
        ${DG_ARGS:-} --steps 3 --warmup 1 --cpu-sample 0 > $OUT/write.log 2>&1 || { echo WRITE_FAILED; tail $OUT/write.log; exit 1; }
    python3 tools/prof_summary.py --kt $KT --fetch $(find $OUT/fetch -name '*.db' | head -1) \
        --write $(find $OUT/write -name '*.db' | head -1) --out $OUT/summary
else
    python3 tools/prof_summary.py --kt $KT --out $OUT/summary
fi
cat $OUT/summary_kernels.txt
