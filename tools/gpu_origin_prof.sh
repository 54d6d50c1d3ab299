# GPU box: the config3_origin leg (tools/origin_ab.py, no parity) under rocprofv3:
# kernel trace and, with PMC=1, FETCH_SIZE / WRITE_SIZE passes -> summary
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=${V:-no_origin_rules}; OUT=gpurun_out/${NAME:-origin_$V}; rm -rf $OUT; mkdir -p $OUT
CMD="python3 tools/origin_ab.py $V 2"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd -d $OUT/kt -o kt -- $CMD > $OUT/leg.json 2> $OUT/kt.err || { echo KT_FAILED; tail $OUT/kt.err; exit 1; }
cat $OUT/leg.json
KT=$(find $OUT/kt -name '*.db' | head -1)
if [ -n "$PMC" ]; then
    timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format rocpd -d $OUT/fetch -o fetch -- $CMD > $OUT/fetch.log 2>&1 || { echo FETCH_FAILED; tail $OUT/fetch.log; exit 1; }
    timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format rocpd -d $OUT/write -o write -- $CMD > $OUT/write.log 2>&1 || { echo WRITE_FAILED; tail $OUT/write.log; exit 1; }
    python3 tools/prof_summary.py --kt $KT --fetch $(find $OUT/fetch -name '*.db' | head -1) --write $(find $OUT/write -name '*.db' | head -1) --out $OUT/summary
else
    python3 tools/prof_summary.py --kt $KT --out $OUT/summary
fi
head -25 $OUT/summary_kernels.txt
