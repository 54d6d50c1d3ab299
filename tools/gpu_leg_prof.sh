# GPU box: one bench leg (tools/leg_run.py LEG [k=v ...]) under rocprofv3: serialized kernel trace
# (SF_SERIAL_STREAMS=1) and, with PMC=1, FETCH_SIZE / WRITE_SIZE passes of the pipelined run
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
LEG=${LEG:-config2}; OUT=gpurun_out/${NAME:-leg_$LEG}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python3 tools/leg_run.py $LEG parity=0 $LEG_ARGS > $OUT/leg.json 2> $OUT/leg.err || { echo LEG_FAILED; tail $OUT/leg.err; exit 1; }
cat $OUT/leg.json
SF_SERIAL_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd -d $OUT/kt -o kt -- python3 tools/leg_run.py $LEG parity=0 $LEG_ARGS > $OUT/leg_serial.json 2> $OUT/kt.err || { echo KT_FAILED; tail $OUT/kt.err; exit 1; }
KT=$(find $OUT/kt -name '*.db' | head -1)
if [ -n "$PMC" ]; then
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format rocpd -d $OUT/fetch -o fetch -- python3 tools/leg_run.py $LEG parity=0 $LEG_ARGS > $OUT/fetch.log 2>&1 || { echo FETCH_FAILED; tail $OUT/fetch.log; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format rocpd -d $OUT/write -o write -- python3 tools/leg_run.py $LEG parity=0 $LEG_ARGS > $OUT/write.log 2>&1 || { echo WRITE_FAILED; tail $OUT/write.log; exit 1; }
    python3 tools/prof_summary.py --kt $KT --fetch $(find $OUT/fetch -name '*.db' | head -1) --write $(find $OUT/write -name '*.db' | head -1) --out $OUT/summary
else
    python3 tools/prof_summary.py --kt $KT --out $OUT/summary
fi
head -30 $OUT/summary_kernels.txt
