# GPU box: SQ counters per kernel of a short serialized bench (tools/sq_summary.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${NAME:-sq}; rm -rf $OUT; mkdir -p $OUT
CTRS=${CTRS:-SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD}
SF_SERIAL_STREAMS=1 timeout -s KILL 400 rocprofv3 --pmc $CTRS --output-format rocpd -d $OUT/sq -o sq -- python3 bench.py ${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu --no-metric-log --no-degrade --no-legs} > $OUT/bench.json 2> $OUT/bench.err || { echo SQ_FAILED; tail $OUT/bench.err; exit 1; }
python3 tools/sq_summary.py $(find $OUT/sq -name '*.db' | head -1) | tee $OUT/sq.txt
