# GPU box: rocprofv3 kernel trace of one bench leg (LEG=config2|config4, LEG_ARGS), then the kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NAME=${NAME:-ktl_leg}; OUT=gpurun_out/$NAME; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd -d $OUT/kt -o kt -- python3 tools/leg_run.py ${LEG:-config2} ${LEG_ARGS} > $OUT/leg.json 2> $OUT/leg.err || { echo KT_FAILED; tail $OUT/leg.err; exit 1; }
cat $OUT/leg.json
python3 tools/prof_summary.py --kt $(find $OUT/kt -name '*.db' | head -1) --out $OUT/summary && head -40 $OUT/summary_kernels.txt
