# GPU box: the default bench (no oracle, no legs) under several environment
# variants, REPS rounds of all variants interleaved.  VARIANTS: space-separated
# specs, each a comma-separated list of NAME=VALUE (or "-" for none), e.g.
#   VARIANTS="SF_SIDE=0 SF_SIDE=1,GPU_MAX_HW_QUEUES=8 SF_SIDE=2"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NAME=${NAME:-var}; OUT=gpurun_out/$NAME; rm -rf $OUT; mkdir -p $OUT
i=0
for r in $(seq ${REPS:-2}); do
  for spec in ${VARIANTS}; do
    i=$((i+1))
    envs=""
    if [ "$spec" != "-" ]; then envs=$(echo "$spec" | tr ',' ' '); fi
    env $envs timeout -k 10 240 python3 -u bench.py --no-cpu --steps 10 --warmup 3 --no-legs --no-degrade --no-metric-log ${BENCH_ARGS} > $OUT/b_$i.json 2> $OUT/b_$i.err || { echo BENCH_FAILED $spec; tail -20 $OUT/b_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_$i.json')); print('$spec', d['ms_per_step'], d['roofline']['kernels_ms'])"
  done
done
