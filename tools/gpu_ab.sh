# GPU box: A/B of engine builds on one box: the bench (no CPU legs) once per
# library in $LIBS (paths relative to the repo; default = the product build).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for L in ${LIBS:-sentinel_amd/libsentinel_flow.so}; do
  n=$(basename $L .so)
  SENTINEL_FLOW_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python3 bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --no-cpu --no-metric-log --no-degrade} > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { echo "AB_FAILED $n"; tail -5 gpurun_out/ab_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$n.json')); print('$n', d['ms_per_step'], d['roofline']['kernels_ms'])"
done
