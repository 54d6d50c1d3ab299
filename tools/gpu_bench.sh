# GPU box: the driver's bench command alone (stderr progress to gpurun_out/bench_driver.err)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T0=$(date +%s); timeout -k 10 ${T:-900} python3 bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${ARGS} > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench_driver.err; exit 1; }
cat gpurun_out/bench_driver.json
echo "bench wall $(( $(date +%s) - T0 )) s"
