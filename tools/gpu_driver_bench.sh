# GPU box: the GPU test suite, smoke(), then the driver's exact bench command.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
T0=$(date +%s); timeout -k 10 560 python3 bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench_driver.err; exit 1; }
cat gpurun_out/bench_driver.json
echo "bench wall $(( $(date +%s) - T0 )) s"
