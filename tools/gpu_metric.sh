cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "metric or snapshot" > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -5 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
