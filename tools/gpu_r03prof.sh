# GPU box: THREAD parity tests, then the rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the config-3 bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "thread or config3 or edge" > gpurun_out/thr_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/thr_tests.log; exit 1; }
tail -1 gpurun_out/thr_tests.log
NAME=${NAME:-r03prof} PMC=1 BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-legs --no-degrade --no-metric-log" bash tools/gpu_profile.sh
