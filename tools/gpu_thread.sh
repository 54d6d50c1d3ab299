# GPU box: the THREAD-grade GPU parity tests, then the head-segment timing (tools/thread_bench.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "thread or config3 or edge" > gpurun_out/thr_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/thr_tests.log; exit 1; }
tail -2 gpurun_out/thr_tests.log
timeout -k 10 200 python -u tools/thread_bench.py > gpurun_out/thr_bench.log 2>&1 || { echo TB_FAILED; tail -20 gpurun_out/thr_bench.log; exit 1; }
cat gpurun_out/thr_bench.log
