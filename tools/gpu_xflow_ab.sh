# GPU box: the xflow + GPU parity tests, then the A/B bench of $LIBS (tools/gpu_ab.sh).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_xflow.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/xflow_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/xflow_tests.log; exit 1; }
tail -2 gpurun_out/xflow_tests.log
bash tools/gpu_ab.sh
