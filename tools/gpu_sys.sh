cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/sys
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "system or param" --timeout 300 --timeout-method thread -s > gpurun_out/sys/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/sys/tests.log; exit 1; }
grep -E "planner rounds|passed|failed" gpurun_out/sys/tests.log
timeout -k 10 400 python3 tools/leg_run.py config4 > gpurun_out/sys/c4.json 2> gpurun_out/sys/c4.err || { echo LEG_FAILED; tail gpurun_out/sys/c4.err; exit 1; }
cat gpurun_out/sys/c4.json
