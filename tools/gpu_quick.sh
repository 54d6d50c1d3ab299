cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -n "$HEAVY_PROFILE" ]; then timeout -k 10 200 python -u tools/heavy_profile.py > gpurun_out/heavy_profile.txt 2>&1 || { echo PROFILE_FAILED; tail gpurun_out/heavy_profile.txt; exit 1; }; head -30 gpurun_out/heavy_profile.txt; fi
