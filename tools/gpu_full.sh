# Full GPU check on the box (repo root): the GPU test suite, then the default
# bench (with the CPU-oracle baseline leg).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 500 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo BENCH_FAILED; tail gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
