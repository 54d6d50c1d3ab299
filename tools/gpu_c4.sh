# GPU box: GPU tests, then config 4 with its SystemRule (tools/system_bench.py, oracle-checked)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh | tail -2 || exit 1
grep -q " failed\|FAILED\|ERROR" gpurun_out/gpu_tests.log && { echo TESTS_FAILED; exit 1; }
timeout -k 10 500 python -u tools/system_bench.py ${C4_ARGS:---reps 2} > gpurun_out/c4.json 2> gpurun_out/c4.err || { echo C4_FAILED; tail gpurun_out/c4.err; exit 1; }
cat gpurun_out/c4.json
