# GPU box: the new parity tests, the N=2 rehearsal on one GPU, then the driver's bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "node_wide or long_run" > gpurun_out/gpu_tests_new.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests_new.log; exit 1; }
tail -2 gpurun_out/gpu_tests_new.log
bash tools/gpu_two_ranks_one_gpu.sh || { echo N2_FAILED; tail -20 gpurun_out/n2_rank0.err; tail -20 gpurun_out/n2_rank1.err; exit 1; }
bash tools/gpu_bench.sh
