# GPU box: a subset (K=...) or all of the GPU tests, verbose, with per-test timeout.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
SEL=()
[ -n "$K" ] && SEL=(-k "$K")
timeout -k 10 ${T:-500} python -u -m pytest ${FILES:-tests} -m gpu -x -v -s --timeout 150 --timeout-method thread "${SEL[@]}" > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|planner|passed|failed" gpurun_out/gpu_tests.log | tail -40
[ $rc -ne 0 ] && tail -40 gpurun_out/gpu_tests.log
exit $rc
