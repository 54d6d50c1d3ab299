# GPU box: the GPU suite, then the bench's config-4 leg (SystemRule at 0.6x offered, every verdict vs the oracle)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error" gpurun_out/gpu_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python3 tools/leg_run.py config4 > gpurun_out/c4leg.json 2> gpurun_out/c4leg.err || { echo C4_FAILED; tail gpurun_out/c4leg.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c4leg.json')); print({k: d[k] for k in ('ms_per_batch','planner_rounds','system_blocks','param_blocks','reps_ms')}, d['parity'])"
