# GPU box: GPU tests (K/T as tools/gpu_tests.sh), then a quick bench line (BENCH_ARGS) with its kernel split
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh | tail -2 || exit 1
grep -q " failed\|FAILED\|ERROR" gpurun_out/gpu_tests.log && { echo TESTS_FAILED; exit 1; }
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu --no-metric-log --no-degrade} > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { echo BENCH_FAILED; tail gpurun_out/bench_q.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_q.json')); print(d['value'], d['ms_per_step']); print(d['roofline']['kernels_ms']); print(d.get('parity'))"
