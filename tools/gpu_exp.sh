# GPU box: quick bench (no parity) for each library variant in VARS, kernel split only
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in ${VARS:-sentinel_flow}; do
SENTINEL_FLOW_LIB=$PWD/sentinel_amd/lib$v.so timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---steps 4 --warmup 1 --no-cpu --no-metric-log --no-degrade} > gpurun_out/exp_$v.json 2> gpurun_out/exp_$v.err || { echo FAIL $v; tail -3 gpurun_out/exp_$v.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/exp_$v.json')); print('$v', d['value'], d['ms_per_step']); print(d['roofline']['kernels_ms'])"
done
