# GPU box: the config-4 leg (timing only) for the product library and each variant, twice, same box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for k in 1 2; do
for v in main ${VARS}; do
  if [ $v = main ]; then lib=$PWD/sentinel_amd/libsentinel_flow.so; else lib=$PWD/sentinel_amd/variants/$v.so; fi
  SENTINEL_FLOW_LIB=$lib timeout -k 10 300 python3 tools/system_bench.py --qps-frac 0.6 --reps 3 --no-check > gpurun_out/c4_$v.json 2> gpurun_out/c4_$v.err || { echo FAIL $v; tail -3 gpurun_out/c4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4_$v.json')); print('$v', d['ms_per_batch'], d['reps_ms'], d['planner_rounds'])"
done
done
