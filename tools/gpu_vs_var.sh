# GPU box: verdict-scatter tile variants (sentinel_amd/variants/<v>.so): scatter parity test,
# serialized scatter kernel times, then the pipelined bench, per variant
#   VARS="vs512 vs1024" bash tools/gpu_vs_var.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/vsvar
A="--steps 10 --warmup 3 --no-cpu --no-metric-log --no-degrade --no-legs"
for v in main $VARS; do
  if [ $v = main ]; then lib=$PWD/sentinel_amd/libsentinel_flow.so; else lib=$PWD/sentinel_amd/variants/$v.so; fi
  echo "== $v"
  SENTINEL_FLOW_LIB=$lib timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "scatter" > gpurun_out/vsvar/$v.tests 2>&1 || { echo TESTS_FAILED; tail -20 gpurun_out/vsvar/$v.tests; exit 1; }
  tail -1 gpurun_out/vsvar/$v.tests
  SENTINEL_FLOW_LIB=$lib SF_SERIAL_STREAMS=1 NAME=vsktl_$v BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-metric-log --no-degrade --no-legs" bash tools/gpu_ktl.sh > gpurun_out/vsvar/$v.ktl 2>&1 || { echo KTL_FAILED; tail gpurun_out/vsvar/$v.ktl; exit 1; }
  grep -E "vs_" gpurun_out/vsvar/$v.ktl | tail -3; rm -rf gpurun_out/vsktl_$v
done
for k in 1 2; do
  for v in main $VARS; do
    if [ $v = main ]; then lib=$PWD/sentinel_amd/libsentinel_flow.so; else lib=$PWD/sentinel_amd/variants/$v.so; fi
    SENTINEL_FLOW_LIB=$lib timeout -k 10 300 python3 bench.py $A > gpurun_out/vsvar/$v.b$k.json 2> gpurun_out/vsvar/$v.b$k.err || { echo BENCH_FAILED $v; tail -5 gpurun_out/vsvar/$v.b$k.err; exit 1; }
    python3 -c "import json; a=json.load(open('gpurun_out/vsvar/$v.b$k.json')); print('$v', a['ms_per_step'], a['roofline']['kernels_ms'])"
  done
done
