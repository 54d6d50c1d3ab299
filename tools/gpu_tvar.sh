# GPU box: tools/thread_bench.py per library variant (sentinel_amd/variants/<v>.so; "main" = the product library)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in main ${VARS}; do
  if [ $v = main ]; then lib=$PWD/sentinel_amd/libsentinel_flow.so; else lib=$PWD/sentinel_amd/variants/$v.so; fi
  SENTINEL_FLOW_LIB=$lib CHECK=${CHECK:-1} timeout -k 10 300 python -u tools/thread_bench.py $ARGS > gpurun_out/thread_$v.txt 2>&1 || { echo FAIL $v; tail -3 gpurun_out/thread_$v.txt; exit 1; }
  echo "== $v"; grep -v "^SF_STREAM_PROF" gpurun_out/thread_$v.txt | tail -8
done
