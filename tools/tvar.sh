# GPU box: tools/thread_bench.py (one heavy THREAD resource, oracle-checked) per library variant
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in ${VARS:-sentinel_flow}; do
SENTINEL_FLOW_LIB=$PWD/sentinel_amd/lib$v.so CHECK=${CHECK:-1} timeout -k 10 300 python -u tools/thread_bench.py $ARGS > gpurun_out/thread_$v.txt 2>&1 || { echo FAIL $v; tail -3 gpurun_out/thread_$v.txt; exit 1; }
echo "== $v"; grep -v "^SF_STREAM_PROF" gpurun_out/thread_$v.txt | tail -8
done
