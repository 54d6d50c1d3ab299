# GPU box: SF_STREAM_PROF build on one THREAD case (ARGS="entries count"), per-wave cycle split
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
SENTINEL_FLOW_LIB=$PWD/sentinel_amd/libsentinel_flow_prof.so CHECK=0 timeout -k 10 200 python -u tools/thread_bench.py $ARGS > gpurun_out/thread_prof.txt 2>&1 || { tail -5 gpurun_out/thread_prof.txt; exit 1; }
grep -v "^SF_STREAM_PROF" gpurun_out/thread_prof.txt | tail -3; grep "^SF_STREAM_PROF" gpurun_out/thread_prof.txt | tail -8
