# GPU box: THREAD parity tests, then the head-segment timing and the per-segment heavy profile per library variant
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "thread or config3 or async or system or edge" > gpurun_out/t.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/t.log | tail -30; exit 1; }
tail -1 gpurun_out/t.log
for v in main ${VARS}; do
  if [ $v = main ]; then lib=$PWD/sentinel_amd/libsentinel_flow.so; else lib=$PWD/sentinel_amd/variants/$v.so; fi
  echo "== $v"
  SENTINEL_FLOW_LIB=$lib CHECK=0 timeout -k 10 120 python -u tools/thread_bench.py 2430000 242 2>&1 | tail -1
  SENTINEL_FLOW_LIB=$lib timeout -k 10 300 python3 tools/heavy_profile.py --top 3 > gpurun_out/hp_$v.txt 2>&1; head -10 gpurun_out/hp_$v.txt
done
