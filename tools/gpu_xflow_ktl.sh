# GPU box: the xflow parity tests, then the serialized kernel timeline of the bench (tools/gpu_ktl.sh).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_xflow.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/xflow_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/xflow_tests.log; exit 1; }
tail -2 gpurun_out/xflow_tests.log
SF_SERIAL_STREAMS=1 NAME=ktl_serial bash tools/gpu_ktl.sh > gpurun_out/ktl_serial.txt 2>&1 || { echo KTL_FAILED; tail -20 gpurun_out/ktl_serial.txt; exit 1; }
tail -70 gpurun_out/ktl_serial.txt
