# wave-walk iteration: its parity tests, then the origin leg timing (profile variant + product library)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_xwave.py tests/test_gpu_origin.py tests/test_xflow.py > gpurun_out/t_xw.log 2>&1 &&
XW_VARIANTS="${XW_VARIANTS:-newprof main}" bash tools/gpu_origin_ab.sh
