# wave-walk change: its parity tests, then the origin leg (both variants) and config 3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_xwave.py tests/test_gpu_origin.py tests/test_gpu_preblocked.py tests/test_xflow.py > gpurun_out/t_xw.log 2>&1 &&
timeout -k 10 1000 python3 -u bench.py --no-metric-log --no-degrade --legs config3_origin > gpurun_out/b_xw.json 2> gpurun_out/b_xw.err
