# whole GPU suite, then the default bench's config3_origin leg with parity (both variants)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/t_all.log 2>&1 &&
timeout -k 10 900 python3 -u bench.py --no-metric-log --no-degrade --legs config3_origin > gpurun_out/b_of.json 2> gpurun_out/b_of.err
