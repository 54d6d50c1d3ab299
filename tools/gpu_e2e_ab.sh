# e2e_pinned on one box: without the CPU baseline, then with it (its order in bench.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u bench.py --no-cpu --no-metric-log --no-degrade --legs e2e_pinned > gpurun_out/e2e_a.json 2> gpurun_out/e2e_a.err &&
timeout -k 10 500 python3 -u bench.py --no-metric-log --no-degrade --legs e2e_pinned > gpurun_out/e2e_b.json 2> gpurun_out/e2e_b.err
