# whole GPU suite, then config 3 + the origin leg's `other` variant (no parity legs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/t_all.log 2>&1 &&
timeout -k 10 600 python3 -u bench.py --no-cpu --no-metric-log --no-degrade --legs config3_origin --origin-variants other_rules_1pct > gpurun_out/b_rc.json 2> gpurun_out/b_rc.err
