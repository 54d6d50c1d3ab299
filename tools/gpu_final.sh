# round-end measurements: the default bench (every leg, CPU baseline, parity), then the
# rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the config-3 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python3 -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || exit 1
NAME=r04final PMC=1 BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-legs --no-degrade --no-metric-log" bash tools/gpu_profile.sh > gpurun_out/r04final.log 2>&1
