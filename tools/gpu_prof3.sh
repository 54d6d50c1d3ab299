# GPU box: kernel traces for round 3 — config3 serialized timeline, config2 leg, config4 leg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export SF_SERIAL_STREAMS=1
NAME=ktl_c3 BENCH_ARGS="--steps 2 --warmup 1 --no-cpu --no-metric-log --no-degrade --no-legs" bash tools/gpu_ktl.sh > gpurun_out/ktl_c3.txt 2>&1 || { echo C3_FAILED; tail gpurun_out/ktl_c3.txt; exit 1; }
unset SF_SERIAL_STREAMS
NAME=ktl_c2 LEG=config2 LEG_ARGS="steps=2" bash tools/gpu_ktl_leg.sh > gpurun_out/ktl_c2.txt 2>&1 || { echo C2_FAILED; tail gpurun_out/ktl_c2.txt; exit 1; }
NAME=ktl_c4 LEG=config4 LEG_ARGS="reps=2" bash tools/gpu_ktl_leg.sh > gpurun_out/ktl_c4.txt 2>&1 || { echo C4_FAILED; tail gpurun_out/ktl_c4.txt; exit 1; }
head -70 gpurun_out/ktl_c3.txt; echo; head -45 gpurun_out/ktl_c2.txt; echo; head -45 gpurun_out/ktl_c4.txt
