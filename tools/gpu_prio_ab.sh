# GPU box: same-box A/B of the decide-phase stream priorities (SF_STREAM_PRIO 0 / 1), two rounds
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
A="--steps 10 --warmup 3 --no-cpu --no-metric-log --no-degrade --no-legs"
for k in 1 2; do
  for p in 0 1; do
    SF_STREAM_PRIO=$p timeout -k 10 300 python3 bench.py $A > gpurun_out/prio${p}_$k.json 2> gpurun_out/prio${p}_$k.err || { echo FAILED; tail -5 gpurun_out/prio${p}_$k.err; exit 1; }
    python3 -c "import json; a=json.load(open('gpurun_out/prio${p}_$k.json')); print('prio$p', a['ms_per_step'], a['roofline']['kernels_ms'])"
  done
done
