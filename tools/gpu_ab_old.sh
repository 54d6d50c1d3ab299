# GPU box: same-box A/B of the tree in abold/ (an older commit, built in place) against this tree.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
A="--steps 10 --warmup 3 --no-cpu --no-metric-log --no-degrade --no-legs"
for k in 1 2; do
  (cd abold && timeout -k 10 300 python3 bench.py $A) > gpurun_out/abold_$k.json 2> gpurun_out/abold_$k.err || { echo OLD_FAILED; tail -5 gpurun_out/abold_$k.err; exit 1; }
  timeout -k 10 300 python3 bench.py $A > gpurun_out/abnew_$k.json 2> gpurun_out/abnew_$k.err || { echo NEW_FAILED; tail -5 gpurun_out/abnew_$k.err; exit 1; }
  python3 -c "import json; a=json.load(open('gpurun_out/abold_$k.json')); b=json.load(open('gpurun_out/abnew_$k.json')); print('old', a['ms_per_step'], a['roofline']['kernels_ms']); print('new', b['ms_per_step'], b['roofline']['kernels_ms'])"
done
