# GPU box: the config-4 leg (tools/leg_run.py config4) under environment variants
# (VARIANTS: specs NAME=VALUE[,NAME=VALUE], "-" for none), REPS rounds interleaved;
# the first run of the first round checks parity against the one-core oracle.
cd $GRAFT_REPO_ROOT
i=0
for r in $(seq ${REPS:-2}); do
  for spec in ${VARIANTS}; do
    i=$((i+1)); envs=""; [ "$spec" != "-" ] && envs=$(echo "$spec" | tr ',' ' ')
    par=0; [ $i -le ${PARITY_RUNS:-0} ] && par=1
    env $envs timeout -k 10 300 python3 tools/leg_run.py config4 parity=$par reps=3 > gpurun_out/c4ab_$i.json 2> gpurun_out/c4ab_$i.err || { echo LEG_FAILED $spec; tail -5 gpurun_out/c4ab_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c4ab_$i.json')); print('$spec', d['ms_per_batch'], d['reps_ms'], d['planner_rounds'], (d.get('parity') or {}).get('exact'))"
  done
done
