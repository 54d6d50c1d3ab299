# GPU box: rehearse bench.py's N=2 path on a one-GPU box: two ranks (gloo
# rendezvous on 127.0.0.1) both on device 0, each with its own resource shard
# and batch.  The RCCL ENTRY_NODE join cannot run with two ranks on one device,
# so its leg reports an error; everything else is the driver's N>1 code path.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 WORLD_SIZE=2 LOCAL_RANK=0
RANK=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps ${STEPS:-5} --warmup ${WARMUP:-2} > gpurun_out/n2_rank1.json 2> gpurun_out/n2_rank1.err &
P1=$!
RANK=0 timeout -k 10 400 python3 bench.py --gpus 2 --steps ${STEPS:-5} --warmup ${WARMUP:-2} > gpurun_out/n2_rank0.json 2> gpurun_out/n2_rank0.err
R0=$?
wait $P1
R1=$?
echo "rank0 rc=$R0 rank1 rc=$R1"
cat gpurun_out/n2_rank0.json
[ $R0 -eq 0 ] && [ $R1 -eq 0 ]
