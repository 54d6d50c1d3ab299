cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc
A="--steps 1 --warmup 0 --no-cpu"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_heavy_fill|k_decide_light" --output-format csv -d gpurun_out/pmc/f -o f -- python3 bench.py $A > gpurun_out/pmc/f.log 2>&1 || { echo F_FAILED; tail gpurun_out/pmc/f.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex "k_heavy_fill|k_decide_light" --output-format csv -d gpurun_out/pmc/w -o w -- python3 bench.py $A > gpurun_out/pmc/w.log 2>&1 || { echo W_FAILED; tail gpurun_out/pmc/w.log; exit 1; }
find gpurun_out/pmc -name "*.csv" | head
