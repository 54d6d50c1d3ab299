cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="--steps 2 --warmup 1 --no-cpu --no-metric-log --no-degrade --legs config3_origin --origin-variants no_origin_rules"
mkdir -p gpurun_out/pmcx
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "k_ox_index|k_ox_lfind|k_ox_lapply" --output-format csv -d gpurun_out/pmcx/p1 -o p1 -- python3 bench.py $A > gpurun_out/pmcx/p1.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_WAIT_ANY --kernel-include-regex "k_ox_index|k_ox_lfind|k_ox_lapply" --output-format csv -d gpurun_out/pmcx/p2 -o p2 -- python3 bench.py $A > gpurun_out/pmcx/p2.log 2>&1
echo rc=$?
