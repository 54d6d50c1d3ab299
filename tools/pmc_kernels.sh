# GPU box: two rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE + 8 SQ counters) over a 1-batch bench,
# kernels matching RE; per-kernel table via tools/pmc_table.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && OUT=gpurun_out/${NAME:-pmc}; rm -rf $OUT; mkdir -p $OUT
A=${BENCH_ARGS:---steps 1 --warmup 0 --no-cpu --no-metric-log --no-degrade}
RE=${RE:-k_heavy_fill|k_decide_light|k_decide_short|k_keys_packed|k_unpack|k_heavy_stream}
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RE" --output-format csv -d $OUT/f -o f -- python3 bench.py $A > $OUT/f.log 2>&1 || { echo F_FAILED; tail $OUT/f.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "$RE" --output-format csv -d $OUT/w -o w -- python3 bench.py $A > $OUT/w.log 2>&1 || { echo W_FAILED; tail $OUT/w.log; exit 1; }
python3 tools/pmc_table.py $OUT
