export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --latency-runs 1"
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_r01
timeout -s KILL 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o p1 -- $B > gpurun_out/pmc_p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR GRBM_COUNT --output-format csv -d $O/p2 -o p2 -- $B > gpurun_out/pmc_p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o p3 -- $B > gpurun_out/pmc_p3.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p4 -o p4 -- $B > gpurun_out/pmc_p4.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p5 -o p5 -- $B > gpurun_out/pmc_p5.log 2>&1
ls -R gpurun_out/pmc_r01 | head -30
