# SQ/TCC/LDS counter passes over one bench step (GPU box), one rocprofv3 run per pass.
#   bash tools/pmc_exec.sh  -> gpurun_out/pmc/{sq,tcc,lds}_counter_collection.csv
set -e
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="bench.py --steps 1 --warmup 1 --no-cpu --no-e2e --no-legs --no-decode-ab"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d gpurun_out/pmc -o sq -- python3 $B > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc -o tcc -- python3 $B > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH --kernel-trace --output-format csv -d gpurun_out/pmc -o lds -- python3 $B > /dev/null 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc/sq_counter_collection.csv gpurun_out/pmc/tcc_counter_collection.csv gpurun_out/pmc/lds_counter_collection.csv
