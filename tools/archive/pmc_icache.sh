# Instruction-fetch counters of one headline step (k_exec i-cache behaviour):
#   bash tools/pmc_icache.sh TAG [library]
set -e
TAG=$1; LIB=${2:-siamese_amd/libsiamese_amd.so}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=gpurun_out/pmc_$TAG
mkdir -p $D
B="bench.py --library $LIB --steps 1 --warmup 1 --no-cpu --no-e2e --no-legs --no-verify"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU --kernel-trace --output-format csv -d $D -o sq -- python3 $B > $D/sq.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ --kernel-trace --output-format csv -d $D -o ic -- python3 $B > $D/ic.log 2>&1
python3 tools/pmc_summary.py $D/sq_counter_collection.csv $D/ic_counter_collection.csv | grep -A 14 "k_exec"
