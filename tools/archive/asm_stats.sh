# Flush assembly time by stage (SGPU_ASM_STATS) on the C2 leg and the headline.
#   bash tools/asm_stats.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SGPU_ASM_STATS=1 timeout -k 10 120 python3 tools/leg_run.py C2 3 2 4 > gpurun_out/asm_c2_$TAG.txt 2>&1
SGPU_ASM_STATS=1 timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-legs > gpurun_out/asm_head_$TAG.txt 2>&1
tail -n 14 gpurun_out/asm_c2_$TAG.txt; tail -n 12 gpurun_out/asm_head_$TAG.txt | cut -c1-200
