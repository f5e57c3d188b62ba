# C2 leg timing (real and null backend) + C3/C5 legs: bash tools/c2_quick.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/c2quick_$TAG.txt
: > $OUT
timeout -k 10 120 python3 tools/leg_run.py C2 6 2 4 >> $OUT 2>&1
timeout -k 10 120 python3 tools/leg_null.py C2 4 2 4 >> $OUT 2>&1
timeout -k 10 120 python3 tools/leg_run.py C3 3 1 8 >> $OUT 2>&1
timeout -k 10 120 python3 tools/leg_run.py C5 2 1 8 >> $OUT 2>&1
SCENARIO_TIMELINE=1 timeout -k 10 120 python3 tools/leg_run.py C2 2 2 4 > gpurun_out/c2tl_gpu_$TAG.txt 2>&1
cat $OUT
