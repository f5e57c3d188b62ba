# Main-thread phase timeline of one C2 run (SCENARIO_TIMELINE=1), real device
# and null backend.  bash tools/c2_timeline.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SCENARIO_TIMELINE=1 timeout -k 10 120 python3 tools/leg_run.py C2 2 2 4 > gpurun_out/c2tl_gpu_$TAG.txt 2>&1
SCENARIO_TIMELINE=1 timeout -k 10 120 python3 tools/leg_null.py C2 2 2 4 > gpurun_out/c2tl_null_$TAG.txt 2>&1
tail -n 2 gpurun_out/c2tl_gpu_$TAG.txt gpurun_out/c2tl_null_$TAG.txt
