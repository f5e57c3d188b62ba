# Round 6 (GPU box): HIP API call statistics of the headline (which calls
# the launcher/completer spend their CPU in).  bash tools/r6_hip_api.sh TAG
set -e
T=${1:-api}
D=$GRAFT_REPO_ROOT/gpurun_out/${T}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --hip-trace --stats --output-format csv -d $D -o api -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 1 --no-cpu --no-e2e --no-legs --no-decode-ab > $D/bench.log 2>&1
ls $D
f=$(ls $D/api_hip_api_stats.csv 2>/dev/null || find $D -name '*hip_api_stats.csv' | head -n1)
head -25 $f
