# Kernel trace + per-flush phase breakdown of one leg run (GPU box).
#   bash tools/leg_trace.sh TAG LEG [groups] [defer] -> gpurun_out/lt_TAG/
set -e
TAG=$1; LEG=$2; G=${3:-1}; DEF=${4:-0}
D=$GRAFT_REPO_ROOT/gpurun_out/lt_$TAG
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SGPU_UPLOAD_STATS=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o trace -- python3 tools/leg_run.py $LEG 1 $G $DEF > $D/leg.log 2> $D/leg.err
gzip -f $D/leg.err
find $D -name "*kernel_stats.csv" -exec cat {} \;
cat $D/leg.log
