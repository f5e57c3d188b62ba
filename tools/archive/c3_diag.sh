# Single-stream latency diagnosis (GPU box): one C3 leg run under a kernel +
# memory-copy + HIP runtime trace, with the engine's per-flush timeline and
# upload/phase breakdown on stderr.
#   bash tools/c3_diag.sh TAG [LEG] -> gpurun_out/c3_TAG/
set -e
TAG=${1:-cur}
LEG=${2:-C3}
D=$GRAFT_REPO_ROOT/gpurun_out/c3_$TAG
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 tools/leg_run.py $LEG 2 1 > $D/plain.log 2>&1
SGPU_TIMELINE=1 SGPU_UPLOAD_STATS=1 SCENARIO_TIMELINE=1 timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $D -o trace -- python3 tools/leg_run.py $LEG 1 1 > $D/leg.log 2> $D/leg.err
gzip -f $D/leg.err
ls -R $D | head -30
cat $D/plain.log
