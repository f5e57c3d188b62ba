# Deferred-output rounds (BatchOptions::defer) on the single-stream and
# Cauchy legs (GPU box): ms per run for each setting.
#   bash tools/defer_sweep.sh TAG -> gpurun_out/defer_TAG.log
set -e
TAG=${1:-cur}
OUT=$GRAFT_REPO_ROOT/gpurun_out/defer_$TAG.log
cd $GRAFT_REPO_ROOT
: > $OUT
for D in 0 1 2 4 8 16; do timeout -k 10 120 python3 tools/leg_run.py C3 3 1 $D >> $OUT 2>&1; done
for D in 0 1 4; do timeout -k 10 120 python3 tools/leg_run.py C2 3 2 $D >> $OUT 2>&1; done
for D in 0 2 8; do timeout -k 10 120 python3 tools/leg_run.py C5 1 1 $D >> $OUT 2>&1; done
for D in 0 1 4; do timeout -k 10 120 python3 tools/leg_run.py C4x1024 3 4 $D >> $OUT 2>&1; done
cat $OUT
