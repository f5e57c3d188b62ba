# Short defer sweep (GPU box): C3, C5, C2 legs at a few settings.
set -e
TAG=${1:-cur}
OUT=$GRAFT_REPO_ROOT/gpurun_out/defer_$TAG.log
cd $GRAFT_REPO_ROOT
: > $OUT
for D in 0 8 16 32; do timeout -k 10 120 python3 tools/leg_run.py C3 3 1 $D >> $OUT 2>&1; done
for D in 0 8 16; do timeout -k 10 120 python3 tools/leg_run.py C5 1 1 $D >> $OUT 2>&1; done
for D in 0 4 8; do timeout -k 10 120 python3 tools/leg_run.py C2 3 2 $D >> $OUT 2>&1; done
cat $OUT
