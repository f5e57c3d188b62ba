# GPU box: parity suite + smoke, then the single-stream legs (no per-launch
# events) and OP_ROWS phase clocks.  bash tools/r3_check.sh TAG
set -e
TAG=${1:-cur}
OUT=$GRAFT_REPO_ROOT/gpurun_out/check_$TAG.log
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gputests_$TAG.log 2>&1 || { tail -40 gpurun_out/gputests_$TAG.log; exit 1; }
tail -2 gpurun_out/gputests_$TAG.log
: > $OUT
timeout -k 10 120 python3 tools/leg_run.py C3 5 1 8 >> $OUT 2>&1
timeout -k 10 120 python3 tools/leg_run.py C3 3 1 16 >> $OUT 2>&1
timeout -k 10 200 python3 tools/leg_run.py C5 3 1 8 >> $OUT 2>&1
timeout -k 10 200 python3 tools/leg_run.py C2 5 2 4 >> $OUT 2>&1
timeout -k 10 120 python3 tools/phase_leg.py siamese_amd/libsiamese_amd_phase.so C3 1 8 >> $OUT 2>&1
cat $OUT
