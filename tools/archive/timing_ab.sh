# Per-launch timing events on/off (GPU box), single-stream legs.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/timing_ab.log
cd $GRAFT_REPO_ROOT
: > $OUT
for T in 1 0 1 0; do
  echo "SGPU_TIMING=$T" >> $OUT
  SGPU_TIMING=$T timeout -k 10 120 python3 tools/leg_run.py C3 3 1 8 >> $OUT 2>&1
  SGPU_TIMING=$T timeout -k 10 120 python3 tools/leg_run.py C5 2 1 8 >> $OUT 2>&1
done
timeout -k 10 120 python3 tools/phase_leg.py siamese_amd/libsiamese_amd_phase.so C3 1 8 >> $OUT 2>&1
cat $OUT
