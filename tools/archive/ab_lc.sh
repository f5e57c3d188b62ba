# GPU box: C2 and C3 legs with and without OP_LINCOMBS batching, interleaved
set -e
for r in 1 2; do
  for v in 0 1; do
    echo "[SIAMESE_AMD_LC_BATCH=$v]"
    SIAMESE_AMD_LC_BATCH=$v timeout -k 10 120 python tools/leg_run.py C2 3 1
    SIAMESE_AMD_LC_BATCH=$v timeout -k 10 120 python tools/leg_run.py C3 1 1
  done
done
