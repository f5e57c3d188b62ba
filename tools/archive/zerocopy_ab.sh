set -e
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for z in 32768 0; do
    echo "[ZEROCOPY_UP=$z] $(SIAMESE_AMD_ZEROCOPY_UP=$z timeout -k 10 200 python tools/leg_run.py C3 3 1 8 2>&1 | tail -1)"
    echo "[ZEROCOPY_UP=$z] $(SIAMESE_AMD_ZEROCOPY_UP=$z timeout -k 10 200 python tools/leg_run.py C5 1 1 8 2>&1 | tail -1)"
  done
done
bash tools/dropin_ab.sh 2 SIAMESE_AMD_ZEROCOPY_UP=32768 SIAMESE_AMD_ZEROCOPY_UP=0
