# k_ldpc item size / depth variants on the C5 and C3 legs, interleaved.
#   bash tools/ab_ldpc.sh TAG VARIANT...   (base = libsiamese_amd.so)
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/ab_ldpc_$TAG.txt
: > $OUT
for rep in 1 2; do
  for v in base "$@"; do
    lib=siamese_amd/libsiamese_amd.so
    [ "$v" = base ] || lib=siamese_amd/libsiamese_amd_$v.so
    echo -n "$v " >> $OUT
    SGPU_LIB=$lib timeout -k 10 150 python3 tools/leg_run.py C5 2 1 8 >> $OUT 2>&1
    echo -n "$v " >> $OUT
    SGPU_LIB=$lib timeout -k 10 100 python3 tools/leg_run.py C3 3 1 8 >> $OUT 2>&1
  done
done
cat $OUT
