# Interleaved headline A/B of the current library against variant libraries
# (siamese_amd/libsiamese_amd_NAME.so).   bash tools/ab_lib.sh TAG NAME...
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/ab_lib_$TAG.txt
: > $OUT
for rep in 1 2 3; do
  for v in base "$@"; do
    lib=siamese_amd/libsiamese_amd.so
    [ "$v" = base ] || lib=siamese_amd/libsiamese_amd_$v.so
    timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --library $lib > gpurun_out/ab.json 2>/dev/null
    python3 tools/bench_summary.py $v gpurun_out/ab.json >> $OUT
  done
done
cat $OUT
