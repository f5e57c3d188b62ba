# k_solve_main timing of instrumented variants (SGPU_SOLVE_AB builds; their
# bytes are wrong, so the bench runs without verification).
#   bash tools/solve_ab.sh TAG VARIANT...
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/solve_ab_$TAG.txt
: > $OUT
for v in base "$@"; do
  lib=siamese_amd/libsiamese_amd.so
  [ "$v" = base ] || lib=siamese_amd/libsiamese_amd_$v.so
  D=gpurun_out/sab_${TAG}_$v
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o t -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-legs --no-verify --library $lib > $D.log 2>&1
  echo "== $v" >> $OUT
  grep -h "k_solve\|k_exec" $D/*kernel_stats.csv | cut -d, -f1-4 | sed 's/(.*)"/"/' >> $OUT
done
cat $OUT
