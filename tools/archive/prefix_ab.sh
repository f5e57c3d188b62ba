# k_solve_prefix A/B (verified bench runs under the kernel trace), then the
# SQ/TCC/LDS counter passes of the current build.   bash tools/prefix_ab.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/prefix_ab_$TAG.txt
: > $OUT
for v in base pipe; do
  lib=siamese_amd/libsiamese_amd.so
  [ "$v" = base ] || lib=siamese_amd/libsiamese_amd_$v.so
  D=gpurun_out/pab_${TAG}_$v
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o t -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-legs --library $lib > $D.log 2>&1
  echo "== $v $(grep -o '"rank0_digest": [0-9]*' $D.log)" >> $OUT
  python3 tools/kstats.py $D >> $OUT
done
cat $OUT
[ -n "$2" ] || exit 0
bash tools/pmc_exec.sh > gpurun_out/pmc_$TAG.txt 2>&1
tail -n 30 gpurun_out/pmc_$TAG.txt
