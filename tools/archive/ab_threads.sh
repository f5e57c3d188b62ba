# Headline with 14/15/16 pool threads (SIAMESE_AMD_THREADS), interleaved.
#   bash tools/ab_threads.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/ab_threads_$TAG.txt
: > $OUT
for rep in 1 2 3; do
  for t in 16 15 14; do
    SIAMESE_AMD_THREADS=$t timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs > gpurun_out/abt.json 2>/dev/null
    python3 tools/bench_summary.py "t$t" gpurun_out/abt.json >> $OUT
  done
done
cat $OUT
