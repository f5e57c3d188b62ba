# Headline A/B on one box: alternates library builds.
#   bash tools/ab_headline.sh ROUNDS LIB...
set -e
N=$1; shift
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for L in "$@"; do
    timeout -k 10 300 python bench.py --no-legs --no-cpu --no-e2e --library $L > gpurun_out/ab_h.log 2>&1
    echo "$(basename $L) $(python tools/bench_summary.py bench gpurun_out/ab_h.log)"
  done
done
