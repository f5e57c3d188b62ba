# A/B-time library variants built by tools/build_variant.sh (GPU box):
#   bash tools/ab_variants.sh w4 w8 ...
# Each variant runs the default bench workload (warm-up verifies every
# recovered byte); a summary line per variant goes to stdout.
set -e
mkdir -p gpurun_out
for v in "$@"; do
    timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e \
        --library siamese_amd/libsiamese_amd_$v.so > gpurun_out/var_$v.log 2>&1
done
for v in "$@"; do
    python tools/bench_summary.py $v gpurun_out/var_$v.log
done
