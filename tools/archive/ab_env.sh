# A/B environment settings of the default bench on the GPU box, interleaved:
#   bash tools/ab_env.sh ROUNDS "VAR=a" "VAR=b" ...
set -e
mkdir -p gpurun_out
R=$1; shift
for r in $(seq 1 $R); do
    i=0
    for a in "$@"; do
        env $a timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-legs > gpurun_out/env_${r}_$i.log 2>&1
        python tools/bench_summary.py "[$a]" gpurun_out/env_${r}_$i.log
        i=$((i+1))
    done
done
