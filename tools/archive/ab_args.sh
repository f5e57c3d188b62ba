# A/B bench.py argument sets on the GPU box (default library):
#   bash tools/ab_args.sh "--groups 2" "--groups 3" ...
set -e
mkdir -p gpurun_out
i=0
for a in "$@"; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu --no-e2e $a > gpurun_out/args_$i.log 2>&1
    python tools/bench_summary.py "[$a]" gpurun_out/args_$i.log
    i=$((i+1))
done
