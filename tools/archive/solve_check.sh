# GPU box: parity suite, then the headline bench (no legs) and its kernel
# trace.  bash tools/solve_check.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gt_$TAG.log 2>&1 || { tail -30 gpurun_out/gt_$TAG.log; exit 1; }
tail -2 gpurun_out/gt_$TAG.log
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-legs > gpurun_out/bench_$TAG.json 2>/dev/null
python3 tools/bench_summary.py $TAG gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=gpurun_out/prof_$TAG
mkdir -p $D
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-legs > $D/bench_trace.log 2>&1
cat $(ls $D/*kernel_stats.csv | head -n1) | cut -d, -f1-4 | sed 's/(.*)"/"/'
