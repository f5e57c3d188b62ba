# Round-3 evidence on the GPU box: parity suite + smoke, the default bench
# line (legs, e2e, CPU baselines), kernel stats and PMC traffic of the
# headline, leg traces.   bash tools/r3_full.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gt_$TAG.log 2>&1 || { tail -30 gpurun_out/gt_$TAG.log; exit 1; }
tail -n 2 gpurun_out/gt_$TAG.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
cat gpurun_out/smoke_$TAG.log
timeout -k 10 420 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
python3 tools/bench_summary.py $TAG gpurun_out/bench_$TAG.json
bash tools/profile_round.sh $TAG > gpurun_out/prof_$TAG.log 2>&1
tail -n 3 gpurun_out/prof_$TAG.log
