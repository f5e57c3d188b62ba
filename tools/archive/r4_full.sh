# Round-4 evidence on the GPU box: parity suite + smoke, the default bench
# line (legs, e2e, CPU baselines), kernel stats and PMC traffic of the
# headline, leg traces, and FETCH/WRITE of the C5 leg per kernel.
#   bash tools/r4_full.sh TAG [skip-tests]
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/gt_$TAG.log 2>&1 || { tail -30 gpurun_out/gt_$TAG.log; exit 1; }
  tail -n 2 gpurun_out/gt_$TAG.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  cat gpurun_out/smoke_$TAG.log
fi
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
python3 tools/bench_summary.py $TAG gpurun_out/bench_$TAG.json
bash tools/profile_round.sh $TAG > gpurun_out/prof_$TAG.log 2>&1
tail -n 3 gpurun_out/prof_$TAG.log
# C5 leg: DRAM bytes per kernel (separate counter passes)
D=gpurun_out/prof_$TAG
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D -o c5_fetch -- python3 tools/leg_run.py C5 1 1 8 > /dev/null 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D -o c5_write -- python3 tools/leg_run.py C5 1 1 8 > /dev/null 2>&1
python3 tools/pmc_traffic.py $(ls $D/c5_fetch*counter_collection.csv | head -n1) $(ls $D/c5_write*counter_collection.csv | head -n1) \
    $D/c5_traffic.json "rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per launch, C5 leg (tools/leg_run.py C5 1 1 8), round 4 tag $TAG"
