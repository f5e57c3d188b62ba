# Round 6 (GPU box): a GPU test subset, the headline modes A/B, and a
# device-elimination kernel trace.   bash tools/r6_round.sh TAG "pytest -k expr"
set -e
mkdir -p gpurun_out
T=$1
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$2" \
      > gpurun_out/${T}_gputests.log 2>&1 || { tail -40 gpurun_out/${T}_gputests.log; exit 1; }
  tail -1 gpurun_out/${T}_gputests.log
fi
bash tools/r6_modes_ab.sh
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-legs --device-ge > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -name '*kernel_stats.csv' -exec cut -c1-30,100-170 {} \;
