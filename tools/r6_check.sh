# Round 6 (GPU box): parity suite, then the headline plain / device-elimination
# A/B, then a kernel-stats capture of the device-elimination headline.
#   bash tools/r6_check.sh TAG [skip-tests]
set -e
mkdir -p gpurun_out
T=${1:-c}
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/${T}_gputests.log 2>&1 || { tail -40 gpurun_out/${T}_gputests.log; exit 1; }
  tail -2 gpurun_out/${T}_gputests.log
fi
for mode in plain dge plain dge; do
  extra="--no-device-ge"; [ $mode = dge ] && extra="--device-ge"
  timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs $extra > gpurun_out/${T}_$mode.json 2> gpurun_out/${T}_$mode.err
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$mode.json')); h=d['host']
print('$mode', d['ms_per_step'], 'ms', 'dev', d['device']['device_ms_per_step'], h['phase_ms_per_step'], d['config'].get('decode'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-legs --device-ge > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -name '*kernel_stats.csv' -exec cat {} \;
