# Round 6 (GPU box): optional GPU test subset, the k_ge phase clocks (timing
# build libsiamese_amd_geclk.so), the headline host / device elimination A/B
# and a kernel-stats capture of the device-elimination headline.
#   bash tools/r6_ab.sh TAG [pytest -k expression]
set -e
mkdir -p gpurun_out
T=${1:-ab}
if [ -n "$2" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$2" \
      > gpurun_out/${T}_gputests.log 2>&1 || { tail -40 gpurun_out/${T}_gputests.log; exit 1; }
  tail -2 gpurun_out/${T}_gputests.log
fi
if [ -f siamese_amd/libsiamese_amd_geclk.so ]; then
  timeout -k 10 150 python bench.py --library siamese_amd/libsiamese_amd_geclk.so --steps 10 --warmup 2 --no-cpu --no-e2e --no-legs --device-ge > gpurun_out/${T}_geclk.json 2> gpurun_out/${T}_geclk.err
  grep "k_ge phases" gpurun_out/${T}_geclk.err || true
fi
for mode in plain dge plain dge; do
  extra="--no-device-ge"; [ $mode = dge ] && extra="--device-ge"
  timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs $extra > gpurun_out/${T}_$mode.json 2> gpurun_out/${T}_$mode.err
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$mode.json')); h=d['host']; v=d['device']
print('$mode', d['ms_per_step'], 'ms dev', v['device_ms_per_step'], 'rounds', v['rounds_per_step'], v['kernel_ms_per_step'], h['phase_ms_per_step']['step'], h['phase_ms_per_step']['flush'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-legs --device-ge > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -name '*kernel_stats.csv' -exec cut -c1-40,100-200 {} \;
