# Round 6 (GPU box): headline plain and with the device elimination, then a
# kernel-stats capture of the device-elimination headline.  Usage: bash tools/r6_base.sh TAG
set -e
mkdir -p gpurun_out
T=${1:-b}
for mode in plain dge plain dge; do
  extra=""; [ $mode = dge ] && extra="--device-ge"
  timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs $extra > gpurun_out/${T}_$mode.json 2> gpurun_out/${T}_$mode.err
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$mode.json')); h=d['host']
print('$mode', d['ms_per_step'], 'ms', 'dev', d['device']['device_ms_per_step'], d['config'].get('decode'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-legs --device-ge > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -name '*kernel_stats.csv' -exec cat {} \;
