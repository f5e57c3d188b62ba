# Round 5 (GPU box): the headline N times (plain), then once with per-call
# TSC timers and fork-join efficiency.  Usage: bash tools/r5_head.sh N TAG
set -e
mkdir -p gpurun_out
N=${1:-3}; T=${2:-h}
for i in $(seq 1 $N); do
  timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs > gpurun_out/${T}_$i.json 2> gpurun_out/${T}_$i.err
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$i.json')); h=d['host']
print('run $i', d['ms_per_step'], 'ms', h['phase_ms_per_step'], h['engine_ms_per_step'], 'dev', d['device']['device_ms_per_step'])"
done
SCENARIO_BATCH_CALLS=1 timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs > gpurun_out/${T}_calls.json 2> gpurun_out/${T}_calls.err
grep "^batch" gpurun_out/${T}_calls.err | tail -11
