# Round 6 (GPU box): the device-elimination headline over stream-group counts,
# interleaved.  bash tools/r6_groups_ab.sh TAG G...
set -e
mkdir -p gpurun_out
T=$1; shift
for rep in 1 2; do
  for G in "$@"; do
    timeout -k 10 150 python bench.py --groups $G --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --no-decode-ab > gpurun_out/${T}_g${G}_$rep.json 2> gpurun_out/${T}_g${G}_$rep.err
    python3 -c "
import json; d=json.load(open('gpurun_out/${T}_g${G}_$rep.json')); h=d['host']; v=d['device']
print('groups $G', d['ms_per_step'], 'ms dev', v['device_ms_per_step'], 'rounds', v['rounds_per_step'], h['phase_ms_per_step']['step'], h['phase_ms_per_step']['flush'])"
  done
done
