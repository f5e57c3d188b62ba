# Round 6 (GPU box): the headline over stream-group counts, device and host
# elimination, interleaved.  bash tools/r6_groups_ab2.sh TAG
set -e
mkdir -p gpurun_out
T=$1
for rep in 1 2; do
  for cfg in "8 dge" "12 dge" "16 dge" "4 dge" "4 plain" "8 plain"; do
    set -- $cfg
    extra="--device-ge"; [ $2 = plain ] && extra="--no-device-ge"
    timeout -k 10 150 python bench.py --groups $1 $extra --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --no-decode-ab > gpurun_out/${T}_g$1$2_$rep.json 2> gpurun_out/${T}_g$1$2_$rep.err
    python3 -c "
import json; d=json.load(open('gpurun_out/${T}_g$1$2_$rep.json')); h=d['host']; v=d['device']
print('groups $1 $2', d['ms_per_step'], 'ms dev', v['device_ms_per_step'], 'rounds', v['rounds_per_step'], h['phase_ms_per_step']['step'], h['phase_ms_per_step']['flush'], v['kernel_ms_per_step'])"
  done
done
