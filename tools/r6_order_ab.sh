# Round 6 (GPU box): the headline inside the full default bench with the
# reference's first 16-thread run after the timed steps (default) or before
# them (--cpu-first), twice each, interleaved.  bash tools/r6_order_ab.sh TAG
set -e
mkdir -p gpurun_out
T=${1:-ord}
for k in 1 2; do for o in new old; do
  extra=""; [ $o = old ] && extra="--cpu-first"
  timeout -k 10 400 python bench.py --no-legs --no-e2e $extra > gpurun_out/${T}_${o}_$k.json 2> gpurun_out/${T}_${o}_$k.err
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_${o}_$k.json')); h=d['host']
print('$o', d['ms_per_step'], 'ab', d['decode_ab']['sgpu_decode_ms_per_step'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['ratio'], h['timed_region_cpu']['process_cpus'], h['timed_region_cpu']['cpu_ms_per_step_by_thread']['sgpu-step'], d['roofline']['frac'], d['roofline']['traffic_build_matches'])"
done; done
