# Round 6 (GPU box): host sampling profile of the headline (merged rounds),
# then headline ms/step by stream groups, interleaved.  bash tools/r6_prof_groups.sh TAG
set -e
mkdir -p gpurun_out
T=${1:-pg}
bash tools/host_profile.sh --no-decode-ab
cp gpurun_out/hprof_report.txt gpurun_out/${T}_hprof_report.txt
cp gpurun_out/hprof_sgpu.txt gpurun_out/${T}_hprof_sgpu.txt
for k in 1 2; do for g in 6 8 12; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --no-decode-ab --groups $g > gpurun_out/${T}_g${g}_$k.json 2> gpurun_out/${T}_g${g}_$k.err
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_g${g}_$k.json')); h=d['host']
print('groups $g', d['ms_per_step'], 'ms dev', d['device']['device_ms_per_step'], 'rounds', d['device']['rounds_per_step'], h['phase_ms_per_step']['step'], h['engine_ms_per_step'], h['timed_region_cpu']['process_cpus'])"
done; done
