# Round 6 (GPU box): fork-join blocks homed by stream (SCENARIO_HOMED=1,
# default) vs dealt to any free thread (=0): GPU suite, then interleaved
# headline runs.   bash tools/r6_homed_ab.sh TAG [skip-tests]
set -e
mkdir -p gpurun_out
T=${1:-hm}
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/${T}_gputests.log 2>&1 || { tail -40 gpurun_out/${T}_gputests.log; exit 1; }
  tail -1 gpurun_out/${T}_gputests.log
fi
for k in 1 2 3; do for m in 0 1; do
  SCENARIO_HOMED=$m timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --no-decode-ab > gpurun_out/${T}_${m}_$k.json 2> gpurun_out/${T}_${m}_$k.err
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_${m}_$k.json')); h=d['host']
print('homed $m', d['ms_per_step'], 'ms dev', d['device']['device_ms_per_step'], h['phase_ms_per_step']['step'], h['timed_region_cpu']['process_cpus'], h['timed_region_cpu']['cpu_ms_per_step_by_thread'])"
done; done
