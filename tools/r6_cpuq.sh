# Round 6 (GPU box): does the headline hit the box's CPU quota?  GPU suite
# (optional), then headline runs printing ms/step and the timed region's
# process CPUs / cgroup throttling.   bash tools/r6_cpuq.sh TAG [tests] [extra bench args]
set -e
mkdir -p gpurun_out
T=${1:-q}
cat /proc/self/cgroup; cat /sys/fs/cgroup$(sed -n 's/^0:://p' /proc/self/cgroup)/cpu.max 2>/dev/null || true
if [ "$2" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/${T}_gputests.log 2>&1 || { tail -40 gpurun_out/${T}_gputests.log; exit 1; }
  tail -1 gpurun_out/${T}_gputests.log
fi
shift 2 || true
for k in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --no-decode-ab "$@" > gpurun_out/${T}_$k.json 2> gpurun_out/${T}_$k.err
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$k.json')); h=d['host']
print('$k', d['ms_per_step'], 'ms dev', d['device']['device_ms_per_step'], h['phase_ms_per_step']['step'], h['engine_ms_per_step'], h['timed_region_cpu'])"
done
