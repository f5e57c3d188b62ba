# Round 6 (GPU box): headline over library builds, interleaved, 3 rounds
# (GPU suite first unless skip-tests).  bash tools/r6_lib_ab.sh TAG [skip-tests] LIB...
set -e
mkdir -p gpurun_out
T=$1; shift
MODE=$1; shift
if [ "$MODE" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/${T}_gputests.log 2>&1 || { tail -40 gpurun_out/${T}_gputests.log; exit 1; }
  tail -1 gpurun_out/${T}_gputests.log
fi
for rep in 1 2 3; do
  for L in "$@"; do
    timeout -k 10 150 python bench.py --library siamese_amd/$L --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --no-decode-ab > gpurun_out/${T}_${L}_$rep.json 2> gpurun_out/${T}_${L}_$rep.err
    python3 -c "
import json; d=json.load(open('gpurun_out/${T}_${L}_$rep.json')); h=d['host']; v=d['device']
print('$L', d['ms_per_step'], 'ms dev', v['device_ms_per_step'], h['phase_ms_per_step']['step'], h['engine_ms_per_step'], h['timed_region_cpu']['process_cpus'], h['timed_region_cpu'].get('cpu_ms_per_step_by_thread'))"
  done
done
