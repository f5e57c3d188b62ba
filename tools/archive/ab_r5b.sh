# Round 5 A/B (GPU box): fork-join task size, assembly threads and pool
# niceness of the headline, interleaved rounds.
set -e
mkdir -p gpurun_out
run() {
  local label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu --no-e2e --no-legs > gpurun_out/ab5b.json 2> gpurun_out/ab5b.err
  python3 -c "
import json
d=json.load(open('gpurun_out/ab5b.json')); h=d['host']
print('%-22s %6.3f ms  step %.3f flush %.3f asm %.3f compl %.3f dev %.3f' % ('$label', d['ms_per_step'], h['phase_ms_per_step']['step'], h['phase_ms_per_step']['flush'], h['engine_ms_per_step']['assemble'], h['engine_ms_per_step']['complete'], d['device']['device_ms_per_step']))"
}
for r in 1 2 3; do
  run default X=1
  run block1 SCENARIO_BLOCK=1
  run asm2 SIAMESE_AMD_ASM_THREADS=2
  run nice0 SIAMESE_AMD_WORKER_NICE=0
  run block4 SCENARIO_BLOCK=4
done
