# Round 5 A/B (GPU box): pool niceness and thread settings of the headline,
# interleaved rounds.  Each line: label, ms/step, phases.
set -e
mkdir -p gpurun_out
run() {  # label env... -- args
  local label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs $EXTRA > gpurun_out/ab5a.json 2> gpurun_out/ab5a.err
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/ab5a.json'))
print('%-28s %6.3f ms  step %.3f create %.3f finish %.3f asm %.3f compl %.3f dev %.3f' % ('$label', d['ms_per_step'], d['host']['phase_ms_per_step']['step'], d['host']['phase_ms_per_step']['create'], d['host']['phase_ms_per_step']['finish'], d['host']['engine_ms_per_step']['assemble'], d['host']['engine_ms_per_step']['complete'], d['device']['device_ms_per_step']))"
}
for r in 1 2 3; do
  EXTRA= run default X=1
  EXTRA= run nice0 SIAMESE_AMD_WORKER_NICE=0
  EXTRA="--threads 16" run harness16 X=1
  EXTRA= run nice0_asm2 SIAMESE_AMD_WORKER_NICE=0 SIAMESE_AMD_ASM_THREADS=2
  EXTRA= run nice5 SIAMESE_AMD_WORKER_NICE=5
done
