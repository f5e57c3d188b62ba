# Round 5 A/B (GPU box): stepping threads, assembly threads and stream groups
# of the headline, interleaved rounds.
set -e
mkdir -p gpurun_out
run() {
  local label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu --no-e2e --no-legs $EXTRA > gpurun_out/ab5c.json 2> gpurun_out/ab5c.err
  python3 -c "
import json
d=json.load(open('gpurun_out/ab5c.json')); h=d['host']
print('%-22s %6.3f ms  step %.3f flush %.3f asm %.3f compl %.3f dev %.3f' % ('$label', d['ms_per_step'], h['phase_ms_per_step']['step'], h['phase_ms_per_step']['flush'], h['engine_ms_per_step']['assemble'], h['engine_ms_per_step']['complete'], d['device']['device_ms_per_step']))"
}
for r in 1 2 3; do
  EXTRA= run default X=1
  EXTRA= run thr15 SIAMESE_AMD_THREADS=15
  EXTRA= run thr14_asm2 SIAMESE_AMD_THREADS=14 SIAMESE_AMD_ASM_THREADS=2
  EXTRA="--groups 2" run groups2 X=1
  EXTRA="--groups 8" run groups8 X=1
done
