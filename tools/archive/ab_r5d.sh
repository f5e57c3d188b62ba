# Round 5 A/B (GPU box): SMT siblings in the placement, headline and e2e.
set -e
mkdir -p gpurun_out
run() {
  local label=$1; shift
  env "$@" timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-cpu --no-legs $EXTRA > gpurun_out/ab5d.json 2> gpurun_out/ab5d.err
  python3 -c "
import json
d=json.load(open('gpurun_out/ab5d.json')); h=d['host']
print('%-22s %6.3f ms  step %.3f flush %.3f asm %.3f compl %.3f dev %.3f e2e %.3f' % ('$label', d['ms_per_step'], h['phase_ms_per_step']['step'], h['phase_ms_per_step']['flush'], h['engine_ms_per_step']['assemble'], h['engine_ms_per_step']['complete'], d['device']['device_ms_per_step'], d['end_to_end']['ms_per_step']))"
}
for r in 1 2 3; do
  EXTRA= run default X=1
  EXTRA= run smt SIAMESE_AMD_SMT=1
  EXTRA= run smt_asm8 SIAMESE_AMD_SMT=1 SIAMESE_AMD_ASM_THREADS=8
done
