# Round 6 (GPU box): headline by assembly-pool threads (SIAMESE_AMD_ASM_THREADS), interleaved.
#   bash tools/r6_asm_ab.sh TAG
set -e
mkdir -p gpurun_out
T=${1:-asm}
for k in 1 2; do for a in 4 2 3; do
  SIAMESE_AMD_ASM_THREADS=$a timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --no-decode-ab > gpurun_out/${T}_${a}_$k.json 2> gpurun_out/${T}_${a}_$k.err
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_${a}_$k.json')); h=d['host']
print('asm $a', d['ms_per_step'], h['timed_region_cpu']['process_cpus'], h['timed_region_cpu']['cpu_ms_per_step_by_thread'])"
done; done
