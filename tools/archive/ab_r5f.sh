# Round 5 A/B (GPU box): host LDPC pick draws by AVX-512 vs cached offsets
# (decode_region phase clocks), headline.
set -e
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1; do
    SIAMESE_AMD_VECTOR_PICKS=$v SIAMESE_AMD_DECODE_CLOCKS=1 timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-cpu --no-e2e --no-legs > gpurun_out/ab5f.json 2> gpurun_out/ab5f.err
    python3 -c "
import json
d=json.load(open('gpurun_out/ab5f.json'))
print('vpicks=$v', d['ms_per_step'])"
    grep "medians" gpurun_out/ab5f.err
  done
done
