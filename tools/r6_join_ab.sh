# Round 6 (GPU box): where the codec stream joins the matrix jobs' side stream:
# before the decoders (default) or before the first k_exec (variant build).
set -e
mkdir -p gpurun_out
for rep in 1 2 3; do
  for L in libsiamese_amd.so libsiamese_amd_early.so; do
    timeout -k 10 150 python bench.py --library siamese_amd/$L --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --no-decode-ab > gpurun_out/join_$L.json 2> gpurun_out/join_$L.err
    python3 -c "
import json; d=json.load(open('gpurun_out/join_$L.json')); h=d['host']; v=d['device']; r=d['roofline']
print('$L', d['ms_per_step'], 'ms dev', v['device_ms_per_step'], 'exec/launch', r['exec_ms_per_launch'], 'k_ge', v['kernel_ms_per_step']['k_ge'], 'flush', h['phase_ms_per_step']['flush'])"
  done
done
