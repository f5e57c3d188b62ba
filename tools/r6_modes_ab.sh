# Round 6 (GPU box): headline modes interleaved: host elimination, device
# elimination (in-line), device elimination on the side stream (variant build).
set -e
mkdir -p gpurun_out
for rep in 1 2 3; do
  for mode in plain dge side; do
    lib=siamese_amd/libsiamese_amd.so; extra="--device-ge"
    [ $mode = plain ] && extra="--no-device-ge"
    [ $mode = side ] && lib=siamese_amd/libsiamese_amd_side.so
    timeout -k 10 150 python bench.py --library $lib --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs $extra > gpurun_out/modes_$mode.json 2> gpurun_out/modes_$mode.err
    python3 -c "
import json; d=json.load(open('gpurun_out/modes_$mode.json')); h=d['host']; v=d['device']
print('$mode', d['ms_per_step'], 'ms dev', v['device_ms_per_step'], 'step', h['phase_ms_per_step']['step'], 'flush', h['phase_ms_per_step']['flush'])"
  done
done
