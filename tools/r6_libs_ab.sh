# Round 6 (GPU box): the device-elimination headline over several library
# builds, interleaved, plus the k_ge clocks of each clock build.
#   bash tools/r6_libs_ab.sh TAG LIB... (names under siamese_amd/, e.g. libsiamese_amd.so)
set -e
mkdir -p gpurun_out
T=$1; shift
for rep in 1 2; do
  for L in "$@"; do
    timeout -k 10 150 python bench.py --library siamese_amd/$L --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --device-ge > gpurun_out/${T}_${L}_$rep.json 2> gpurun_out/${T}_${L}_$rep.err
    python3 -c "
import json; d=json.load(open('gpurun_out/${T}_${L}_$rep.json')); h=d['host']; v=d['device']
print('$L', d['ms_per_step'], 'ms dev', v['device_ms_per_step'], v['kernel_ms_per_step'], h['phase_ms_per_step']['step'], h['phase_ms_per_step']['flush'])"
    grep "k_ge" gpurun_out/${T}_${L}_$rep.err || true
  done
done
