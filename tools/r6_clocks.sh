# Round 6 (GPU box): the device-elimination headline with the decoder's phase
# clocks (SIAMESE_AMD_DECODE_CLOCKS) and the per-call host timers.
set -e
mkdir -p gpurun_out
T=${1:-clk}
SIAMESE_AMD_DECODE_CLOCKS=1 SCENARIO_BATCH_CALLS=1 timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --no-decode-ab > gpurun_out/${T}.json 2> gpurun_out/${T}.err
grep -v "^batch" gpurun_out/${T}.err | tail -8
grep "^batch" gpurun_out/${T}.err | tail -10
