# Round 5 probe 4 (GPU box): per-call TSC costs and fork-join efficiency, host
# control plane alone (null backend) at 1 and 16 threads, and the headline.
set -e
mkdir -p gpurun_out
for t in 1 16; do
  SCENARIO_BATCH_CALLS=1 timeout -k 10 200 python bench.py --library tools/libsiamese_null.so --steps 8 --warmup 1 --no-cpu --no-e2e --no-legs --no-verify --threads $t > gpurun_out/p4_null_$t.json 2> gpurun_out/p4_null_$t.err
done
SCENARIO_BATCH_CALLS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs > gpurun_out/p4_head.json 2> gpurun_out/p4_head.err
