# Round 5 host probe (GPU box): the bench headline with per-call timing, and
# the host control plane alone (null backend) at 1 and 16 stepping threads.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs > gpurun_out/p_head.json 2> gpurun_out/p_head.err
SCENARIO_BATCH_CALLS=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-legs > gpurun_out/p_calls.json 2> gpurun_out/p_calls.err
for t in 1 4 16; do
  SCENARIO_BATCH_CALLS=1 timeout -k 10 200 python bench.py --library tools/libsiamese_null.so --steps 6 --warmup 1 --no-cpu --no-e2e --no-legs --no-verify --threads $t > gpurun_out/p_null_$t.json 2> gpurun_out/p_null_$t.err
done
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
