# Round 5 probe 3 (GPU box): host CPU topology, and the host control plane
# alone (null backend) at 1..16 stepping threads, then the headline.
set -e
mkdir -p gpurun_out
(lscpu; grep Cpus_allowed_list /proc/self/status; cat /sys/fs/cgroup/cpu.max) > gpurun_out/p3_cpu.txt 2>&1 || true
for t in 1 2 4 8 12 16; do
  timeout -k 10 200 python bench.py --library tools/libsiamese_null.so --steps 8 --warmup 1 --no-cpu --no-e2e --no-legs --no-verify --threads $t > gpurun_out/p3_null_$t.json 2> gpurun_out/p3_null_$t.err
done
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs > gpurun_out/p3_head.json 2> gpurun_out/p3_head.err
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --threads 16 > gpurun_out/p3_head16.json 2> gpurun_out/p3_head16.err
