set -e
mkdir -p gpurun_out
timeout -k 10 200 python tools/host_profile.py gpurun_out/hprof --steps 30 --warmup 2 --no-cpu --no-e2e > gpurun_out/hprof_bench.log 2>&1
f=$(ls gpurun_out/hprof.* | head -n1)
python tools/sampler_report.py $f --top 60 > gpurun_out/hprof_report.txt 2>&1
python tools/sampler_report.py $f --top 40 --filter sgpu > gpurun_out/hprof_sgpu.txt 2>&1 || true
