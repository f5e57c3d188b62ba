# Sampling profile of the host threads during bench.py (GPU box): writes
# gpurun_out/hprof.<pid> and the summaries hprof_report.txt / hprof_sgpu.txt.
set -e
mkdir -p gpurun_out
rm -f gpurun_out/hprof.*
timeout -k 10 200 python tools/host_profile.py gpurun_out/hprof --steps 30 --warmup 2 --no-cpu --no-e2e --no-legs "$@" > gpurun_out/hprof_bench.log 2>&1
f=$(ls gpurun_out/hprof.* | head -n1)
python tools/sampler_report.py $f --top 70 > gpurun_out/hprof_report.txt 2>&1
python tools/sampler_report.py $f --top 70 --filter sgpu > gpurun_out/hprof_sgpu.txt 2>&1 || true
