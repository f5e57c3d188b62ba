# Round 5 probe 2 (GPU box): pipeline timeline of the headline (harness and
# engine events), then a sampling profile of all host threads.
set -e
mkdir -p gpurun_out
SCENARIO_TIMELINE=1 SGPU_TIMELINE=1 timeout -k 10 200 python bench.py --steps 4 --warmup 2 --no-cpu --no-e2e --no-legs > gpurun_out/p2_tl.json 2> gpurun_out/p2_tl.err
SIAMESE_AMD_DECODE_CLOCKS=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-legs > gpurun_out/p2_dc.json 2> gpurun_out/p2_dc.err
rm -f gpurun_out/hprof.*
timeout -k 10 200 python tools/host_profile.py gpurun_out/hprof --steps 40 --warmup 2 --no-cpu --no-e2e --no-legs > gpurun_out/hprof_bench.log 2>&1
f=$(ls gpurun_out/hprof.* | head -n1)
python tools/sampler_report.py $f --top 90 > gpurun_out/hprof_report.txt 2>&1
