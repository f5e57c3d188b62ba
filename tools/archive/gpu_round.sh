# GPU box: parity + smoke + bench (tools/gpu_check.sh), then the end-to-end
# phase probe; every step time-boxed, the chain stops at the first failure.
set -e
bash tools/gpu_check.sh "$@"
timeout -k 10 300 python tools/e2e_probe.py 10 > gpurun_out/e2e_probe.log 2>&1 || { tail -20 gpurun_out/e2e_probe.log; exit 1; }
cat gpurun_out/e2e_probe.log
