set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
bash tools/ab_env.sh 2 SIAMESE_AMD_POOL_SPIN=0 SIAMESE_AMD_POOL_SPIN=4096
timeout -k 10 300 python tools/e2e_probe.py 10 > gpurun_out/e2e_probe.log 2>&1 || { tail -20 gpurun_out/e2e_probe.log; exit 1; }
cat gpurun_out/e2e_probe.log
