# GPU box: parity suite, then the headline with the batch laid out on the
# caller's thread (0) or on the launcher thread (1), interleaved
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
bash tools/ab_env.sh 3 SIAMESE_AMD_ASYNC_ASSEMBLY=0 SIAMESE_AMD_ASYNC_ASSEMBLY=1
