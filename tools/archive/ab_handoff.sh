# GPU box: launcher/wait hand-off spin off (0) vs on (100 us): C3 leg and the headline, interleaved
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
for r in 1 2; do
  for v in 0 100; do
    echo "[SIAMESE_AMD_HANDOFF_SPIN_US=$v]"
    SIAMESE_AMD_HANDOFF_SPIN_US=$v timeout -k 10 120 python tools/leg_run.py C3 1 1
    SIAMESE_AMD_HANDOFF_SPIN_US=$v timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-legs > gpurun_out/ho_${r}_$v.log 2>&1
    python tools/bench_summary.py bench gpurun_out/ho_${r}_$v.log
  done
done
