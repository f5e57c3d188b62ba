# GPU box: parity suite, then the C2/C3/C5 legs and a short bench line
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
for r in 1 2; do timeout -k 10 120 python tools/leg_run.py C2 3 1; done
timeout -k 10 120 python tools/leg_run.py C3 1 1
timeout -k 10 120 python tools/leg_run.py C5 1 1
timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-legs > gpurun_out/bench_lc.log 2>&1
python tools/bench_summary.py bench gpurun_out/bench_lc.log
