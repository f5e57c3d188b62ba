# GPU box: parity suite, smoke, then one default bench line (each step time-boxed,
# the chain stops at the first failure).  Logs under gpurun_out/.
#   bash tools/gpu_check.sh [extra bench args]
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python bench.py "$@" > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
python tools/bench_summary.py bench gpurun_out/bench.log
