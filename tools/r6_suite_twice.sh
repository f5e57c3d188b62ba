# Round 6 (GPU box): the GPU suite twice (no -x), summaries and failures.
#   bash tools/r6_suite_twice.sh TAG
mkdir -p gpurun_out
T=${1:-st}
for k in 1 2; do
  timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_$k.log 2>&1
  rc=$?
  grep -E "FAILED|passed|failed" gpurun_out/${T}_$k.log | tail -5
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
exit 0
