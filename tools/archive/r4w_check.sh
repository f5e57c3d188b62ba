set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gt_r4w.log 2>&1 || { tail -30 gpurun_out/gt_r4w.log; exit 1; }
tail -n 2 gpurun_out/gt_r4w.log
bash tools/tr_check.sh r4w > gpurun_out/tr_r4w.out 2>&1
tail -12 gpurun_out/tr_r4w.out
