# Solve kernel change: parity subset (solves of every size, incl. edge_maxloss's
# narrow path and the fused prefix), then headline kernel stats.
#   bash tools/solve_check2.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "batch_api_matches_reference or full_size_every_byte or dropin_api_matches_reference" > gpurun_out/gt_$TAG.log 2>&1 || { tail -30 gpurun_out/gt_$TAG.log; exit 1; }
tail -n 2 gpurun_out/gt_$TAG.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=gpurun_out/sc_$TAG
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o t -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-legs > $D.log 2>&1
grep -h "k_solve\|k_exec" $D/*kernel_stats.csv | cut -d, -f1-4 | sed 's/(.*)"/"/'
