# rocprofv3 kernel trace of the C2 leg (one run, one stream group) -> gpurun_out/c2_trace/
set -e
mkdir -p gpurun_out/c2_trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c2_trace -o c2 -- python3 tools/leg_run.py C2 2 1 > gpurun_out/c2_trace/run.log 2>&1
cat gpurun_out/c2_trace/run.log | tail -2
cat $(ls gpurun_out/c2_trace/*kernel_stats.csv | head -n1)
