# GPU box: e2e phase probe (with pinned PCIe rates), then a rocprofv3 kernel +
# memory-copy trace of a short e2e probe run -> gpurun_out/e2e_trace/
set -e
mkdir -p gpurun_out/e2e_trace
timeout -k 10 300 python tools/e2e_probe.py 10 > gpurun_out/e2e_probe.log 2>&1 || { tail -20 gpurun_out/e2e_probe.log; exit 1; }
cat gpurun_out/e2e_probe.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2e_trace -o tr -- python3 tools/e2e_probe.py 3 > gpurun_out/e2e_trace/probe.log 2>&1 || { tail -20 gpurun_out/e2e_trace/probe.log; exit 1; }
python3 tools/copy_summary.py gpurun_out/e2e_trace
