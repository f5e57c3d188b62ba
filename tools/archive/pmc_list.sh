set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcic
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmcic/list.txt 2>&1 || true
grep -i "icache\|ifetch\|SQC_" gpurun_out/pmcic/list.txt | head -40
