# Round-3 probe (GPU box): C3 kernel trace with deferred outputs, C5 / C2
# leg repeats, a short headline bench.  bash tools/r3_probe.sh TAG
set -e
TAG=${1:-cur}
D=$GRAFT_REPO_ROOT/gpurun_out/probe_$TAG
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o c3 -- python3 tools/leg_run.py C3 2 1 8 > $D/c3.log 2>&1
timeout -k 10 200 python3 tools/leg_run.py C5 3 1 8 > $D/c5.log 2>&1
timeout -k 10 200 python3 tools/leg_run.py C2 5 2 4 > $D/c2.log 2>&1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-legs --no-cpu > $D/bench.log 2>&1
cat $D/c3.log $D/c5.log $D/c2.log
python3 tools/bench_summary.py bench $D/bench.log
find $D -name "c3_kernel_stats.csv" -exec cat {} \;
