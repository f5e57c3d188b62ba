# Round 6 (GPU box): kernel + copy traces of the headline with the host and
# the device elimination (5 steps each), for round-latency comparisons.
set -e
mkdir -p gpurun_out
T=${1:-tm}
cd /tmp && export TMPDIR=/tmp
for mode in plain dge; do
  extra="--no-device-ge"; [ $mode = dge ] && extra="--device-ge"
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_$mode -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-legs --no-decode-ab $extra > $GRAFT_REPO_ROOT/gpurun_out/${T}_$mode.log 2>&1
  grep -o '"ms_per_step": [0-9.]*' $GRAFT_REPO_ROOT/gpurun_out/${T}_$mode.log || true
done
find $GRAFT_REPO_ROOT/gpurun_out/${T}_plain $GRAFT_REPO_ROOT/gpurun_out/${T}_dge -name '*.csv' | head
