# Round 6 (GPU box): kernel + copy traces of the device-elimination headline
# over library builds (5 steps each).  bash tools/r6_trace_libs.sh TAG LIB...
set -e
mkdir -p gpurun_out
T=$1; shift
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_$L -o run -- python3 $GRAFT_REPO_ROOT/bench.py --library $GRAFT_REPO_ROOT/siamese_amd/$L --steps 5 --warmup 2 --no-cpu --no-e2e --no-legs --no-decode-ab > $GRAFT_REPO_ROOT/gpurun_out/${T}_$L.log 2>&1
  grep -o '"ms_per_step": [0-9.]*' $GRAFT_REPO_ROOT/gpurun_out/${T}_$L.log || true
done
