# k_exec launch durations of a short bench (GPU box): rocprofv3 kernel trace,
# then the per-launch list (encoder / decoder launches alternate per flush).
#   bash tools/exec_trace.sh TAG [env...]  -> gpurun_out/et_TAG/
set -e
TAG=$1; shift
D=$GRAFT_REPO_ROOT/gpurun_out/et_$TAG
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-legs ${LIB:+--library $LIB} > $D/bench.log 2>&1
python3 - $D <<'PY'
import csv, sys, glob, statistics
d = sys.argv[1]
f = glob.glob(d + "/**/trace_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f))]
ks = [r for r in rows if "k_exec" in r["Kernel_Name"]]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks]
grid = [int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0) for r in ks]
print("k_exec launches", len(dur), "mean us %.1f" % statistics.mean(dur))
for g, t in list(zip(grid, dur))[-16:]:
    print("  grid %7d  %8.1f us" % (g, t))
PY
