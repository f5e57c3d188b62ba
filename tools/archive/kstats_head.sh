# Kernel statistics of a short headline bench: bash tools/kstats_head.sh TAG
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=gpurun_out/ks_$1
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o ks --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --no-legs > $D/bench.json 2> $D/err.txt
f=$(find $D -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-40s %6s calls  avg %8.1f us  total %8.2f ms" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
