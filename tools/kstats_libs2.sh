# k_solve_* average durations of a short headline bench per library variant:
#   bash tools/kstats_libs2.sh TAG head preinv ...
set -e
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$@"; do
  lib=siamese_amd/libsiamese_amd.so
  [ "$v" != head ] && lib=siamese_amd/libsiamese_amd_$v.so
  D=gpurun_out/ks2_${TAG}_$v
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o ks --output-format csv -- python3 bench.py --library $lib --no-verify --steps 3 --warmup 1 --no-cpu --no-e2e --no-legs > $D/bench.json 2> $D/err.txt
  f=$(find $D -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
out = []
for r in csv.DictReader(open(sys.argv[1])):
    if "solve" in r["Name"] or "k_exec" in r["Name"]:
        out.append("%s %.1f" % (r["Name"].split("(")[0].replace("sgpu::", ""), float(r["AverageNs"]) / 1e3))
print("%-8s %s" % (sys.argv[2], "  ".join(out)))
PY
done
