# Kernel stats (rocprofv3 --kernel-trace --stats) of the default headline bench
# per library variant (tools/build_variant.sh; "head" = the product .so),
# unverified (timing variants may compute wrong bytes):
#   bash tools/kstats_libs.sh TAG head v1 ...
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$@"; do
  lib=siamese_amd/libsiamese_amd.so
  [ "$v" != head ] && lib=siamese_amd/libsiamese_amd_$v.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_${TAG}_$v -o ks \
      -- python3 bench.py --library $lib --no-verify --steps 10 --warmup 2 --no-cpu --no-e2e --no-legs \
      > gpurun_out/ks_${TAG}_$v.log 2>&1
  python3 - $v gpurun_out/ks_${TAG}_$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[2] + "/**/*kernel_stats.csv", recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0].replace("sgpu::", "")
    if n.startswith("k_"):
        out.append("%s %.1f" % (n, float(r["AverageNs"]) / 1000))
print("%-6s %s" % (sys.argv[1], "  ".join(out)))
PY
done
