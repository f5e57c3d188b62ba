# Same-box A/B of the headline's host path (round 4): range calls with
# slabs (default) / per-packet calls with slabs / per-packet calls without
# slabs (round 3's path), interleaved.   bash tools/ab_r4_ranges.sh TAG [reps]
set -e
TAG=${1:-cur}
REPS=${2:-2}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/ab_ranges_$TAG.txt
: > $out
for r in $(seq $REPS); do
  for v in ranges perpacket noslabs; do
    case $v in
      ranges) env_=""; args="";;
      perpacket) env_=""; args="--no-ranges";;
      noslabs) env_="SIAMESE_AMD_SLABS=0"; args="--no-ranges";;
    esac
    env $env_ timeout -k 10 240 python bench.py --no-cpu --no-e2e --no-legs $args > gpurun_out/ab_${TAG}_${v}_$r.json 2>> gpurun_out/ab_${TAG}.err
    python3 - "$v" gpurun_out/ab_${TAG}_${v}_$r.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
h = d["host"]["phase_ms_per_step"]
print("%-9s %8.3f ms/step %8.1f GB/s  device %.3f ms  upload %.1f MB  create %.3f step %.3f flush %.3f  digest %s" % (
    sys.argv[1], d["ms_per_step"], d["value"], d["device"]["device_ms_per_step"],
    d["device"]["upload_bytes_per_step"] / 1e6, h["create"], h["step"], h["flush"], d["device"]["rank0_digest"]))
PY
    tail -n 1 $out
  done
done
