# Interleaved same-box A/B of headline variants (round 4).  Each variant is
# "name|ENV=V ...|bench args"; REPS rounds, one bench headline run per
# variant per round.   bash tools/ab_head.sh TAG REPS 'a||' 'b|X=1|--no-ranges' ...
set -e
TAG=$1; REPS=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/ab_$TAG.txt
: > $out
for r in $(seq $REPS); do
  for v in "$@"; do
    name=${v%%|*}; rest=${v#*|}; envs=${rest%%|*}; args=${rest#*|}
    env $envs timeout -k 10 240 python bench.py --no-cpu --no-e2e --no-legs --steps 20 $args \
        > gpurun_out/ab_${TAG}_${name}_$r.json 2>> gpurun_out/ab_${TAG}.err
    python3 - "$name" gpurun_out/ab_${TAG}_${name}_$r.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
h = d["host"]["phase_ms_per_step"]
print("%-10s %8.3f ms/step %8.1f GB/s  device %.3f ms  exec %.3f  upload %.1f MB  create %.3f step %.3f flush %.3f finish %.3f  digest %s" % (
    sys.argv[1], d["ms_per_step"], d["value"], d["device"]["device_ms_per_step"], d["device"]["exec_ms_per_step"],
    d["device"]["upload_bytes_per_step"] / 1e6, h["create"], h["step"], h["flush"], h["finish"], d["device"]["rank0_digest"]))
PY
    tail -n 1 $out
  done
done
