# k_exec time per headline launch under timing variants (tools/variant_src.py;
# outputs may be wrong, so no verification), interleaved:
#   bash tools/ab_exec_variants.sh TAG ROUNDS head norows ...
set -e
TAG=$1; R=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/abexec_$TAG.txt
: > $out
for r in $(seq 1 $R); do
  for v in "$@"; do
    lib=siamese_amd/libsiamese_amd.so
    [ "$v" != head ] && lib=siamese_amd/libsiamese_amd_$v.so
    timeout -k 10 150 python bench.py --library $lib --steps 6 --warmup 1 --no-cpu --no-e2e --no-legs --no-verify \
        > gpurun_out/abexec_${TAG}_${v}_$r.json 2>> gpurun_out/abexec_$TAG.err
    python3 - "$v" gpurun_out/abexec_${TAG}_${v}_$r.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = d["device"]["kernel_ms_per_step"]
print("%-8s k_exec %7.1f us/launch  (%s)" % (sys.argv[1], d["roofline"]["exec_ms_per_launch"] * 1e3, k))
PY
  done
done
cat $out
