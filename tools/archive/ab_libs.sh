# Interleaved A/B of library variants (tools/build_variant.sh) on the default
# headline bench, every recovered byte verified in the warm-up; prints
# ms/step, device time, per-kernel-class time and the digest per run.
#   bash tools/ab_libs.sh TAG ROUNDS head w16 ...   ("head" = the product .so)
set -e
TAG=$1; R=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/ablibs_$TAG.txt
: > $out
for r in $(seq 1 $R); do
  for v in "$@"; do
    lib=siamese_amd/libsiamese_amd.so
    [ "$v" != head ] && lib=siamese_amd/libsiamese_amd_$v.so
    timeout -k 10 150 python bench.py --library $lib --steps 20 --warmup 2 --no-cpu --no-e2e --no-legs \
        > gpurun_out/ablibs_${TAG}_${v}_$r.json 2>> gpurun_out/ablibs_$TAG.err
    python3 - "$v" gpurun_out/ablibs_${TAG}_${v}_$r.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("%-7s %8.3f ms/step  device %.3f  kernels %s  digest %s" % (sys.argv[1], d["ms_per_step"],
      d["device"]["device_ms_per_step"], d["device"]["kernel_ms_per_step"], d["device"]["rank0_digest"]))
PY
  done
done
cat $out
