# The inverses on the side stream: GPU suite, interleaved headline A/B of
# SGPU_INV_SIDE=0/1, kernel stats of the default.
#   bash tools/side_check.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gt_$TAG.log 2>&1 || { tail -30 gpurun_out/gt_$TAG.log; exit 1; }
tail -n 1 gpurun_out/gt_$TAG.log
out=gpurun_out/side_ab_$TAG.txt
: > $out
for r in 1 2 3; do
  for v in 0 1; do
    SGPU_INV_SIDE=$v timeout -k 10 150 python bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-legs \
        > gpurun_out/side_${TAG}_${v}_$r.json 2>> gpurun_out/side_$TAG.err
    python3 - "side=$v" gpurun_out/side_${TAG}_${v}_$r.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("%-7s %8.3f ms/step  device %.3f  kernels %s  digest %s" % (sys.argv[1], d["ms_per_step"],
      d["device"]["device_ms_per_step"], d["device"]["kernel_ms_per_step"], d["device"]["rank0_digest"]))
PY
  done
done
cat $out
bash tools/kstats_libs.sh $TAG head
