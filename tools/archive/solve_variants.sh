# k_solve_mfma phase timing by variant builds (tools/build_variant.sh):
# VARIANTS="name ..." (default: skipT skipMMA skipBoth) beside the head build;
# outputs are wrong in these builds, so bench runs unverified.
#   bash tools/solve_variants.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/solvevar_$TAG.txt
: > $out
for v in ${VARIANTS:-"" skipT skipMMA skipBoth}; do
  lib=siamese_amd/libsiamese_amd${v:+_$v}.so
  timeout -k 10 200 python bench.py --library $lib --no-verify --steps 10 --warmup 1 --no-cpu --no-e2e --no-legs \
      > gpurun_out/solvevar_${TAG}_${v:-head}.json 2>> gpurun_out/solvevar_$TAG.err
  python3 - "${v:-head}" gpurun_out/solvevar_${TAG}_${v:-head}.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("%-9s %8.3f ms/step  device %.3f  kernels %s" % (sys.argv[1], d["ms_per_step"], d["device"]["device_ms_per_step"],
      d["device"]["kernel_ms_per_step"]))
PY
done
cat $out
