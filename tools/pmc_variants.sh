# SQ instruction counters of k_exec per headline dispatch for library variants:
#   bash tools/pmc_variants.sh TAG head norows ...
set -e
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$@"; do
  lib=siamese_amd/libsiamese_amd.so
  [ "$v" != head ] && lib=siamese_amd/libsiamese_amd_$v.so
  D=gpurun_out/pmcv_${TAG}_$v
  mkdir -p $D
  B="bench.py --library $lib --steps 1 --warmup 1 --no-cpu --no-e2e --no-legs --no-verify"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $D -o sq -- python3 $B > $D/sq.log 2>&1
  echo "== $v"; python3 tools/pmc_summary.py $D/sq_counter_collection.csv | grep -A 9 "k_exec" | tail -8
done
