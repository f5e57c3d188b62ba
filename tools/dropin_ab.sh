# Drop-in C1 latency per call under environment settings, interleaved:
#   bash tools/dropin_ab.sh ROUNDS "VAR=a" "VAR=b" ...
set -e
cd $GRAFT_REPO_ROOT
R=$1; shift
for r in $(seq 1 $R); do
  for a in "$@"; do
    env $a timeout -k 10 120 python -c "
import sys; sys.path.insert(0, '.'); import bench, json
o = bench.dropin_leg('siamese_amd/libsiamese_amd.so', False)
print('[$a]', o['us_per_call'], 'us/call', o['codec_ms_per_run'], 'ms codec/run')"
  done
done
