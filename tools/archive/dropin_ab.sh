# Drop-in legs (C1 per call, C2 from 16 threads) under environment settings,
# interleaved on one box:  bash tools/dropin_ab.sh ROUNDS "VAR=a" "VAR=b" ...
set -e
cd $GRAFT_REPO_ROOT
R=$1; shift
for r in $(seq 1 $R); do
  for a in "$@"; do
    env $a timeout -k 10 120 python -c "
import sys; sys.path.insert(0, '.'); import bench
o = bench.dropin_leg('siamese_amd/libsiamese_amd.so', False, runs=3)
t = bench.dropin_threads_leg('siamese_amd/libsiamese_amd.so', False, threads=16, runs=2)
print('[$a]', o['us_per_call'], 'us/call; C2x16', t['wall_ms_all'], 'ms')"
  done
done
