# Drop-in legs (C1 per call, C2 from 16 threads) of several library builds,
# interleaved on one box:  bash tools/dropin_libs.sh ROUNDS LIB1 LIB2 ...
set -e
cd $GRAFT_REPO_ROOT
R=$1; shift
for r in $(seq 1 $R); do
  for lib in "$@"; do
    timeout -k 10 120 python -c "
import sys; sys.path.insert(0, '.'); import bench
o = bench.dropin_leg('$lib', False, runs=3)
t = bench.dropin_threads_leg('$lib', False, threads=16, runs=2)
print('[$lib]', o['us_per_call'], 'us/call; C2x16', t['wall_ms_all'], 'ms')"
  done
done
