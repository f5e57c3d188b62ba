# One leg (C2 / C3 / C5) through library variants, interleaved; prints the
# run time and per-kernel device time per run.
#   bash tools/leg_ab.sh LEG ROUNDS head tpi1 ...
set -e
LEG=$1; R=$2; shift 2
cd $GRAFT_REPO_ROOT
for r in $(seq 1 $R); do
  for v in "$@"; do
    lib=siamese_amd/libsiamese_amd.so
    [ "$v" != head ] && lib=siamese_amd/libsiamese_amd_$v.so
    timeout -k 10 200 python3 - $LEG $lib $v <<'PY'
import sys
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import bench, scenario_lib as S
leg, lib, tag = sys.argv[1:4]
cfg = S.replace(S.CONFIGS[leg], hash_data=0)
defer = 4 if leg == "C2" else 8
o = bench.run_leg(leg, lib, cfg, 0, 0, 2, None, 1, "", defer)
print("%-6s %s run %.2f ms  device %.2f  %s" % (tag, leg, o["ms_per_run"], o["device_ms_per_run"],
      {k: round(v, 3) for k, v in o["kernel_ms_per_run"].items() if v}))
PY
  done
done
