# C2 leg under deferred-output depths, interleaved: bash tools/c2_defer_ab.sh ROUNDS 4 8 16
set -e
R=$1; shift
cd $GRAFT_REPO_ROOT
for r in $(seq 1 $R); do
  for df in "$@"; do
    timeout -k 10 200 python3 - $df <<'PY'
import sys
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import bench, scenario_lib as S
df = int(sys.argv[1])
cfg = S.replace(S.CONFIGS["C2"], hash_data=0)
o = bench.run_leg("C2", S.AMD_LIB, cfg, 0, 0, 3, None, 1, "", df)
print("defer %2d  C2 run %.2f ms (runs %s)  device %.2f" % (df, o["ms_per_run"], o.get("runs_ms"), o["device_ms_per_run"]))
PY
  done
done
