# The bench's legs without CPU baselines or the e2e leg; prints per-leg times.
#   bash tools/legs_probe.sh TAG
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --no-cpu --no-e2e > gpurun_out/legs_$1.json 2> gpurun_out/legs_$1.err
python3 - gpurun_out/legs_$1.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("head", d["ms_per_step"], "ms/step", d["device"]["kernel_ms_per_step"])
for k, v in d["legs"].items():
    print(k, {x: v[x] for x in ("ms_per_run", "wall_ms", "device_ms_per_run", "us_per_call", "wall_ms_all",
                                "kernel_ms_per_run", "runs_ms") if x in v})
PY
