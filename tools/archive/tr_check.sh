# k_solve_tr on the GPU box: its parity tests, an interleaved headline A/B
# against the sweeps, and kernel stats of the TR build.
#   bash tools/tr_check.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "product_solve_paths or C4x1024h or C2h" \
    --timeout 300 --timeout-method thread > gpurun_out/tr_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tr_tests_$TAG.log; exit 1; }
tail -n 2 gpurun_out/tr_tests_$TAG.log
out=gpurun_out/tr_ab_$TAG.txt
: > $out
for r in 1 2 3; do
  for v in 0 1; do
    SGPU_TR_SOLVE=$v timeout -k 10 150 python bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-legs \
        > gpurun_out/tr_${TAG}_${v}_$r.json 2>> gpurun_out/tr_$TAG.err
    python3 - "tr=$v" gpurun_out/tr_${TAG}_${v}_$r.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("%-5s %8.3f ms/step  device %.3f  kernels %s  digest %s" % (sys.argv[1], d["ms_per_step"],
      d["device"]["device_ms_per_step"], d["device"]["kernel_ms_per_step"], d["device"]["rank0_digest"]))
PY
  done
done
cat $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SGPU_TR_SOLVE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr_prof_$TAG -o tr \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-legs > gpurun_out/tr_prof_$TAG.log 2>&1
python3 - gpurun_out/tr_prof_$TAG <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("%-40s %6s calls  avg %8.1f us" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1000))
PY
