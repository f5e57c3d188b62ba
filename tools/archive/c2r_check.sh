# C2 with range calls: parity (new fixtures, the full hashed leg), then the
# leg A/B (per-packet vs range calls), interleaved.
#   bash tools/c2r_check.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "C2x64r or C1r or C1var_r or C2hr" \
    --timeout 300 --timeout-method thread > gpurun_out/c2r_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/c2r_tests_$TAG.log; exit 1; }
tail -n 1 gpurun_out/c2r_tests_$TAG.log
for r in 1 2; do
  for rg in 0 1; do
    timeout -k 10 200 python - $rg <<'PY'
import sys, os
sys.path.insert(0, "tests")
import scenario_lib as S
rg = int(sys.argv[1])
cfg = S.replace(S.CONFIGS["C2"], hash_data=0, add_ranges=rg)
sess = S.BatchSession(os.path.join("siamese_amd", "libsiamese_amd.so"), cfg, device=0)
try:
    res0, rep0 = sess.run(steps=0, warmup=1, verify=True, threads=0, groups=2, defer=4)
    assert rep0.mismatches == 0 and not any(r.status for r in res0)
    ms = []
    for _ in range(3):
        res, rep = sess.run(steps=1, warmup=0, verify=False, threads=0, groups=2, digest=False, defer=4)
        ms.append(round(rep.seconds * 1e3, 2))
finally:
    sess.close()
print("C2 ranges=%d ms/run %s" % (rg, ms))
PY
  done
done
