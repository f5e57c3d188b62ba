# HIP runtime-API and kernel stats of drop-in C2 (64 streams) from 16 threads:
#   bash tools/dropin_api_trace.sh TAG
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dapi_$1
cat > gpurun_out/dapi_$1/run.py <<'PY'
import sys; sys.path.insert(0, '.'); sys.path.insert(0, 'tests'); import scenario_lib as S
cfg = S.replace(S.CONFIGS['C2'], hash_data=0, streams=64)
for _ in range(2):
    res, sec, wall = S.run_capi('siamese_amd/libsiamese_amd.so', cfg, threads=16)
    print('wall', wall * 1e3, 'ms', file=sys.stderr)
PY
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d gpurun_out/dapi_$1 -o tr -- python3 gpurun_out/dapi_$1/run.py > gpurun_out/dapi_$1/log.txt 2>&1
find gpurun_out/dapi_$1 -name "*stats.csv" | while read f; do echo "== $f"; head -25 "$f"; done
rm -f gpurun_out/dapi_$1/*/*/*trace.csv gpurun_out/dapi_$1/*/*trace.csv 2>/dev/null || true
