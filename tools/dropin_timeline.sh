# Engine timeline of drop-in C2 (64 streams) from 16 threads: bash tools/dropin_timeline.sh TAG
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SGPU_TIMELINE=1 timeout -k 10 200 python -u -c "
import sys; sys.path.insert(0, '.'); sys.path.insert(0, 'tests'); import scenario_lib as S
cfg = S.replace(S.CONFIGS['C2'], hash_data=0, streams=64)
S.run_capi('siamese_amd/libsiamese_amd.so', cfg, threads=16)
res, sec, wall = S.run_capi('siamese_amd/libsiamese_amd.so', cfg, threads=16)
print('wall', wall * 1e3, 'ms', file=sys.stderr)
" 2> gpurun_out/dtl_$1.txt
python3 tools/timeline_stats.py gpurun_out/dtl_$1.txt
