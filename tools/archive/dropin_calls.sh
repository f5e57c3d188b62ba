# Per-call times of drop-in C2 from 1 and 16 threads: bash tools/dropin_calls.sh TAG
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for T in 1 16; do
SCENARIO_CAPI_CALLS=1 timeout -k 10 200 python -u -c "
import sys; sys.path.insert(0, '.'); sys.path.insert(0, 'tests'); import scenario_lib as S
cfg = S.replace(S.CONFIGS['C2'], hash_data=0)
S.run_capi('siamese_amd/libsiamese_amd.so', cfg, threads=1)
res, sec, wall = S.run_capi('siamese_amd/libsiamese_amd.so', cfg, threads=$T)
print('threads $T wall', wall * 1e3, 'ms codec', sec * 1e3, file=sys.stderr)
" 2> gpurun_out/dcalls_$1_$T.txt
python3 - gpurun_out/dcalls_$1_$T.txt <<'PY'
import sys, collections
agg = collections.defaultdict(lambda: [0.0, 0.0])
for ln in open(sys.argv[1]):
    p = ln.split()
    if p and p[0] == 'capi':
        agg[p[1]][0] += float(p[2]); agg[p[1]][1] += float(p[4])
    elif p: print(ln.strip())
for k, (c, us) in agg.items():
    print('%-14s %9.0f calls %10.1f us %7.2f us/call' % (k, c, us, us / max(c, 1)))
PY
done
