# Drop-in legs only (C1 latency per call, C2 from 16 threads with the
# reference's digests and wall time beside it): bash tools/dropin_probe.sh TAG
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "
import sys, json; sys.path.insert(0, '.'); import bench
o = {'dropin_C1': bench.dropin_leg('siamese_amd/libsiamese_amd.so', True),
     'dropin_C2_threads': bench.dropin_threads_leg('siamese_amd/libsiamese_amd.so', True, threads=16, runs=5)}
json.dump(o, open('gpurun_out/dropin_$1.json', 'w'), indent=1)
print('C1', o['dropin_C1']['us_per_call'], 'us/call ref', (o['dropin_C1']['cpu_baseline'] or {}).get('us_per_call'))
t = o['dropin_C2_threads']
print('C2x16', t['wall_ms_all'], 'ms; ref', (t['cpu_baseline'] or {}).get('wall_ms_all'), 'digests', t['digests_match_reference'])
"
