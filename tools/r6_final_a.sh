# Round 6 (GPU box): the whole GPU suite, smoke, then the profile round
# (kernel stats, PMC traffic, leg traces) of this build.  bash tools/r6_final_a.sh TAG
set -e
mkdir -p gpurun_out
T=${1:-r6}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_gputests_full.log 2>&1 || { tail -40 gpurun_out/${T}_gputests_full.log; exit 1; }
tail -1 gpurun_out/${T}_gputests_full.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
bash tools/profile_round.sh $T > gpurun_out/${T}_profile_round.log 2>&1 || { tail -20 gpurun_out/${T}_profile_round.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/prof_$T/traffic.json')); print('step traffic', d.get('_step_traffic_bytes'), {k: v['traffic_bytes'] for k, v in d.items() if k.startswith('sgpu')})"
