# Round 6 (GPU box): tools/r6_final_a.sh (GPU suite, smoke, profile round),
# then the full default bench line of the same build.  bash tools/r6_final_b.sh TAG
set -e
T=${1:-r6}
bash tools/r6_final_a.sh $T
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('traffic_build_matches'))"
