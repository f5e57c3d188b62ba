# Round 6 (GPU box): the headline's host pipeline timeline (SCENARIO_TIMELINE=1:
# one stderr line per phase and job) and the per-call timers, 8 groups.
#   bash tools/r6_timeline.sh TAG
set -e
mkdir -p gpurun_out
T=${1:-tl}
SCENARIO_TIMELINE=1 timeout -k 10 150 python bench.py --steps 6 --warmup 2 --no-cpu --no-e2e --no-legs --no-decode-ab > gpurun_out/${T}.json 2> gpurun_out/${T}_timeline.txt
SCENARIO_BATCH_CALLS=1 timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-legs --no-decode-ab > gpurun_out/${T}_calls.json 2> gpurun_out/${T}_calls.txt
tail -16 gpurun_out/${T}_calls.txt
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_calls.json')); print(d['ms_per_step'], d['host'])"
