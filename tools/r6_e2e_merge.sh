# Round 6 (GPU box): GPU suite, then the end-to-end leg with merged rounds
# (default) vs one fork-join per round (SCENARIO_MERGE_ROUNDS=0), interleaved.
#   bash tools/r6_e2e_merge.sh TAG
set -e
mkdir -p gpurun_out
T=${1:-e2m}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_gputests.log 2>&1 || { tail -40 gpurun_out/${T}_gputests.log; exit 1; }
tail -1 gpurun_out/${T}_gputests.log
for k in 1 2 3; do for m in 0 1; do
  SCENARIO_MERGE_ROUNDS=$m timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-legs --no-decode-ab > gpurun_out/${T}_${m}_$k.json 2> gpurun_out/${T}_${m}_$k.err
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_${m}_$k.json'))
print('merge $m', 'headline', d['ms_per_step'], 'e2e', d['end_to_end']['ms_per_step'])"
done; done
