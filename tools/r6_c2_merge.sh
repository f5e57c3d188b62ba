# Round 6 (GPU box): C2 leg with rounds merged in the deferred mode too
# (SCENARIO_MERGE_ROUNDS=2) vs not, interleaved.  bash tools/r6_c2_merge.sh TAG
set -e
mkdir -p gpurun_out
T=${1:-c2m}
for k in 1 2; do for m in 1 2; do for g in 2 4; do
  SCENARIO_MERGE_ROUNDS=$m timeout -k 10 120 python tools/leg_run.py C2 3 $g 4 | sed "s/^/merge $m /" >> gpurun_out/${T}.txt 2>&1
done; done; done
cat gpurun_out/${T}.txt
