# Round 6 (GPU box): per-call host timers of the headline (SCENARIO_BATCH_CALLS),
# host and device elimination.
set -e
mkdir -p gpurun_out
for mode in plain dge; do
  extra="--no-device-ge"; [ $mode = dge ] && extra="--device-ge"
  SCENARIO_BATCH_CALLS=1 timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs $extra > gpurun_out/calls_$mode.json 2> gpurun_out/calls_$mode.err
  echo "== $mode"; grep "^batch" gpurun_out/calls_$mode.err | tail -14
done
