# Round 6 (GPU box): C2 leg ms/run by stream groups and deferral depth
#   bash tools/r6_c2_sweep.sh TAG
set -e
mkdir -p gpurun_out
T=${1:-c2s}
for g in 2 4 8; do for d in 2 4 8; do
  timeout -k 10 120 python tools/leg_run.py C2 3 $g $d >> gpurun_out/${T}.txt 2>&1
done; done
for g in 2 4; do for d in 4; do
  timeout -k 10 120 python tools/leg_run.py C2 3 $g $d >> gpurun_out/${T}.txt 2>&1
done; done
cat gpurun_out/${T}.txt
