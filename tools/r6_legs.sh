# Round 6 (GPU box): the single-stream legs (and C2) over library builds,
# interleaved.  bash tools/r6_legs.sh LIB... (names under siamese_amd/)
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for L in "$@"; do
    for leg in "C3 3 1 8" "C5 2 1 8" "C2 3 2 4"; do
      SGPU_LIB=siamese_amd/$L timeout -k 10 200 python tools/leg_run.py $leg > gpurun_out/leg_tmp.log 2>&1 || { cat gpurun_out/leg_tmp.log; exit 1; }
      echo "$L $(cat gpurun_out/leg_tmp.log)"
    done
  done
done
