# C2 leg timing by stream groups (interleaved, 3 rounds)
set -e
for r in 1 2 3; do for g in 1 2; do timeout -k 10 120 python tools/leg_run.py C2 3 $g; done; done
