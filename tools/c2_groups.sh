set -e
for r in 1 2; do for g in 1 2 4; do timeout -k 10 120 python tools/leg_run.py C2 3 $g; done; done
