# C2 on the GPU box: the real leg (groups/defer variants) beside the host
# control plane alone (null backend), and the drop-in per-call probe.
#   bash tools/c2_probe.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/c2probe_$TAG.txt
: > $OUT
for a in "5 2 4" "5 1 4" "5 2 8" "5 4 4"; do
  timeout -k 10 120 python3 tools/leg_run.py C2 $a >> $OUT 2>&1
done
for a in "3 2 4 0" "3 1 4 0" "3 2 4 1"; do
  timeout -k 10 200 python3 tools/leg_null.py C2 $a >> $OUT 2>&1
done
timeout -k 10 120 python3 tools/dropin_probe.py >> $OUT 2>&1
cat $OUT
