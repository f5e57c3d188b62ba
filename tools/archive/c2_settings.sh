# C2 leg under stream-group / deferral settings (verified warm-up, 3 timed runs each)
#   bash tools/c2_settings.sh TAG "g d" ...
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for gd in "$@"; do
  set -- $gd
  timeout -k 10 200 python tools/leg_run.py C2 3 $1 $2 2>&1 | tail -1
done
