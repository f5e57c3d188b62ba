# Kernel + runtime-API timeline of the drop-in C1 leg (where an encode's
# round trip goes).   bash tools/dropin_trace.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=gpurun_out/dropin_$TAG
mkdir -p $D
timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $D -o tr -- python3 tools/dropin_probe.py siamese_amd/libsiamese_amd.so 2 > $D/probe.log 2>&1
ls $D
