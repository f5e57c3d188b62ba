# GPU box: parity suite, smoke, the default bench line, then the rocprofv3
# evidence of this build (tools/profile_round.sh TAG); chain stops at the first failure
set -e
TAG=${1:-cur}
bash tools/gpu_check.sh
cp gpurun_out/bench.log gpurun_out/bench_$TAG.log
bash tools/profile_round.sh $TAG > gpurun_out/profile_$TAG.log 2>&1 || { tail -20 gpurun_out/profile_$TAG.log; exit 1; }
tail -3 gpurun_out/profile_$TAG.log
