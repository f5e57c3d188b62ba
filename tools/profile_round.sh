# Collect the rocprofv3 evidence behind bench.py's roofline for one build.
# Usage (on the GPU box, from the repo root):  bash tools/profile_round.sh TAG
# Writes gpurun_out/prof_TAG/{trace,pmc_fetch,pmc_write}* and gpurun_out/prof_TAG/traffic.json.
# Each pass is its own run (counters never combined with runtime tracing).
set -e
TAG=${1:-cur}
D=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-legs --no-decode-ab"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o trace -- python3 $B > $D/bench_trace.log 2>&1
B1="bench.py --steps 1 --warmup 1 --no-cpu --no-e2e --no-legs --no-decode-ab"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D -o pmc_fetch -- python3 $B1 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D -o pmc_write -- python3 $B1 > /dev/null 2>&1
# (B1 runs 1 + 1 + 2 workload steps: timed, warm-up, the verified warm-up and the unique-bytes step)
python3 tools/pmc_traffic.py $(ls $D/pmc_fetch*counter_collection.csv | head -n1) $(ls $D/pmc_write*counter_collection.csv | head -n1) $D/traffic.json "rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per dispatch (averages), bench.py --steps 1 --warmup 1 --no-legs, tag $TAG" siamese_amd/libsiamese_amd.so 4 > /dev/null
ls -R $D | head -n 40
# single-stream legs: kernel traces of C3 and C5 (tools/leg_run.py)
# (groups and deferred-output depth as bench.py runs them)
for L in "C3 1 1 8" "C5 1 1 8" "C2 1 4 4"; do
  set -- $L
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o leg_$1 -- python3 tools/leg_run.py $L > $D/leg_$1.log 2>&1
done
# single-stream legs: PMC traffic per dispatch (each counter its own pass)
for L in "C3 1 1 8" "C5 1 1 8"; do
  set -- $L
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D -o leg_$1_fetch -- python3 tools/leg_run.py $L > /dev/null 2>&1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D -o leg_$1_write -- python3 tools/leg_run.py $L > /dev/null 2>&1
  python3 tools/pmc_traffic.py $(ls $D/leg_$1_fetch*counter_collection.csv | head -n1) $(ls $D/leg_$1_write*counter_collection.csv | head -n1) $D/leg_$1_traffic.json "rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per dispatch (averages), tools/leg_run.py $L, tag $TAG" siamese_amd/libsiamese_amd.so > /dev/null
done
