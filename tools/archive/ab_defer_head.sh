# Headline with deferred decode outputs (bench.py --defer), interleaved A/B.
#   bash tools/ab_defer_head.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/ab_defer_$TAG.txt
: > $OUT
for rep in 1 2; do
  for d in 0 1 2 4 8; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --defer $d > gpurun_out/b.json 2>/dev/null
    python3 tools/bench_summary.py "d$d" gpurun_out/b.json >> $OUT
  done
done
timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu --no-legs --defer 4 > gpurun_out/b.json 2>/dev/null
python3 -c "import json;d=json.load(open('gpurun_out/b.json'));print('e2e defer4', d['end_to_end']['ms_per_step'], d['ms_per_step'])" >> $OUT
cat $OUT
