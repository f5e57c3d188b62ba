# host control plane alone (null backend) at several thread counts (GPU box's host)
set -e
for t in 1 4 8 16; do
    echo "T=$t"; T=$t STEPS=${STEPS:-6} bash tools/host_only_bench.sh
done
