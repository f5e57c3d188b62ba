# GPU box: the e2e probe under environment variants, interleaved
#   bash tools/ab_e2e.sh ROUNDS "VAR=a" "VAR=b" ...
set -e
mkdir -p gpurun_out
R=$1; shift
for r in $(seq 1 $R); do
    i=0
    for a in "$@"; do
        env $a timeout -k 10 200 python tools/e2e_probe.py 10 > gpurun_out/e2e_${r}_$i.log 2>&1 || { tail -20 gpurun_out/e2e_${r}_$i.log; exit 1; }
        echo "[$a]"; grep e2e= gpurun_out/e2e_${r}_$i.log
        i=$((i+1))
    done
done
