# Round 6 (GPU box): the solve tests, then the headline and the legs over two
# library builds, interleaved.  bash tools/r6_split_ab.sh TAG LIB_A LIB_B
set -e
mkdir -p gpurun_out
T=$1; shift
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "solve" \
    > gpurun_out/${T}_gputests.log 2>&1 || { tail -40 gpurun_out/${T}_gputests.log; exit 1; }
tail -1 gpurun_out/${T}_gputests.log
bash tools/r6_libs_ab.sh $T "$@"
bash tools/r6_legs.sh "$@"
