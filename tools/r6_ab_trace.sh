# Round 6 (GPU box): tools/r6_swap_ab.sh (tests, headline A/B, placements),
# then kernel + copy traces of both builds (tools/r6_trace_libs.sh) and their
# per-round latency (tools/trace_rounds.py).  bash tools/r6_ab_trace.sh TAG LIB_A LIB_B
set -e
T=$1; shift
bash tools/r6_swap_ab.sh $T "$@"
bash tools/r6_trace_libs.sh ${T}t "$@"
for L in "$@"; do python3 tools/trace_rounds.py gpurun_out/${T}t_$L; done
