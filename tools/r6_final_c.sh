# Round 6 (GPU box): tools/r6_final_b.sh (GPU suite, smoke, profile round,
# full bench), then the k_exec SQ/TCC/LDS counter passes (tools/pmc_exec.sh).
#   bash tools/r6_final_c.sh TAG
set -e
T=${1:-r6}
bash tools/r6_final_b.sh $T
bash tools/pmc_exec.sh > gpurun_out/${T}_pmc_exec.txt 2>&1 || { tail -5 gpurun_out/${T}_pmc_exec.txt; exit 1; }
grep -A 20 "k_exec" gpurun_out/${T}_pmc_exec.txt | head -24
