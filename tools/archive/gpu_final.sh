# GPU box: parity suite, smoke, default bench line, then the k_exec SQ/TCC/LDS counter passes
set -e
bash tools/gpu_check.sh
bash tools/pmc_exec.sh > gpurun_out/pmc_summary.txt 2>&1 || { tail -20 gpurun_out/pmc_summary.txt; exit 1; }
grep -A20 "k_exec" gpurun_out/pmc_summary.txt | head -24
