# T build in registers: solve-path tests, kernel stats against the LDS
# T build, VALU issue rates.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "random_systems or product_solve or C4x1024h or C2h" \
    --timeout 200 --timeout-method thread > gpurun_out/st_r4z.log 2>&1 || { tail -30 gpurun_out/st_r4z.log; exit 1; }
tail -n 1 gpurun_out/st_r4z.log
bash tools/kstats_libs.sh r4z head tbold
timeout -k 10 60 ./tools/valu_rate
