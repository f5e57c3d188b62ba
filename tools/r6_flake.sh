# Round 6 (GPU box): repeat the deferred-output C2x64r parity case with the
# current harness, then with the previous one.  bash tools/r6_flake.sh TAG
set -e
mkdir -p gpurun_out
T=${1:-fl}
timeout -k 10 300 python -u tools/r6_flake.py C2x64r 1 12 > gpurun_out/${T}_cur.txt 2>&1; tail -3 gpurun_out/${T}_cur.txt
cp harness/libscenario.so /tmp/libscenario_cur.so
cp harness/libscenario_prev.so harness/libscenario.so
timeout -k 10 300 python -u tools/r6_flake.py C2x64r 1 12 > gpurun_out/${T}_prev.txt 2>&1; tail -3 gpurun_out/${T}_prev.txt
cp /tmp/libscenario_cur.so harness/libscenario.so
