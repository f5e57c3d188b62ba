# Round 6 (GPU box): the suite-sequence deferred stress (tools/r6_flake3.py)
# with the current library, then with LIB copied over it.  bash tools/r6_flake_libs.sh TAG REPS LIB
mkdir -p gpurun_out
T=$1; R=$2; L=$3
timeout -k 10 500 python -u tools/r6_flake3.py $R > gpurun_out/${T}_cur.txt 2>&1; tail -2 gpurun_out/${T}_cur.txt
cp siamese_amd/libsiamese_amd.so /tmp/cur.so && cp siamese_amd/$L siamese_amd/libsiamese_amd.so
timeout -k 10 500 python -u tools/r6_flake3.py $R > gpurun_out/${T}_alt.txt 2>&1; tail -2 gpurun_out/${T}_alt.txt
cp /tmp/cur.so siamese_amd/libsiamese_amd.so
