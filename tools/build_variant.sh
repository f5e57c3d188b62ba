# Build an experimental variant of the product library with extra defines
# (applied to host and device code alike), for A/B timing on the GPU box:
#   bash tools/build_variant.sh NAME -DFOO=1 ...
# Produces siamese_amd/libsiamese_amd_NAME.so (git-ignored; run it with
# `python bench.py --library siamese_amd/libsiamese_amd_NAME.so`).
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd $ROOT/siamese_amd
OUT=build/var_$NAME
mkdir -p $OUT
HOST="gf codedef pool placement engine encoder decoder arq api batch frames"
for f in $HOST; do
    g++ -std=c++17 -O2 -g -mavx2 -fPIC -ftls-model=initial-exec -fvisibility=hidden "$@" -c csrc/$f.cpp -o $OUT/$f.o &
done
/opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -fPIC -ftls-model=initial-exec -fvisibility=hidden \
    -Wno-unused-parameter -Wno-unused-result "$@" -c csrc/backend_hip.hip -o $OUT/backend_hip.o
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libsiamese_amd_$NAME.so $OUT/*.o -lpthread
echo built siamese_amd/libsiamese_amd_$NAME.so
