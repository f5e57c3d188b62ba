set -e
cd $GRAFT_REPO_ROOT
bash tools/dropin_libs.sh 3 siamese_amd/libsiamese_amd_slots.so siamese_amd/libsiamese_amd_split.so > gpurun_out/split_dropin.txt 2>&1
bash tools/leg_ab.sh C3 2 slots split > gpurun_out/split_c3.txt 2>&1
bash tools/leg_ab.sh C2 2 slots split > gpurun_out/split_c2.txt 2>&1
bash tools/ab_libs.sh split 3 slots split > /dev/null 2>&1
