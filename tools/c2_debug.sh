set -e
SGPU_LIB=siamese_amd/libsiamese_amd_old.so SCENARIO_LIB=harness/libscenario_old.so timeout -k 10 120 python tools/c2_debug.py 1024 4
SGPU_LIB=siamese_amd/libsiamese_amd_old.so SCENARIO_LIB=harness/libscenario_old.so timeout -k 10 120 python tools/c2_debug.py 1024 4
timeout -k 10 120 python tools/c2_debug.py 1024 4
timeout -k 10 120 python tools/c2_debug.py 256 4
