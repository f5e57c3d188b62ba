set -e
timeout -k 10 120 python tools/c2_debug.py 1024 2
timeout -k 10 120 python tools/c2_debug.py 1024 4
