# host control plane alone (tools/libsiamese_null.so backend): T threads, STEPS steps
timeout 600 python bench.py --library ${LIB:-tools/libsiamese_null.so} --steps ${STEPS:-20} --warmup 2 --no-cpu --no-e2e --no-legs --no-verify --threads ${T:-8} "$@" 2>&1 | python -c "
import json,sys
for l in sys.stdin:
    try: d=json.loads(l)
    except: print(l, end=''); continue
    print(d['ms_per_step'], d['host'], d['device']['rounds_per_step'], d['device']['upload_bytes_per_step'])"
