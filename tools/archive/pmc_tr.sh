# SQ counters of the solve kernels on the headline (one counter pass):
#   bash tools/pmc_tr.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS \
    --kernel-trace --output-format csv -d gpurun_out/pmc_tr_$TAG -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --no-legs \
    > gpurun_out/pmc_tr_$TAG.log 2>&1
python3 - gpurun_out/pmc_tr_$TAG <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("sgpu::", "")
    if not k.startswith("k_solve") and k != "k_exec":
        continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, c in acc.items():
    d = max(v for (kk, _), v in n.items() if kk == k)
    print(k, "dispatches", d, " ".join("%s=%.3g" % (cn, v / d) for cn, v in sorted(c.items())))
PY
