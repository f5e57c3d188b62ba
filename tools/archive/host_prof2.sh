# Host sampling profiles on the GPU box: the headline (real device) and the
# C2 leg's host control plane alone (null backend).  bash tools/host_prof2.sh TAG
set -e
TAG=${1:-cur}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hp_$TAG
D=gpurun_out/hp_$TAG
gcc -O2 -shared -fPIC -o tools/libsampler.so tools/sampler.c -ldl -lpthread
timeout -k 10 200 python tools/host_profile.py $D/head --steps 20 --warmup 2 --no-cpu --no-e2e --no-legs > $D/head_bench.log 2>&1
f=$(ls $D/head.* | head -n1)
python tools/sampler_report.py $f --top 80 > $D/head_report.txt 2>&1
cat > /tmp/lp.py <<'PY'
import ctypes, os, sys
os.environ["SAMPLER_OUT"] = sys.argv[1]
ctypes.CDLL(os.path.join(os.environ["GRAFT_REPO_ROOT"], "tools", "libsampler.so"))
sys.argv = ["x"] + sys.argv[2:]
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "tools"))
import leg_null
leg_null.main()
PY
timeout -k 10 200 python /tmp/lp.py $D/c2 C2 8 2 4 0 > $D/c2.log 2>&1
f=$(ls $D/c2.* | grep -v log | head -n1)
python tools/sampler_report.py $f --top 80 > $D/c2_report.txt 2>&1
head -3 $D/head_bench.log; cat $D/c2.log
