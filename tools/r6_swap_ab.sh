# Round 6 (GPU box): the device-elimination, solve, headline-shard, large-symbol and
# end-to-end tests, then the headline over two builds interleaved (twice), and the
# host / device elimination A/B of the first.  bash tools/r6_swap_ab.sh TAG LIB_A LIB_B
set -e
mkdir -p gpurun_out
T=$1; shift
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "device_ge or chained or solve or C4x1024h or 16_mib or end_to_end" \
    > gpurun_out/${T}_gputests.log 2>&1 || { tail -40 gpurun_out/${T}_gputests.log; exit 1; }
tail -1 gpurun_out/${T}_gputests.log
bash tools/r6_libs_ab.sh $T "$@"
bash tools/r6_libs_ab.sh ${T}b "$@"
for mode in plain dge; do
  extra="--no-device-ge"; [ $mode = dge ] && extra="--device-ge"
  timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-legs --no-decode-ab $extra > gpurun_out/${T}_$mode.json 2> gpurun_out/${T}_$mode.err
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$mode.json')); h=d['host']; v=d['device']
print('$mode', d['ms_per_step'], 'ms dev', v['device_ms_per_step'], 'rounds', v['rounds_per_step'], h['phase_ms_per_step']['step'], h['phase_ms_per_step']['flush'], h['engine_ms_per_step'])"
done
