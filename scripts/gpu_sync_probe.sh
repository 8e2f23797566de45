# host-side completion latency per device scheduling flag (tools/sync_probe, built
# in-tree beforehand), then the driver's 20-step bench line per DMMT_SCHEDULE
set -o pipefail
mkdir -p gpurun_out/sync
for f in "-1 pre" "1 pre" "2 pre" "1 post" "2 post"; do
  timeout -k 10 60 ./tools/sync_probe $f >> gpurun_out/sync/probe.jsonl 2>> gpurun_out/sync/probe.err || { echo "probe $f failed"; exit 1; }
  tail -1 gpurun_out/sync/probe.jsonl
done
for r in 1 2 3; do
  for s in auto spin yield; do
    DMMT_SCHEDULE=$s timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --ppm-steps 0 > gpurun_out/sync/b_${s}_${r}.json 2>> gpurun_out/sync/bench.err || { echo "bench $s failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/sync/b_${s}_${r}.json')); print('$s', $r, d['value'], d['config']['single_lane_value'])"
  done
done
echo exit=0
