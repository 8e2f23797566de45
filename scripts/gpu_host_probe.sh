# host enqueue vs device time per frame, direct launches and graph replay, and the
# driver-length bench (20 steps) with graph replay.  usage: bash scripts/gpu_host_probe.sh TAG
set -o pipefail
O=gpurun_out/host/${1:-host}
mkdir -p $O
timeout -k 10 200 python scripts/host_probe.py --tag direct > $O/probe_direct.txt 2>&1 || { echo probe failed; tail $O/probe_direct.txt; exit 1; }
cat $O/probe_direct.txt
DMMT_GRAPHS=1 timeout -k 10 200 python scripts/host_probe.py --tag graphs > $O/probe_graphs.txt 2>&1 || { echo probe failed; tail $O/probe_graphs.txt; exit 1; }
cat $O/probe_graphs.txt
for r in 1 2 3; do
  DMMT_GRAPHS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --ppm-steps 0 > $O/g20_r$r.json 2> $O/g20_r$r.err || { echo "bench failed"; tail $O/g20_r$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/g20_r$r.json')); print('graphs steps 20', d['value'], d['ms_per_step'], d['config']['single_lane_ms_per_step'])"
done
echo exit=0
