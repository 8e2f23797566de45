# the driver's bench command (steps 20, warmup 5) with the roofline pass after
# (last) or before (first) the timed region, R repeats each
set -o pipefail
mkdir -p gpurun_out/order
R=${1:-3}
for r in $(seq $R); do
for o in last first; do
  timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} --cpu-seconds 0 --ppm-steps 0 --no-extras --roofline-order $o > gpurun_out/order/$o.$r.json 2> gpurun_out/order/$o.$r.err || { echo "order $o failed"; tail -3 gpurun_out/order/$o.$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/order/$o.$r.json')); print('$o', d['value'], d['ms_per_step'], d['config']['single_lane_ms_per_step'])"
done
done
