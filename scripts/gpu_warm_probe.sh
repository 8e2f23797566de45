# does a short timed region pay for a cold GPU?  20 timed steps after 5 / 50 / 400 warmup steps
set -o pipefail
O=gpurun_out/warm/${1:-warm}
mkdir -p $O
for r in 1 2; do
  for w in 5 50 400; do
    timeout -k 10 200 python bench.py --steps 20 --warmup $w --cpu-seconds 0 --ppm-steps 0 > $O/w${w}_r$r.json 2> $O/w${w}_r$r.err || { echo "bench failed"; tail $O/w${w}_r$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/w${w}_r$r.json')); print('warmup $w', d['value'], d['ms_per_step'], d['config']['single_lane_ms_per_step'])"
  done
done
echo exit=0
