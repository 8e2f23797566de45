# the bench at the driver's step counts (20 steps, 5 warmup) and longer, repeated:
# the fixed cost of a short timed region.  usage: bash scripts/gpu_short_runs.sh TAG
set -o pipefail
O=gpurun_out/short/${1:-short}
mkdir -p $O
for r in 1 2 3; do
  for s in 20 50 200; do
    timeout -k 10 200 python bench.py --steps $s --warmup 5 --cpu-seconds 0 --ppm-steps 0 > $O/s${s}_r$r.json 2> $O/s${s}_r$r.err || { echo "bench $s failed"; tail $O/s${s}_r$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/s${s}_r$r.json')); print('steps $s', d['value'], d['ms_per_step'], d['config']['single_lane_ms_per_step'])"
  done
done
echo exit=0
