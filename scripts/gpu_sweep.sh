# bench lines of every bench.py config (no CPU baseline) + the PCIe-inclusive rates
# usage: bash scripts/gpu_sweep.sh TAG
set -o pipefail
TAG=${1:-sweep}
mkdir -p gpurun_out/$TAG
for c in 4k444q90 1080p420q75x256 8k420q50 8k420q75 8k420q95 32k420r 32k420; do
  timeout -k 10 240 python bench.py --config $c --steps ${STEPS:-30} --warmup 5 --cpu-seconds 0 > gpurun_out/$TAG/$c.json 2> gpurun_out/$TAG/$c.err || { echo "config $c failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$TAG/$c.json')); print('$c', d['value'], d['unit'], d['ms_per_step'], d['config'].get('single_lane_ms_per_step'))"
done
for c in 4k444q90 1080p420q75x256; do
  timeout -k 10 240 python scripts/e2e_rate.py --config $c --seconds 4 > gpurun_out/$TAG/e2e_$c.json 2> gpurun_out/$TAG/e2e_$c.err || { echo "e2e $c failed"; exit 1; }
  cat gpurun_out/$TAG/e2e_$c.json
done
echo exit=0
