# bench value vs number of pipeline lanes
# usage: bash scripts/gpu_lanes.sh cfg "2 4 6 8"
set -o pipefail
mkdir -p gpurun_out/lanes
c=$1
for n in $2; do
  timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-200} --warmup 20 --cpu-seconds 0 --lanes $n > gpurun_out/lanes/$c.$n.json 2> gpurun_out/lanes/$c.$n.err || { echo "lanes $n failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/lanes/$c.$n.json')); print('$c lanes=$n', d['value'], d['ms_per_step'])"
done
