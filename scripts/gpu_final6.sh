# Round 6's closing evidence in one call: PMC passes + smoke + the -m gpu suite +
# the bench line + rocprof of it (gpu_round_pmc.sh), the config sweep
# (gpu_round_measure.sh), then the driver's own command three times.
# usage: bash scripts/gpu_final6.sh TAG
set -o pipefail
T=${1:-r06_final}
bash scripts/gpu_round_pmc.sh $T || exit 1
bash scripts/gpu_round_measure.sh $T || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$T/driver$i.json 2> gpurun_out/$T/driver$i.err || { echo "driver run $i failed"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$T/driver$i.json')); print('driver20', d['value'], d['ms_per_step'], d['config']['single_lane_ms_per_step'])"
done
echo exit=0
