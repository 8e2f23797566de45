# The round's measurement table from one box and one build:
# every bench config device-resident (4 lanes; 4K also at 1 lane), then the
# PCIe-inclusive host-batch rates.  usage: bash scripts/gpu_round_measure.sh TAG
set -o pipefail
TAG=${1:-round}
O=gpurun_out/measure/$TAG
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --cpu-seconds 0 --no-extras "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail $O/$n.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['steps'])"
}
run 4k444q90 --steps 400 --warmup 40
for c in 8k420q50 8k420q75 8k420q95; do run $c --config $c --steps 200 --warmup 20 --ppm-steps 0; done
run 1080p420q75x256 --config 1080p420q75x256 --steps 30 --warmup 5 --ppm-steps 0
run 32k420r --config 32k420r --steps 10 --warmup 2 --ppm-steps 0
run 32k420 --config 32k420 --steps 10 --warmup 2 --ppm-steps 0
for cfg in "4k444q90 --batch 8" "4k444q90 --batch 1" "1080p420q75x256 --batch 64"; do
  timeout -k 10 120 python scripts/e2e_rate.py --config $cfg --seconds 4 >> $O/e2e.jsonl 2>> $O/e2e.err || { echo "e2e $cfg failed"; tail $O/e2e.err; exit 1; }
  tail -1 $O/e2e.jsonl
done
# the same at the C ABI, no Python in between (tools/e2e_c, built in-tree beforehand)
if [ -x tools/e2e_c ]; then
  for a in "3840 2160 0 90 8 8" "3840 2160 0 90 1 1" "1920 1080 2 75 64 8"; do
    timeout -k 10 60 ./tools/e2e_c $a 4 >> $O/e2e_c.jsonl 2>> $O/e2e.err || { echo "e2e_c $a failed"; exit 1; }
    tail -1 $O/e2e_c.jsonl
  done
fi
echo exit=0
