# 4K bench by lane count (400 steps), R repeats: bash scripts/gpu_lanes_ab.sh "3 4 5" R
set -o pipefail
mkdir -p gpurun_out/lanesab
for r in $(seq ${2:-2}); do
  for l in $1; do
    timeout -k 10 200 python bench.py --steps 400 --warmup 20 --lanes $l --cpu-seconds 0 --ppm-steps 0 > gpurun_out/lanesab/l$l.json 2> gpurun_out/lanesab/l$l.err || { echo "lanes $l failed"; tail -3 gpurun_out/lanesab/l$l.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/lanesab/l$l.json')); print('lanes $l', d['value'], d['ms_per_step'])"
  done
done
