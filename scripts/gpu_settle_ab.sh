# the bench with and without the settle phase: the driver's command (steps 20,
# warmup 5) and the default 200 steps, R repeats, plus the rep-by-rep probe
set -o pipefail
mkdir -p gpurun_out/settle
R=${1:-3}
for r in $(seq $R); do
for ms in 60 0; do
for st in "20 5" "200 20"; do
  set -- $st
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 --cpu-seconds 0 --ppm-steps 0 --no-extras --settle-ms $ms > gpurun_out/settle/s$ms.$1.$r.json 2> gpurun_out/settle/s$ms.$1.$r.err || { echo "settle $ms failed"; tail -3 gpurun_out/settle/s$ms.$1.$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/settle/s$ms.$1.$r.json')); print('settle_ms=$ms steps=$1 warmup=$2', d['value'], d['ms_per_step'], d['config']['settle'])"
done
done
done
