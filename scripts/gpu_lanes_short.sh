# bench value by pipeline lane count at the driver's 20 steps and at 400 steps
set -o pipefail
O=gpurun_out/lanes_short/${1:-x}
mkdir -p $O
for r in 1 2; do
  for l in 2 3 4 6; do
    for s in 20 400; do
      timeout -k 10 200 python bench.py --steps $s --warmup 5 --lanes $l --cpu-seconds 0 --ppm-steps 0 > $O/l${l}_s${s}_r$r.json 2> $O/l${l}_s${s}_r$r.err || { echo "bench failed"; tail $O/l${l}_s${s}_r$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/l${l}_s${s}_r$r.json')); print('lanes $l steps $s', d['value'], d['ms_per_step'])"
    done
  done
done
echo exit=0
