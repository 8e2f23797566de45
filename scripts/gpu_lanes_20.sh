# bench value by pipeline lane count at the driver's 20 steps (4 runs) and 200 steps
set -o pipefail
O=gpurun_out/lanes20
mkdir -p $O
for r in 1 2 3 4; do
  for l in 3 4 5 6; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --lanes $l --cpu-seconds 0 --ppm-steps 0 > $O/l${l}_r$r.json 2>> $O/err || { echo "bench failed"; exit 1; }
    python -c "import json; d=json.load(open('$O/l${l}_r$r.json')); print('lanes $l steps 20', d['value'])"
  done
done
for l in 3 4 5 6; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --lanes $l --cpu-seconds 0 --ppm-steps 0 > $O/l${l}_200.json 2>> $O/err || { echo "bench failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/l${l}_200.json')); print('lanes $l steps 200', d['value'])"
done
echo exit=0
