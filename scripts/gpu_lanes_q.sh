# lanes x GPU_MAX_HW_QUEUES sweep of the settled bench (steps 200)
set -o pipefail
mkdir -p gpurun_out/lanesq
for q in ${QS:-4 8}; do
for l in ${LANES:-3 4 5 6 8}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps ${STEPS:-200} --warmup ${WARMUP:-20} --cpu-seconds 0 --ppm-steps 0 --no-extras --lanes $l > gpurun_out/lanesq/q$q.l$l.json 2> gpurun_out/lanesq/q$q.l$l.err || { echo "q$q l$l failed"; tail -3 gpurun_out/lanesq/q$q.l$l.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/lanesq/q$q.l$l.json')); print('Q=$q lanes=$l steps=${STEPS:-200}', d['value'], d['ms_per_step'])"
done
done
