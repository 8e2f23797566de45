# pipelined bench by HIP hardware-queue count (GPU_MAX_HW_QUEUES) and lane count
set -o pipefail
O=gpurun_out/hwq
mkdir -p $O
for r in 1 2; do
  for q in 4 8 16; do
    for l in 4 6 8; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 400 --warmup 20 --lanes $l --cpu-seconds 0 --ppm-steps 0 > $O/q${q}_l${l}.json 2> $O/q${q}_l${l}.err || { echo "bench failed"; tail $O/q${q}_l${l}.err; exit 1; }
      python -c "import json; d=json.load(open('$O/q${q}_l${l}.json')); print('hwq $q lanes $l', d['value'], d['ms_per_step'])"
    done
  done
done
echo exit=0
