# 4-lane bench under environment variants: bash scripts/gpu_env_ab.sh R "VAR=a" "VAR=b" ...
set -o pipefail
mkdir -p gpurun_out/envab
R=$1; shift
for r in $(seq $R); do
  for e in "$@"; do
    env $e timeout -k 10 200 python bench.py --steps ${STEPS:-400} --warmup 20 --cpu-seconds 0 --ppm-steps 0 > gpurun_out/envab/out.json 2> gpurun_out/envab/err.txt || { echo "bench $e failed"; tail -3 gpurun_out/envab/err.txt; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/envab/out.json')); print('$e', d['value'], d['ms_per_step'])"
  done
done
