# 4-lane bench value per library variant ("base" = product lib), R repeats each
# usage: bash scripts/gpu_bench_variants.sh cfg "v1 v2 ..." [R]
set -o pipefail
mkdir -p gpurun_out/benchv
c=$1; R=${3:-2}
for r in $(seq $R); do
for v in $2; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-400} --warmup ${WARMUP:-20} --cpu-seconds 0 --ppm-steps 0 --no-extras > gpurun_out/benchv/$c.$v.json 2> gpurun_out/benchv/$c.$v.err || { echo "variant $v failed"; tail -3 gpurun_out/benchv/$c.$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/benchv/$c.$v.json')); k=d['roofline']['kernels']; print('$c', '$v', d['value'], d['ms_per_step'], d['config']['single_lane_ms_per_step'], ' '.join(f'{n[2:]}={v[\"avg_launch_us\"]}' for n, v in k.items()))"
done
done
