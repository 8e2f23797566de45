# A/B timing of experiment builds (make VARIANT=x): bench ms/step + k_front event time per variant
# usage: bash scripts/gpu_variants.sh name1 name2 ...   ("base" = the product lib)
set -o pipefail
mkdir -p gpurun_out/variants
for v in "$@"; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 ${BENCH_ARGS} > gpurun_out/variants/$v.json 2> gpurun_out/variants/$v.err || { echo "variant $v failed"; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/variants/$v.json')); print('$v', d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
