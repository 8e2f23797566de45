# A/B timing of experiment builds (no parity run: variants may skip work)
# usage: bash scripts/gpu_exp.sh "cfg1 cfg2" name1 name2 ...   (name "base" = product lib)
set -o pipefail
mkdir -p gpurun_out/exp
CFGS=$1; shift
for c in $CFGS; do
for v in "$@"; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-100} --warmup 10 --cpu-seconds 0 > gpurun_out/exp/$c.$v.json 2> gpurun_out/exp/$c.$v.err || { echo "variant $v failed"; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/exp/$c.$v.json')); print('$c $v', d['ms_per_step'], d['config']['single_lane_ms_per_step'], d['roofline']['avg_launch_us'])"
done; done
