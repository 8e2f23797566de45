# parity suite on the product lib, then A/B timing of variants over several configs
# usage: bash scripts/gpu_ab.sh "cfg1 cfg2" name1 name2 ...
set -o pipefail
mkdir -p gpurun_out/ab
CFGS=$1; shift
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/ab/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/ab/gpu_tests.log; exit 1; }
tail -1 gpurun_out/ab/gpu_tests.log
for c in $CFGS; do
for v in "$@"; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-100} --warmup 10 --cpu-seconds 0 > gpurun_out/ab/$c.$v.json 2> gpurun_out/ab/$c.$v.err || { echo "variant $v failed"; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab/$c.$v.json')); print('$c $v', d['ms_per_step'], d['config']['single_lane_ms_per_step'], d['roofline']['avg_launch_us'])"
done; done
