# parity suite on the product lib, then per-kernel rocprof stats (one lane) per variant
# usage: bash scripts/gpu_abprof.sh CONFIG name1 name2 ...   ("base" = the product lib)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/vprof
CFG=$1; shift
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/vprof/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/vprof/gpu_tests.log; exit 1; }
tail -1 gpurun_out/vprof/gpu_tests.log
for v in "$@"; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/vprof/$v -o run --output-format csv -- python bench.py --config $CFG --steps 30 --warmup 5 --cpu-seconds 0 --lanes 1 > gpurun_out/vprof/$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
  echo "== $v"; python scripts/kstats.py gpurun_out/vprof/$v/run_kernel_stats.csv | head -6
done
