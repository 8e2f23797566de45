# per-kernel times of experiment builds: rocprofv3 kernel stats per variant
# usage: bash scripts/gpu_variants_prof.sh name1 name2 ...   ("base" = the product lib)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/vprof
for v in "$@"; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/vprof/$v -o run --output-format csv -- python bench.py --steps 30 --warmup 5 --cpu-seconds 0 --lanes 1 > gpurun_out/vprof/$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
  echo "== $v"; python scripts/kstats.py gpurun_out/vprof/$v/run_kernel_stats.csv | head -6
done
