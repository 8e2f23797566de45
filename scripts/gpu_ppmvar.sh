# per-kernel times of the PPM ingest kernels for experiment builds
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ppmvar
for v in "$@"; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ppmvar/$v -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --lanes 1 > gpurun_out/ppmvar/$v.log 2>&1 || { echo "variant $v failed"; tail -3 gpurun_out/ppmvar/$v.log; exit 1; }
  echo "== $v"; python scripts/kstats.py gpurun_out/ppmvar/$v/run_kernel_stats.csv | grep "ppm_fast\|ppm_count"
done
