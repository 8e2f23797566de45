# rocprofv3 kernel stats of one bench config per library variant
# usage: bash scripts/gpu_kstats.sh cfg name1 name2 ...   (name "base" = product lib)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/kstats
c=$1; shift
for v in "$@"; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kstats/$v -o run --output-format csv -- python bench.py --config $c --steps 50 --warmup 5 --cpu-seconds 0 --lanes 1 --no-extras > gpurun_out/kstats/$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
  f=$(find gpurun_out/kstats/$v -name 'run_kernel_stats.csv' | head -1)
  python scripts/kstats.py $f | sed "s/^/$v /"
done
