# rocprofv3 kernel stats of the PPM ingest (scripts/ppm_probe.py) per library variant
# usage: bash scripts/gpu_ppm_kstats.sh TAG name1 name2 ...   (name "base" = product lib)
set -o pipefail
export TMPDIR=/tmp
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
for v in "$@"; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 scripts/ppm_probe.py 100 > $O/$v.log 2>&1 || { echo "variant $v failed"; tail -3 $O/$v.log; exit 1; }
  f=$(find $O/$v -name 'run_kernel_stats.csv' | head -1)
  python scripts/kstats.py $f | grep ppm | sed "s/^/$v /"
done
echo exit=0
