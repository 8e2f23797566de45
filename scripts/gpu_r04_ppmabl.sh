# PPM kernel time per library variant (rocprof kernel stats of scripts/ppm_probe.py)
# usage: bash scripts/gpu_r04_ppmabl.sh TAG "base v1 v2"
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for v in $2; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 scripts/ppm_probe.py 30 > $O/$v.log 2>&1 || { echo "variant $v failed"; tail -5 $O/$v.log; exit 1; }
  python scripts/kstats.py $(find $O/$v -name run_kernel_stats.csv | head -1) | grep ppm | sed "s/^/$v /"
done
echo exit=0
