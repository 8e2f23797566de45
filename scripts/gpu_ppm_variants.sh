# PPM ingest time (bench.py's ppm_ingest line, 4K P3 text in HBM) per library variant
# usage: bash scripts/gpu_ppm_variants.sh "v1 v2" R
set -o pipefail
mkdir -p gpurun_out/ppmv
for r in $(seq ${2:-2}); do
for v in $1; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --ppm-steps 100 > gpurun_out/ppmv/$v.json 2> gpurun_out/ppmv/$v.err || { echo "variant $v failed"; tail -3 gpurun_out/ppmv/$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ppmv/$v.json'))['ppm_ingest']; print('$v', d['ms'], d['mpixel_per_s'], d['samples_match'])"
done
done
