# ppm_ingest A/B of library variants (bench.py's PPM leg only, no encode timing of note)
set -o pipefail
mkdir -p gpurun_out/ppmab
for v in "$@"; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --ppm-steps 50 > gpurun_out/ppmab/$v.json 2> gpurun_out/ppmab/$v.err || { echo "variant $v failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ppmab/$v.json'))['ppm_ingest']; print('$v', d['ms'], d['achieved_gbs'], d['samples_match'])"
done
