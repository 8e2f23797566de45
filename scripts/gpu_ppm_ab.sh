# PPM ingest A/B: parity (the PPM GPU tests), the bench's ppm_ingest leg, and
# rocprof kernel stats, per library variant ("base" = lib/).
# usage: bash scripts/gpu_ppm_ab.sh "v1 v2" [repeats]
set -o pipefail
export TMPDIR=/tmp
V=$1; R=${2:-2}
mkdir -p gpurun_out/ppmab
lib() { if [ "$1" = base ]; then echo $PWD/dmmt-jpeg-encoder_amd/lib/libdmmt_jpeg.so; else echo $PWD/dmmt-jpeg-encoder_amd/lib_$1/libdmmt_jpeg.so; fi; }
for v in $V; do
  DMMT_LIB_PATH=$(lib $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_ppm.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ppmab/tests_$v.log 2>&1 || { echo "ppm tests $v failed"; tail -20 gpurun_out/ppmab/tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/ppmab/tests_$v.log)"
done
for r in $(seq $R); do
for v in $V; do
  DMMT_LIB_PATH=$(lib $v) timeout -k 10 120 python scripts/ppm_probe.py 300 > gpurun_out/ppmab/$v.$r.json 2>&1 || { echo "probe $v failed"; tail gpurun_out/ppmab/$v.$r.json; exit 1; }
  echo "$v $(cat gpurun_out/ppmab/$v.$r.json)"
done
done
for v in $V; do
  DMMT_LIB_PATH=$(lib $v) timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/ppmab/prof_$v -o run --output-format csv -- python3 scripts/ppm_probe.py 100 > gpurun_out/ppmab/prof_$v.log 2>&1 || { echo "rocprof $v failed"; exit 1; }
  f=$(find gpurun_out/ppmab/prof_$v -name 'run_kernel_stats.csv' | head -1)
  echo "== $v"; python scripts/kstats.py $f | grep -i ppm
done
echo exit=0
