# Round-3 validation of the working tree: the PPM tests and a PPM kernel profile on
# the product library, then the parity subset and the 4-lane bench A/B of the
# library variants given (lib_<v>), each GPU step under its own time limit.
# usage: bash scripts/gpu_r03_validate.sh "v1 v2"
set -o pipefail
export TMPDIR=/tmp
V=$1
O=gpurun_out/val
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "ppm or cli or convert" > $O/ppm_tests.log 2>&1 || { echo "ppm tests failed"; tail -30 $O/ppm_tests.log; exit 1; }
tail -1 $O/ppm_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ppmprof -o run --output-format csv -- python3 bench.py --cpu-seconds 0 --ppm-steps 50 --steps 20 --warmup 3 > $O/ppm_bench.json 2> $O/ppmprof.err || { echo "ppm profile failed"; tail -5 $O/ppmprof.err; exit 1; }
python scripts/kstats.py $(find $O/ppmprof -name run_kernel_stats.csv | head -1) | grep -i "ppm\|copy\|fill"
python -c "import json; print(json.load(open('$O/ppm_bench.json'))['ppm_ingest'])"
for v in $V; do
  DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "parity or fuzz or regress or baseline" > $O/${v}_tests.log 2>&1 || { echo "$v tests failed"; tail -30 $O/${v}_tests.log; exit 1; }
  echo "$v: $(tail -1 $O/${v}_tests.log)"
done
STEPS=200 bash scripts/gpu_bench_variants.sh 4k444q90 "base $V" 3 || exit 1
STEPS=200 bash scripts/gpu_bench_variants.sh 8k420q75 "base $V" 2 || exit 1
echo exit=0
