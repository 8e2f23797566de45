# Round-3 A/B: product lib vs variants (bench, LDS-conflict counters, parity)
# usage: bash scripts/gpu_ab_r03.sh "v1 v2" [bench repeats]
set -o pipefail
export TMPDIR=/tmp
V=$1; R=${2:-3}
bash scripts/gpu_bench_variants.sh 4k444q90 "base $V" $R || exit 1
bash scripts/gpu_bench_variants.sh 8k420q75 "base $V" 2 || exit 1
mkdir -p gpurun_out/pmcab
for v in base $V; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES -d gpurun_out/pmcab/$v -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --ppm-steps 0 > gpurun_out/pmcab/$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/pmcab/$v 2>/dev/null | sed "s/^/$v /" || true
done
for v in $V; do
  DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "parity or fuzz or restart or stripes" > gpurun_out/ab_tests_$v.log 2>&1; echo "tests $v rc=$?"; tail -1 gpurun_out/ab_tests_$v.log
done
echo exit=0
