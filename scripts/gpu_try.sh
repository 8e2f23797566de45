# Parity first, then the bench: each library variant must pass the parity subset
# (fuzz, parity, restart, stripes, the regression shapes) before it is timed.
# usage: bash scripts/gpu_try.sh "v1 v2" [bench repeats]
set -o pipefail
export TMPDIR=/tmp
V=$1; R=${2:-2}
mkdir -p gpurun_out/try
for v in $V; do
  if [ "$v" = base ]; then L=$PWD/dmmt-jpeg-encoder_amd/lib/libdmmt_jpeg.so; else L=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  DMMT_LIB_PATH=$L timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "${TRY_K:-parity or fuzz or restart or stripes or regressions}" > gpurun_out/try/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 gpurun_out/try/tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/try/tests_$v.log)"
done
bash scripts/gpu_bench_variants.sh 4k444q90 "${BASE:-base} $V" $R || exit 1
bash scripts/gpu_bench_variants.sh 8k420q75 "${BASE:-base} $V" 1 || exit 1
echo exit=0
