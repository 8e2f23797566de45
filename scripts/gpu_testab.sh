# parity suite on the product lib, then A/B timing of variants (scripts/gpu_exp.sh)
# usage: bash scripts/gpu_testab.sh "cfg1 cfg2" name1 name2 ...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash scripts/gpu_exp.sh "$@"
