# One experiment in one call: the -m gpu suite on the product library, rocprof
# one-lane kernel stats of each variant, then the 4-lane bench A/B.
# usage: bash scripts/gpu_exp.sh TAG "base v1 ..." [R] [cfg]
set -o pipefail
export TMPDIR=/tmp
T=$1; V=$2; R=${3:-3}; C=${4:-4k444q90}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash scripts/gpu_kstats.sh $C $V 2>&1 | grep -E "k_front|k_hist|k_emit|k_stuffwrite|failed" | tee $O/kstats.txt || exit 1
bash scripts/gpu_ab.sh $C "$V" $R 2>&1 | tee $O/ab.txt || exit 1
echo exit=0
