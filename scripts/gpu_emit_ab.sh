# Round-4 k_emit check: the k_emit-sensitive GPU tests on the product library,
# then the 4-lane bench A/B of the product against library variants (lib_<v>),
# then rocprof one-lane kernel stats of each.
# usage: bash scripts/gpu_emit_ab.sh TAG "v1 v2" [R]
set -o pipefail
export TMPDIR=/tmp
T=$1; V=$2; R=${3:-2}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "parity or fuzz or regress or restart or stripes or lanes" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
STEPS=200 bash scripts/gpu_bench_variants.sh 4k444q90 "base $V" $R || exit 1
STEPS=100 bash scripts/gpu_bench_variants.sh 8k420q75 "base $V" 1 || exit 1
bash scripts/gpu_kstats.sh 4k444q90 base $V || exit 1
echo exit=0
