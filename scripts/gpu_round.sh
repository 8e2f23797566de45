# One round check on the GPU box, every step under its own time limit, stopping at
# the first failure: smoke, the whole -m gpu suite, the default bench line, and
# rocprofv3 kernel stats of the same bench command (profiles/<TAG>_*).
# usage: bash scripts/gpu_round.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-r03}
K=${2:-}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread "${KA[@]}" > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-extras > $O/bench_prof.json 2> $O/bench_prof.err || { echo "rocprof bench failed"; tail $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name 'run_kernel_stats.csv' | head -1)
cp $f $O/kernel_stats.csv
python scripts/kstats.py $f
python scripts/kstats_passes.py $(dirname $f)/run_kernel_trace.csv $O/kernel_passes.csv 20 200 $O/bench_prof.json
echo exit=0
