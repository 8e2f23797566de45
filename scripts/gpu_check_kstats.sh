# GPU suite, then kernel stats (one lane) and three 20-step + one 200-step bench
# lines of the current build.  usage: bash scripts/gpu_check_kstats.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-cur}
O=gpurun_out/ck/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --ppm-steps 0 --lanes 1 > $O/prof.log 2>&1 || { echo "prof failed"; tail $O/prof.log; exit 1; }
python scripts/kstats.py $(find $O/prof -name 'run_kernel_stats.csv' | head -1)
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --ppm-steps 0 > $O/b20_$r.json 2>> $O/bench.err || { echo "bench failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/b20_$r.json')); print('20 steps', d['value'], 'single lane', d['config']['single_lane_value'])"
done
timeout -k 10 120 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 --ppm-steps 0 > $O/b200.json 2>> $O/bench.err || { echo "bench failed"; exit 1; }
python -c "import json; d=json.load(open('$O/b200.json')); print('200 steps', d['value'], 'single lane', d['config']['single_lane_value'])"
echo exit=0
