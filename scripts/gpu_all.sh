# smoke -> gpu tests -> bench -> rocprofv3 kernel stats; stops at the first failure
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds ${CPU_SECONDS:-12} > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/$TAG -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --lanes 1 > gpurun_out/prof_bench.log 2>&1
echo "exit=$?"
