# quick iteration: gpu parity tests -> bench (no CPU baseline) -> phase trace -> kernel stats
# usage: bash scripts/gpu_iter.sh TAG [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-iter}
mkdir -p gpurun_out/$TAG
K=${2:+-k "$2"}
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider $K > gpurun_out/$TAG/gpu_tests.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err && \
timeout -k 10 200 python scripts/phase_trace.py > gpurun_out/$TAG/trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --lanes 1 > gpurun_out/$TAG/prof.log 2>&1
rc=$?
echo "exit=$rc"
tail -2 gpurun_out/$TAG/gpu_tests.log
exit $rc
