# bench lines of the main configs (no CPU baseline), then GPU parity tests
# usage: bash scripts/gpu_configs.sh TAG
set -o pipefail
TAG=${1:-cfg}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/$TAG/gpu_tests.log 2>&1 || { echo "tests failed"; tail -5 gpurun_out/$TAG/gpu_tests.log; exit 1; }
for c in 4k444q90 8k420q75 1080p420q75x256; do
  timeout -k 10 200 python bench.py --config $c --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/$TAG/$c.json 2> gpurun_out/$TAG/$c.err || exit 1
done
tail -1 gpurun_out/$TAG/gpu_tests.log
echo exit=0
