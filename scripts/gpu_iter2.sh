# one build-measure iteration: GPU parity suite (stop on failure), then per-stage times
# and the bench line.  usage: bash scripts/gpu_iter2.sh TAG [configs...]
set -o pipefail
mkdir -p gpurun_out/iter
TAG=${1:-iter}; shift
CFGS=${@:-4k444q90 8k420q75}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/iter/${TAG}_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/iter/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/iter/${TAG}_tests.log
for c in $CFGS; do
  timeout -k 10 120 python scripts/stage_times.py --config $c --tag $TAG >> gpurun_out/iter/${TAG}_stages.jsonl 2>> gpurun_out/iter/${TAG}.err || { echo "stage times $c failed"; tail gpurun_out/iter/${TAG}.err; exit 1; }
  tail -1 gpurun_out/iter/${TAG}_stages.jsonl
done
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/iter/${TAG}_bench.json 2>> gpurun_out/iter/${TAG}.err || { echo "bench failed"; tail gpurun_out/iter/${TAG}.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/iter/${TAG}_bench.json')); print('bench', d['value'], d['ms_per_step'], d['config']['single_lane_ms_per_step'], d['roofline']['avg_launch_us'])"
