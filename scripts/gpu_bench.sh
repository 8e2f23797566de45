set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 12 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/prof_bench.log 2>&1
echo "exit=$?"
