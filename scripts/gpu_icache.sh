# instruction-cache counters of the current build, 4K q90, one lane
set -o pipefail
TAG=${1:-ic}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU -d gpurun_out/$TAG/p1 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --lanes 1 > gpurun_out/$TAG/p1.log 2>&1
echo "exit=$?"
