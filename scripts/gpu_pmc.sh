# PMC counter passes (kernel-trace only, never with sys/runtime traces)
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
TAG=${1:-pmc}
shift
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc/$TAG/p$i -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-extras > gpurun_out/pmc/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "exit=0"
