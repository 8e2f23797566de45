# launch-gap experiment: graphs on/off, device kernargs on/off (kernel traces)
set -o pipefail
mkdir -p gpurun_out/gaps
export TMPDIR=/tmp
for v in "1 0" "0 0" "1 1"; do
  set -- $v
  tag=g$1k$2
  if [ "$2" = 1 ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
  DMMT_GRAPHS=$1 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/gaps/$tag.json 2>&1 || exit 1
done
unset HIP_FORCE_DEV_KERNARG
DMMT_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gaps/prof -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/gaps/prof.log 2>&1
echo "exit=$?"
