# HBM traffic + VALU counters of the bench workload, one counter group per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), kernel-trace only.
# usage: bash scripts/gpu_traffic.sh TAG [bench args...]   -> gpurun_out/pmc/TAG/p*/
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-traffic}
shift
mkdir -p gpurun_out/pmc/$TAG
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc/$TAG/p$i -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-extras --settle-ms 0 "$@" > gpurun_out/pmc/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "exit=0"
