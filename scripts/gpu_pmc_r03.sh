# Per-kernel SQ counters of the product library (or lib_<v> for each v given):
# two passes of 8 SQ counters each, kernel-trace only, each pass under its own
# KILL timeout.  usage: bash scripts/gpu_pmc_r03.sh TAG [v...]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r03}
shift
O=gpurun_out/pmc_$TAG
mkdir -p $O
P1="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_BUSY_CYCLES"
for v in base "$@"; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  i=0
  for C in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $O/$v/p$i -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --ppm-steps 0 > $O/${v}_p$i.log 2>&1 || { echo "pmc $v pass $i failed"; tail -3 $O/${v}_p$i.log; exit 1; }
  done
  python3 scripts/pmc_summary.py $O/$v > $O/$v.txt && sed "s/^/$v /" $O/$v.txt
done
echo exit=0
