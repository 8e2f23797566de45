# PMC passes over the PPM ingest (scripts/ppm_probe.py): one counter group per run,
# kernel trace only (never with sys/runtime traces)
# usage: bash scripts/gpu_pmc_ppm.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-ppmpmc}
O=gpurun_out/$T
mkdir -p $O
i=0
for C in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE" "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $O/p$i -o run --output-format csv -- python3 scripts/ppm_probe.py 20 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 1; }
done
python scripts/pmc_summary.py $O ppm
echo exit=0
