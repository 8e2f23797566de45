# PMC counters of the PPM ingest kernels (kernel-trace only, one group per pass)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ppmpmc
i=0
for C in "SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY" "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/ppmpmc/p$i -o run --output-format csv -- python scripts/ppm_probe.py 5 > gpurun_out/ppmpmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/ppmpmc/p$i.log; exit 1; }
done
python scripts/pmc_summary.py gpurun_out/ppmpmc ppm_ || true
echo done
