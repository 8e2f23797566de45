# phase trace + SQ counters (two passes) of the current build, 4K q90, one lane
set -o pipefail
TAG=${1:-m}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 200 python scripts/phase_trace.py --config 4k444q90 --steps 20 > gpurun_out/$TAG/phase.txt 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/$TAG/p1 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --lanes 1 > gpurun_out/$TAG/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM -d gpurun_out/$TAG/p2 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --lanes 1 > gpurun_out/$TAG/p2.log 2>&1
echo "exit=$?"
