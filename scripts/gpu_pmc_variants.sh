# one SQ counter pass per library variant (kernel-trace only)
# usage: bash scripts/gpu_pmc_variants.sh name1 name2 ...   (name "base" = product lib)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcv
for v in "$@"; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU -d gpurun_out/pmcv/$v/p1 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/pmcv/$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
  echo "== $v"; python scripts/pmc_summary.py gpurun_out/pmcv/$v | grep -A6 "k_front<1\|k_emit(" | grep -v "^--"
done
