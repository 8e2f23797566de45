# per-stage HIP-event times (one lane) of one config per library variant ("base" = product lib)
# usage: bash scripts/gpu_stage_variants.sh cfg name1 name2 ...
set -o pipefail
mkdir -p gpurun_out/stages
c=$1; shift
for v in "$@"; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 120 python scripts/stage_times.py --config $c --tag $v >> gpurun_out/stages/$c.jsonl 2>> gpurun_out/stages/$c.err || { echo "variant $v failed"; tail -5 gpurun_out/stages/$c.err; exit 1; }
  tail -1 gpurun_out/stages/$c.jsonl
done
