# A/B of library variants and environment switches on the 4-lane bench, R rounds.
# usage: bash scripts/gpu_ab.sh cfg "spec1 spec2 ..." [R]
#   spec = variant[:VAR=value[,VAR=value]]   (variant "base" = the product library)
#   e.g. "base base:DMMT_FRONT_HIST=0 s0"
# STEPS / WARMUP from the environment (default 200 / 20); BENCH_ARGS appended to
# the bench command, ABTAG to the run names (e.g. BENCH_ARGS="--lanes 3" ABTAG=_l3).
set -o pipefail
mkdir -p gpurun_out/ab
c=$1; R=${3:-2}
for r in $(seq $R); do
for spec in $2; do
  v=${spec%%:*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*:}
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  tag=$(echo "$spec" | tr ':,=' '___')
  env ${envs//,/ } timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-200} --warmup ${WARMUP:-20} --cpu-seconds 0 --ppm-steps 0 --no-extras ${BENCH_ARGS} > gpurun_out/ab/$c.$tag${ABTAG}.json 2> gpurun_out/ab/$c.$tag${ABTAG}.err || { echo "spec $spec failed"; tail -3 gpurun_out/ab/$c.$tag${ABTAG}.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab/$c.$tag${ABTAG}.json')); k=d['roofline']['kernels']; print('$c', '$spec${ABTAG}', d['value'], d['ms_per_step'], d['config']['single_lane_ms_per_step'], ' '.join(f'{n[2:]}={v[\"avg_launch_us\"]}' for n, v in k.items()))"
done
done
