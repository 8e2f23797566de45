# A variant library against the product one: the GPU suite on the variant, kernel
# stats (one lane) of both, then alternating bench lines.
# usage: bash scripts/gpu_variant_ab.sh VARIANT "cfg1 cfg2" [runs]
set -o pipefail
export TMPDIR=/tmp
V=$1; CFGS=$2; RUNS=${3:-2}
O=gpurun_out/vab/$V
mkdir -p $O
VLIB=$PWD/dmmt-jpeg-encoder_amd/lib_$V/libdmmt_jpeg.so
DMMT_LIB_PATH=$VLIB timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed on $V"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in $CFGS; do
  for v in base $V; do
    if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$VLIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_$v -o run --output-format csv -- python bench.py --config $c --steps 50 --warmup 5 --cpu-seconds 0 --ppm-steps 0 --lanes 1 > $O/prof_${c}_$v.log 2>&1 || { echo "prof $v failed"; exit 1; }
    python scripts/kstats.py $(find $O/prof_${c}_$v -name 'run_kernel_stats.csv' | head -1) | grep -E "k_hist|k_emit|k_front" | sed "s/^/$c $v /"
  done
  unset DMMT_LIB_PATH
  for r in $(seq $RUNS); do
    for v in base $V; do
      if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$VLIB; fi
      for s in 20 200; do
        timeout -k 10 200 python bench.py --config $c --steps $s --warmup 5 --cpu-seconds 0 --ppm-steps 0 > $O/b_${c}_${v}_${s}_$r.json 2>> $O/bench.err || { echo "bench $v failed"; exit 1; }
        python -c "import json; d=json.load(open('$O/b_${c}_${v}_${s}_$r.json')); print('$c', '$v', 'steps $s', d['value'], 'single', d['config']['single_lane_ms_per_step'])"
      done
    done
  done
  unset DMMT_LIB_PATH
done
echo exit=0
