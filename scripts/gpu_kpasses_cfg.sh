# rocprofv3 kernel statistics of the bench on other BASELINE configs, split into
# the settle / timed (pipelined) / one-lane passes (scripts/kstats_passes.py).
# usage: bash scripts/gpu_kpasses_cfg.sh TAG "cfg:steps:warmup ..."
set -o pipefail
T=$1
for spec in $2; do
  IFS=: read c K W <<< "$spec"
  O=gpurun_out/$T/$c; mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config $c --steps $K --warmup $W --cpu-seconds 0 --ppm-steps 0 --no-extras > $O/bench_prof.json 2> $O/bench_prof.err || { echo "rocprof $c failed"; tail $O/bench_prof.err; exit 1; }
  f=$(ls $O/prof/*/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$f" ] || f=$(find $O/prof -name 'run_kernel_stats.csv' | head -1)
  cp $f $O/kernel_stats.csv
  python scripts/kstats_passes.py $(dirname $f)/run_kernel_trace.csv $O/kernel_passes.csv $W $K $O/bench_prof.json || exit 1
  echo "== $c"; grep -v "^k_synthetic\|^__amd" $O/kernel_passes.csv | grep "timed\|one_lane" || true
done
echo exit=0
