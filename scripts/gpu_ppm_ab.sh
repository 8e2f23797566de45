# PPM A/B: the PPM GPU tests on the product and on each variant, then
# scripts/ppm_probe.py timings (R repeats) of each.
# usage: bash scripts/gpu_ppm_ab.sh TAG "v1 v2" [R]
set -o pipefail
export TMPDIR=/tmp
T=$1; V=$2; R=${3:-3}
O=gpurun_out/$T
mkdir -p $O
for v in base $V; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  [ "$v" = head ] || timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "ppm or convert" > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/tests_$v.log; exit 1; }
  [ "$v" = head ] || tail -1 $O/tests_$v.log
done
for r in $(seq $R); do
for v in base $V; do
  if [ "$v" = base ]; then unset DMMT_LIB_PATH; else export DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  timeout -k 10 120 python scripts/ppm_probe.py 200 > $O/probe_$v.json 2> $O/probe_$v.err || { echo "probe $v failed"; tail -5 $O/probe_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/probe_$v.json')); print('$v', d['ms'], d['frac'], d['samples_match'])"
done
done
echo exit=0
