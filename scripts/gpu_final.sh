# Round-4 closing measurements on one box: the round check (smoke, whole -m gpu
# suite, default bench line, rocprof of it), the DESIGN §5 config sweep, and the
# in-process multi-member leg (two members on GPU 0).
# usage: bash scripts/gpu_final.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-r04_final}
bash scripts/gpu_round.sh $T || exit 1
bash scripts/gpu_round_measure.sh $T || exit 1
O=gpurun_out/$T
timeout -k 10 300 python bench.py --inproc --devices 0,0 --steps 100 --warmup 10 > $O/inproc.json 2> $O/inproc.err || { echo "inproc failed"; tail -5 $O/inproc.err; exit 1; }
cat $O/inproc.json
echo exit=0
