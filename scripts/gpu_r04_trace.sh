# phase traces of thread 0's wave (lib_trace) and thread 192's (lib_trace3: the
# chunk's heaviest blocks in k_emit) at 4K q90
set -o pipefail
O=gpurun_out/r04_trace
mkdir -p $O
for v in trace trace3; do
  DMMT_TRACE_LIB=lib_$v timeout -k 10 120 python scripts/phase_trace.py --config 4k444q90 --steps 20 > $O/$v.txt 2>&1 || { echo "trace $v failed"; tail -5 $O/$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/$v.txt
done
echo exit=0
