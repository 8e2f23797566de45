# per-phase cycle trace of the `make TRACE=1` build (lib_trace), 4K and 8K
set -o pipefail
mkdir -p gpurun_out/trace
for c in ${CONFIGS:-4k444q90 8k420q75}; do
  timeout -k 10 120 python scripts/phase_trace.py --config $c --steps 20 > gpurun_out/trace/$c.txt 2>&1 || { echo "trace $c failed"; tail -5 gpurun_out/trace/$c.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/trace/$c.txt | sed "s/^/$c /"
done
