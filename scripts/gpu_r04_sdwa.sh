# Round-4 SDWA study (profiles/r03_kemit_fault_study.md, "Round 4"): the failing
# round-2 build (study_wip/ = commit 71130cf + profiles/r03_kemit_fault_wip.patch,
# rebuilt here, not committed) at the failing shape (8K 4:2:0 q95, frame 95):
#  lib        as shipped then (-O3, SDWA peephole on), walk order from LDS atomics
#  lib_det    the same with ties in the walk order broken by thread index
#  lib_detnosdwa  lib_det without the SDWA peephole
set -o pipefail
O=$PWD/gpurun_out/sdwa
mkdir -p $O
cd study_wip
for v in lib lib_det lib_detnosdwa; do
  DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/$v/libdmmt_jpeg.so timeout -k 10 240 python scripts/debug_determinism.py --n 3 > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  grep -v amdgpu.ids $O/$v.log
done
echo exit=0
