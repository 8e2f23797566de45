# k_emit fault study, step 6: the failing build's device assembly replayed
# unchanged (control) and with `s_nop 1` before / after each of k_emit's 605
# SDWA instructions (nothing else changed: same registers, same schedule).
set -o pipefail
O=$PWD/gpurun_out/fault6
mkdir -p $O
cd study_wip
for v in ${VARIANTS:-as_orig as_nop_before as_nop_after}; do
  DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so timeout -k 10 200 python scripts/debug_determinism.py --n 4 > $O/$v.log 2>&1
  echo "$v rc=$?"; grep -v amdgpu.ids $O/$v.log
done
echo exit=0
