# SDWA bisection of the round-3 k_emit fault (tools/sdwa_bisect.py builds the
# variants into sdwa_study/libs/; profiles/r03_kemit_fault_study.md "Round 5").
# Each variant: 3 encodes of the failing shape (8K 4:2:0 q95, frame 95), whole
# path and back half, against the oracle (the study tree's determinism script).
#   bash scripts/gpu_sdwa_bisect.sh [--product] VARIANT...
# --product also runs tests/test_gpu_parity.py on this tree's SDWA-on build
# (make VARIANT=sdwa SDWA=1).  sdwa_study/ is in .gpurunignore: drop that line
# to run this again.
set -o pipefail
O=$PWD/gpurun_out/sdwa_bisect
S=$PWD/sdwa_study
mkdir -p $O
if [ "$1" = "--product" ]; then
  shift
  DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_sdwa/libdmmt_jpeg.so timeout -k 10 500 \
    python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 240 --timeout-method thread > $O/product_sdwa.log 2>&1
  rc=$?
  tail -3 $O/product_sdwa.log
  # (failures are a result here; a time limit, abort or fault ends the run)
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "product_sdwa rc=$rc"; exit 1; fi
fi
for v in "$@"; do
  DMMT_LIB_PATH=$S/libs/$v/libdmmt_jpeg.so timeout -k 10 240 python3 $S/scripts/debug_determinism.py --n 3 > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  grep -v amdgpu.ids $O/$v.log
done
echo exit=0
