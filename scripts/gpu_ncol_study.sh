# column-truncated coefficients at the 8K 4:2:0 q95 shape: whole path vs back half,
# product flags vs no SDWA peephole, and the first differing bit of the product build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ncol
for v in base ncnosdwa; do
  if [ "$v" = base ]; then L=$PWD/dmmt-jpeg-encoder_amd/lib/libdmmt_jpeg.so; else L=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so; fi
  DMMT_LIB_PATH=$L timeout -k 10 240 python -u tests/tools/determinism.py --n 3 > gpurun_out/ncol/det_$v.log 2>&1 || { echo "det $v failed"; tail -5 gpurun_out/ncol/det_$v.log; exit 1; }
  cat gpurun_out/ncol/det_$v.log | grep -v amdgpu.ids
done
timeout -k 10 300 python -u tests/tools/first_diff_bit.py 7680 4320 2 95 > gpurun_out/ncol/fdb.log 2>&1; tail -12 gpurun_out/ncol/fdb.log
echo exit=0
