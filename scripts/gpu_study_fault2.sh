# k_emit fault study, step 2: variants of the failing round-2 WIP build
# (study_wip/dmmt-jpeg-encoder_amd/lib_<v>): 8K 4:2:0 q95, 3 encodes each.
set -o pipefail
O=$PWD/gpurun_out/fault2
mkdir -p $O
cd study_wip
for v in ${VARIANTS:-wait kmax63 noreadfirst rewalk}; do
  DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so timeout -k 10 200 python scripts/debug_determinism.py --n 3 > $O/$v.log 2>&1
  echo "$v rc=$?"; grep -v amdgpu.ids $O/$v.log
done
[ -n "$NOBITS" ] || timeout -k 10 200 python scripts/debug_bits.py 7680 4320 2 95 > $O/bits_fail.log 2>&1; echo "bits rc=$?"; grep -v amdgpu.ids $O/bits_fail.log
echo exit=0
