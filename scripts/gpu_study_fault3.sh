# k_emit fault study, step 3: per-block dump of what the failing WIP k_emit's walk
# read (its DC difference) and wrote (its first slot word); -O3 and -O1 builds.
set -o pipefail
O=$PWD/gpurun_out/fault3
mkdir -p $O
cd study_wip
for v in dump dumpo1; do
  DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_$v/libdmmt_jpeg.so timeout -k 10 280 python scripts/study_dump.py > $O/$v.log 2>&1
  echo "$v rc=$?"; grep -v amdgpu.ids $O/$v.log
done
echo exit=0
