# k_emit fault study, step 4: every chunk's assembled window vs its slots.
set -o pipefail
O=$PWD/gpurun_out/fault4
mkdir -p $O
cd study_wip
DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_dump2/libdmmt_jpeg.so timeout -k 10 400 python scripts/study_dump2.py > $O/dump2.log 2>&1
echo "dump2 rc=$?"; grep -v amdgpu.ids $O/dump2.log
echo exit=0
