# The k_emit "wrong bits at the head of a wave's first block" study:
# the 8K 4:2:0 q95 encode repeated with (1) the round-2 WIP build that showed it
# (study_wip/: commit 71130cf with the zigzag permutation taken out again),
# (2) the current tree with the walk straight over the column-major registers
# (lib_colmajor), (3) the current product library.  No GPU fault is involved:
# wrong bytes only; every step runs under its own time limit.
set -o pipefail
O=gpurun_out/fault
mkdir -p $O
( cd study_wip && timeout -k 10 240 python scripts/debug_determinism.py --n 4 ) > $O/wip.log 2>&1; echo "wip rc=$?"; cat $O/wip.log | grep -v amdgpu.ids
DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_colmajor/libdmmt_jpeg.so timeout -k 10 240 python tests/tools/determinism.py --n 4 > $O/colmajor.log 2>&1; echo "colmajor rc=$?"; grep -v amdgpu.ids $O/colmajor.log
timeout -k 10 240 python tests/tools/determinism.py --n 2 > $O/product.log 2>&1; echo "product rc=$?"; grep -v amdgpu.ids $O/product.log
echo exit=0
