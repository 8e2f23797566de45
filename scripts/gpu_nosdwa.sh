# SDWA peephole off (the k_emit fault study): bench A/B and the parity suite on the variant
set -o pipefail
bash scripts/gpu_bench_variants.sh 4k444q90 "base nosdwa" 3 && \
bash scripts/gpu_bench_variants.sh 8k420q75 "base nosdwa" 2 && \
DMMT_LIB_PATH=$PWD/dmmt-jpeg-encoder_amd/lib_nosdwa/libdmmt_jpeg.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "parity or fuzz or restart" > gpurun_out/nosdwa_tests.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/nosdwa_tests.log
