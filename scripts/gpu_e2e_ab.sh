# parity suite, then the PCIe-inclusive host-batch rate (dmmt_jpeg_encode_batch) of the
# current library for each config; the loop over variants keeps only 'default' since
# the frame pipeline was reverted (A/B runs build the variant libraries themselves)
set -o pipefail
mkdir -p gpurun_out/e2e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/e2e/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/e2e/gpu_tests.log; exit 1; }
tail -1 gpurun_out/e2e/gpu_tests.log
for cfg in "4k444q90 --batch 8" "4k444q90 --batch 1" "${E2E_CFG2:-1080p420q75x256 --batch 64}"; do
  for p in default; do
    timeout -k 10 120 python scripts/e2e_rate.py --config $cfg --seconds 4 >> gpurun_out/e2e/rates.jsonl 2>> gpurun_out/e2e/rates.err || { echo "e2e $cfg $p failed"; tail gpurun_out/e2e/rates.err; exit 1; }
    tail -1 gpurun_out/e2e/rates.jsonl
  done
done
