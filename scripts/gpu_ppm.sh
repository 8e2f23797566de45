# Round-4 PPM ingest check: the PPM / CLI / convert GPU tests, the ppm_ingest
# timing of bench.py (scripts/ppm_probe.py) and a rocprofv3 kernel profile of it.
# usage: bash scripts/gpu_ppm.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-ppm}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "ppm or cli or convert" > $O/ppm_tests.log 2>&1 || { echo "ppm tests failed"; tail -40 $O/ppm_tests.log; exit 1; }
tail -1 $O/ppm_tests.log
timeout -k 10 120 python scripts/ppm_probe.py 200 > $O/ppm_probe.json 2> $O/ppm_probe.err || { echo "probe failed"; tail -5 $O/ppm_probe.err; exit 1; }
cat $O/ppm_probe.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/ppm_probe.py 50 > $O/prof.log 2>&1 || { echo "profile failed"; tail -5 $O/prof.log; exit 1; }
python scripts/kstats.py $(find $O/prof -name run_kernel_stats.csv | head -1)
echo exit=0
