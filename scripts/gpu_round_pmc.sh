# A round's evidence in one call: the bench workload's PMC passes (HBM bytes, VALU /
# SALU / LDS counters) into gpurun_out/pmc_4k444q90.json -- copied into profiles/ on
# the box so that the bench line's roofline reads this build's counters -- then the
# PPM ingest's PMC passes, then gpu_round.sh (smoke, every -m gpu test, the bench
# line, rocprof of it).
# usage: bash scripts/gpu_round_pmc.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-round}
bash scripts/gpu_traffic.sh ${T}_pmc || exit 1
python scripts/pmc_json.py gpurun_out/pmc/${T}_pmc gpurun_out/${T}_pmc_4k444q90.json 4k444q90 > gpurun_out/${T}_pmc_bytes.txt || exit 1
cp gpurun_out/${T}_pmc_4k444q90.json profiles/pmc_4k444q90.json
bash scripts/gpu_pmc_ppm.sh ${T}_ppmpmc > gpurun_out/${T}_ppm_pmc.txt || exit 1
bash scripts/gpu_round.sh $T || exit 1
echo exit=0
