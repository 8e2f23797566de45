# k_front throughput vs resident workgroups per CU (DMMT_FRONT_PER_CU knob)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/occ
for n in 1 2 3 4; do
  DMMT_FRONT_PER_CU=$n timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/occ/p$n -o run --output-format csv -- python bench.py --steps 30 --warmup 5 --cpu-seconds 0 > gpurun_out/occ/b$n.json 2> gpurun_out/occ/b$n.err || exit 1
done
echo exit=0
