set -o pipefail
mkdir -p gpurun_out
python -c "import torch,sys; print(torch.__version__, torch.cuda.is_available())" > gpurun_out/env.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
echo "exit=$?"
