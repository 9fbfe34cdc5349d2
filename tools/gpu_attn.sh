set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "mhada" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 && \
timeout -k 10 240 python -u tools/attn_ab.py > gpurun_out/attn_ab.log 2>&1
