set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "linear or conv or gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/opbench.py gemm > gpurun_out/opbench_gemm.log 2>&1 && \
timeout -k 10 300 python -u tools/opbench.py gemmk > gpurun_out/gemmk.log 2>&1 && \
timeout -k 10 300 python -u tools/opbench.py conv > gpurun_out/opbench_conv.log 2>&1
