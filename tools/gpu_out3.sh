set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "out3" -x -q --timeout 120 --timeout-method thread > gpurun_out/out3_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/opbench.py out3 > gpurun_out/opbench_out3.log 2>&1
