set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MHADA_ATTN_KERNEL=fsp MHADA_ATTN_TK=128 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "mhada and not late_max" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 && \
timeout -k 10 240 python -u tools/attn_ab.py > gpurun_out/attn_ab.log 2>&1
