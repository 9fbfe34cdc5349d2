set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_train_attn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/train_attn_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/train_attn_bench.py > gpurun_out/train_attn_ab.log 2>&1 && \
MHADA_TRAIN_DKV_OCC=1 timeout -k 10 120 python -u tools/train_attn_bench.py >> gpurun_out/train_attn_ab.log 2>&1
