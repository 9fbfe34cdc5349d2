set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05h; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_attn.py tests/test_gpu_train.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
ITERS=5 timeout -k 10 200 python -u tools/dkv_only.py > $OUT/dkv.log 2>&1 || exit 2
echo done
