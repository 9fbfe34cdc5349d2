set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05i; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_ops.py -m gpu -v --timeout 300 --timeout-method thread -k "loss" > $OUT/tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
timeout -k 10 200 python -u tools/loss_attn_time.py > $OUT/loss_attn_time.log 2>&1 || exit 2
echo done
