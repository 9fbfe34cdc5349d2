set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05d; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_kernels.py -m gpu -v --timeout 120 --timeout-method thread -k "loss_attn or attn or gemm_f32" > $OUT/tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u tools/loss_attn_time.py > $OUT/loss_attn_time.log 2>&1 || exit 2
echo done
