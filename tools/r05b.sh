set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05b; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -v --timeout 120 --timeout-method thread -k "gemm_f32_persistent or upsample2x or linear or c64 or conv3x3" > $OUT/tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u tools/opbench.py gemmk32 > $OUT/opbench_gemmk32.log 2>&1 || exit 2
echo done
