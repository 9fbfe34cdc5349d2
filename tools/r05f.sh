set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05f; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -v --timeout 120 --timeout-method thread -k "wino" > $OUT/tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u tools/wino_ab.py ablate > $OUT/wino_ablate.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/wino_ab.py > $OUT/wino_ab.log 2>&1 || exit 3
echo done
