# SPLIT3 fp32 attention evidence (one gpurun call): its kernel tests (fp64 accuracy, late max jump,
# plane image) and the interleaved A/B against the fp32-MFMA kernel (tools/attn_s3_ab.py).
#   usage: bash tools/gpu_s3.sh <tag> [tests ab golden]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-s3}; shift
STEPS=${*:-tests ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    # test FAILURES (pytest rc 1) do not stop the run; a crash, fault or time-out (any other rc) does
    tests) timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -v --timeout 120 --timeout-method thread -k "split3 or attn_late or mhada_block" > $OUT/s3_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1 ;;
    golden) timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 3 ;;
    ab) timeout -k 10 400 python -u tools/attn_s3_ab.py ${S3_WAVES:-0} > $OUT/s3_ab.log 2>&1 || exit 2 ;;
  esac
done
echo "gpu_s3 $TAG done"
