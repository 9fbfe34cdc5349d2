set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05m; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "out3 or full_size" > $OUT/tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u tools/opbench.py out3 > $OUT/out3.log 2>&1 || exit 2
echo done
