set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05g; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || exit 2
echo done
