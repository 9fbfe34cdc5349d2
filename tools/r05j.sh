set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05j; mkdir -p $OUT
timeout -k 10 300 python -u tools/opbench.py gemm > $OUT/gemm.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/opbench.py conv > $OUT/conv.log 2>&1 || exit 2
echo done
