# per-op microbenchmarks (ours vs hipBLASLt / MIOpen) -> gpurun_out/<tag>/opbench_*.log
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-ops}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for s in ${*:-gemm conv}; do
  timeout -k 10 300 python -u tools/opbench.py $s > $OUT/opbench_$s.log 2>&1 || exit 1
done
