# HBM traffic of the bench's GEMM shapes: FETCH_SIZE and WRITE_SIZE passes of
# tools/gemm_traffic_shapes.py (separate --pmc runs), then tools/gemm_traffic_sum.py.
#   usage: bash tools/gemm_traffic.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-gemmtraffic}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 tools/gemm_traffic_shapes.py > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 tools/gemm_traffic_shapes.py > $OUT/write.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 tools/gemm_traffic_shapes.py > $OUT/trace.log 2>&1 || exit 3
python3 tools/gemm_traffic_sum.py $OUT > $OUT/summary.txt 2>&1 || exit 4
echo gemm_traffic done
