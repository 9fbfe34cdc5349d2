set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/proj_pmc
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/proj_only.py bf16 > $OUT/kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p1 -o run -- python3 tools/proj_only.py bf16 4 16384 5 > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p2 -o run -- python3 tools/proj_only.py bf16 4 16384 5 > $OUT/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p3 -o run -- python3 tools/proj_only.py f32 8 4096 5 > $OUT/p3.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p4 -o run -- python3 tools/proj_only.py f32 8 4096 5 > $OUT/p4.log 2>&1 || exit 1
echo done
