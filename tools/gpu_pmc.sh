# rocprofv3 evidence for the bench line: kernel-trace stats of the default bench command, then two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) for the attention kernel's HBM traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 && \
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/pmc_write.log 2>&1
