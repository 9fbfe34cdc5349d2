# per-op microbenchmarks (ours vs hipBLASLt) and a kernel-trace profile of the bf16 1024^2 bench config
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/opbench.py gemm > gpurun_out/opbench_gemm.log 2>&1 && \
timeout -k 10 300 python -u tools/opbench.py conv > gpurun_out/opbench_conv.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bf16 -o run -- python3 bench.py --only-secondary --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_bf16.log 2>&1
