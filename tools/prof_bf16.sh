set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bf16 -o run -- python3 bench.py --only-secondary --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_bf16.log 2>&1
