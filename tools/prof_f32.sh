set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f32 -o run -- python3 bench.py --no-secondary --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_f32.log 2>&1 && \
timeout -k 10 300 python -u tools/opbench.py conv > gpurun_out/opbench_conv.log 2>&1
