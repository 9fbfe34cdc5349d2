# per-config kernel-time profiles of the bench (bf16 1024^2 B4, then fp32 512^2 B8)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bf16 -o run -- python3 bench.py --only-secondary --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_bf16.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f32 -o run -- python3 bench.py --no-secondary --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_f32.log 2>&1
