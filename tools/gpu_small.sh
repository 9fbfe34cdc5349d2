set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "vit_batch or instnorm" -x -q --timeout 120 --timeout-method thread > gpurun_out/small_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_steps -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_steps.log 2>&1
