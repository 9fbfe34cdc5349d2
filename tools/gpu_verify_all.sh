# full GPU check: pytest -m gpu, the default bench line, then the training bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --train --steps 5 --warmup 2 > gpurun_out/train_hip.log 2>&1
