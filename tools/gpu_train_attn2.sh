# training attention: parity tests, train bench, then kernel-trace profile of the train step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_attn.py -x -v --timeout 120 --timeout-method thread > gpurun_out/train_attn_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --train --steps 3 --warmup 1 > gpurun_out/train_hip.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o run -- python3 bench.py --train --steps 3 --warmup 1 > gpurun_out/prof_train.log 2>&1
