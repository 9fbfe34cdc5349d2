# training attention kernels: parity tests, golden train step, then train-step time hip vs torch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_attn.py -x -v --timeout 120 --timeout-method thread > gpurun_out/train_attn_tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread > gpurun_out/train_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --train --steps 3 --warmup 1 > gpurun_out/train_hip.log 2>&1 && \
MHADA_TRAIN_ATTN=torch timeout -k 10 300 python -u bench.py --train --steps 3 --warmup 1 > gpurun_out/train_torch.log 2>&1
