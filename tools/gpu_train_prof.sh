set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/train_probe.py bench0 prof > gpurun_out/train_probe.log 2>&1
