# kernel-time profile of the training step (bench --train, 3 timed + 1 warmup)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o run -- python3 bench.py --train --steps 3 --warmup 1 > gpurun_out/prof_train.log 2>&1
