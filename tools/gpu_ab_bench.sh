# A/B of an env switch on the whole bench: runs bench.py alternately with $AB_VAR unset / =${AB_OFF:-0}
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/ab_bench.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ab_on_$i.log 2>&1 || exit 1
  env $AB_VAR=${AB_OFF:-0} timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ab_off_$i.log 2>&1 || exit 1
done
