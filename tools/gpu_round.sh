# Standard GPU evidence run (one gpurun call): pytest -m gpu, the default bench line, a
# rocprofv3 kernel trace of the inference configs, and two PMC passes (FETCH_SIZE, WRITE_SIZE)
# for the attention kernel's HBM traffic.  Outputs under gpurun_out/<tag>/.
#   usage: [TESTS="tests/x.py ..."] bash tools/gpu_round.sh <tag> [tests|bench|prof|pmc|train|trainprof ...]
#   (default: tests bench prof pmc)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-run}; shift
STEPS=${*:-tests bench prof pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    # test FAILURES (pytest rc 1) do not stop the run; a crash, fault or time-out (any other rc) does
    tests) timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1 ;;
    bench) timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || exit 2 ;;
    prof) timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-train > $OUT/prof_bench.log 2>&1 || exit 3 ;;
    pmc) timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --no-cpu-baseline --no-train --steps 2 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || exit 4
         timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --no-cpu-baseline --no-train --steps 2 --warmup 1 > $OUT/pmc_write.log 2>&1 || exit 5 ;;
    train) timeout -k 10 400 python -u bench.py --train --steps 5 --warmup 2 > $OUT/train.log 2>&1 || exit 6 ;;
    trainprof) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trainprof -o run -- python3 bench.py --train --steps 3 --warmup 1 > $OUT/trainprof.log 2>&1 || exit 7 ;;
  esac
done
echo "gpu_round $TAG done"
