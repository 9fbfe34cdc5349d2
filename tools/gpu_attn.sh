# bf16 attention variant evidence (one gpurun call): the attention variant tests, the interleaved
# variant A/B (tools/attn_ab.py), the in-kernel clock of each variant (tools/attn_clock.py, the
# -DATTN_CLOCK diagnostic build) and a PMC pass per counter group of each variant at 1024^2 B4.
#   usage: bash tools/gpu_attn.sh <tag> [tests ab clock pmc]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-attn}; shift
STEPS=${*:-tests ab clock pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "attn" > $OUT/attn_tests.log 2>&1 || exit 1 ;;
    ab) ATTN_AB_NO_F32=1 timeout -k 10 300 python -u tools/attn_ab.py > $OUT/attn_ab.log 2>&1 || exit 2 ;;
    clock) timeout -k 10 300 python -u tools/attn_clock.py ${CLOCK_VARIANTS:-fsg fsq1 fsp} > $OUT/attn_clock.log 2>&1 || exit 3 ;;
    pmc) for v in ${PMC_VARIANTS:-fsg fsq1 fsp}; do
           i=0
           for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"; do
             i=$((i+1))
             timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_${v}_$i -o run -- python3 tools/attn_only.py bf16 $v > $OUT/pmc_${v}_$i.log 2>&1 || exit 4
           done
         done ;;
  esac
done
echo "gpu_attn $TAG done"
