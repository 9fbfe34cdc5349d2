# PMC counter groups (one rocprofv3 pass per group) on one program:
#   bash tools/gpu_pmc.sh <tag> <program args...>      e.g. tools/attn_only.py bf16 | tools/gemm_only.py bf16 65536 1536 512
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 "$@" > $OUT/p$i.log 2>&1 || exit 1
done
echo done
