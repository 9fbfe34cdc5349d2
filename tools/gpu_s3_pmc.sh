# PMC evidence for the SPLIT3 attention (one gpurun call): HBM traffic of the bench's attention launches
# (FETCH_SIZE / WRITE_SIZE passes -> tools/pmc_traffic.py) and the issue counters of attn_s3_kernel at
# 512^2 B8 (tools/attn_only.py s3).  usage: bash tools/gpu_s3_pmc.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-s3pmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --no-cpu-baseline --no-train --steps 2 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || exit 4
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --no-cpu-baseline --no-train --steps 2 --warmup 1 > $OUT/pmc_write.log 2>&1 || exit 5
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $OUT/pmc_s3_1 -o run -- python3 tools/attn_only.py s3 > $OUT/pmc_s3_1.log 2>&1 || exit 6
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU --output-format csv -d $OUT/pmc_s3_2 -o run -- python3 tools/attn_only.py s3 > $OUT/pmc_s3_2.log 2>&1 || exit 7
echo "gpu_s3_pmc done"
