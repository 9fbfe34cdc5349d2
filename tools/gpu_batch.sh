# One gpurun call for a batch of round-4 checks; every GPU step under its own time limit, chained
# so that a failure (fault, abort, time-out) ends the call.  usage: bash tools/gpu_batch.sh <tag> <step>...
#   attn       attention variant tests + A/B + in-kernel clocks (bf16 variants and fp32)
#   c64        decoder conv3.0 fused vs split upsample (tools/c64_ab.py)
#   newtests   the round-4 GPU tests (ingest, graphs, training forward / folds / 512^2 B1 losses)
#   gpu        the whole pytest -m gpu suite
#   bench      the default bench line
#   trainclock in-kernel clock of the training dK/dV' kernel (diagnostic build)
#   vit        the ViT / batched-training tests (LinearFn residual, batched ViT / AdaFormer, goldens)
#   winotests / winoab  the Winograd conv tests / knob A/B (WINO_KNOB, default wino4)
#   train / trainprof  the training step bench line / its rocprofv3 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu"
for s in "$@"; do
  case $s in
    attn) bash tools/gpu_attn.sh $TAG tests ab clock || exit 1
          timeout -k 10 120 python -u tools/attn_clock.py f32 > $OUT/attn_clock_f32.log 2>&1 || exit 1 ;;
    c64) timeout -k 10 120 python -u tools/c64_ab.py > $OUT/c64_ab.log 2>&1 || exit 2 ;;
    trainclock) timeout -k 10 180 python -u tools/attn_clock.py dkv > $OUT/train_clock.log 2>&1 || exit 6 ;;
    winoab) timeout -k 10 300 python -u tools/wino_knob_ab.py ${WINO_KNOB:-wino4} > $OUT/wino_${WINO_KNOB:-wino4}_ab.log 2>&1 || exit 9 ;;
    vit) timeout -k 10 600 $PYT tests/test_gpu_train_ops.py tests/test_gpu_train.py -k "linear_fn or vit_training or batch_axis or batched or bit_identical or golden or 256_b2 or rccl" > $OUT/vit_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 15 ;;
    winoab2) timeout -k 10 400 python -u tools/wino_knob_ab.py -c wino4=0 -c wino4=1 > $OUT/wino_ab2.log 2>&1 || exit 9 ;;
    winopk) timeout -k 10 300 $PYT tests/test_gpu_kernels.py -k "wino_persistent" > $OUT/wino_pk_tests.log 2>&1 || exit 14 ;;
    winotests) timeout -k 10 300 $PYT tests/test_gpu_kernels.py tests/test_gpu_train_ops.py -k "wino or chain" > $OUT/wino_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 11 ;;
    winodbg) for shp in ${WINO_DBG_SHAPES:-"8 128 256 256" "8 256 128 128" "8 64 512 512"}; do
               WINO_KNOB_VALS=${WINO_KNOB_VALS:-0,1} WINO_LIB_DIR=diag/wino_dbg timeout -k 10 120 python -u tools/wino_dbg.py $shp 0 1 2 4 6 >> $OUT/wino_dbg.log 2>&1 || exit 12
             done ;;
    winopmc) for v in ${WINO_KNOB_VALS//,/ }; do
               timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d $OUT/winopmc_$v -o run -- python3 tools/wino_only.py $v > $OUT/winopmc_$v.log 2>&1 || exit 13
               timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/winopmc2_$v -o run -- python3 tools/wino_only.py $v > $OUT/winopmc2_$v.log 2>&1 || exit 13
               timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d $OUT/winopmc3_$v -o run -- python3 tools/wino_only.py $v > $OUT/winopmc3_$v.log 2>&1 || exit 13
             done ;;
    lapmc) timeout -k 10 120 python -u tools/lossattn_only.py 5 > $OUT/lossattn_time.log 2>&1 || exit 16
           timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d $OUT/lapmc -o run -- python3 tools/lossattn_only.py 2 > $OUT/lapmc.log 2>&1 || exit 16
           timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/lapmc2 -o run -- python3 tools/lossattn_only.py 2 > $OUT/lapmc2.log 2>&1 || exit 16 ;;
    dkvpmc) for v in 0 1; do
              timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d $OUT/dkvpmc_$v -o run -- python3 tools/dkv_only.py $v > $OUT/dkvpmc_$v.log 2>&1 || exit 10
              timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/dkvpmc2_$v -o run -- python3 tools/dkv_only.py $v > $OUT/dkvpmc2_$v.log 2>&1 || exit 10
            done ;;
    train) timeout -k 10 400 python -u bench.py --train --steps 5 --warmup 2 > $OUT/train.log 2>&1 || exit 7 ;;
    trainprof) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trainprof -o run -- python3 bench.py --train --steps 3 --warmup 1 > $OUT/trainprof.log 2>&1 || exit 8 ;;
    # test FAILURES (pytest rc 1) do not stop the batch; a crash, fault or time-out (any other rc) does
    newtests) timeout -k 10 900 $PYT tests/test_ingest.py tests/test_gpu_parity.py tests/test_gpu_train_attn.py tests/test_gpu_train_ops.py tests/test_gpu_train.py tests/test_gpu_kernels.py -k "ingest or graphed or default_path or full_size or fwd_kernels or chain or vgg19_and_decoder or 512_b1 or golden or n64 or bit_identical or feature_loss or mlp_relu or tile_counts or late_max" > $OUT/new_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 3 ;;
    gpu) timeout -k 10 1000 $PYT tests > $OUT/gpu_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 4 ;;
    bench) timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || exit 5 ;;
  esac
done
echo "gpu_batch $TAG done"
