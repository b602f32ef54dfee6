set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD; OUT=$ROOT/gpurun_out/kdcooppmc; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  --output-format csv -d $OUT/p1 -o p -- python3 $ROOT/tools/prof_refmode.py c2 2 1 > $OUT/p1.log 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH \
  --output-format csv -d $OUT/p2 -o p -- python3 $ROOT/tools/prof_refmode.py c2 2 1 > $OUT/p2.log 2>&1 || exit 5
echo ok
