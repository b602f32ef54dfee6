set -u
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$(pwd)
for t in 8 16 32 64; do
(cd /tmp && export TMPDIR=/tmp && BM_CULL_TPR=$t BM_TRACE_VARIANT=12 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/x15_$t -o k -- python3 $ROOT/tools/trace_once.py bunny 20 > $ROOT/gpurun_out/x15_$t.log 2>&1) || exit $?
echo tpr=$t; grep -h "k_cull\|k_trace_rays" $ROOT/gpurun_out/x15_$t/k_kernel_stats.csv | cut -c1-140
done
