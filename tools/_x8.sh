set -u
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$(pwd)
for sc in bunny merged_proxy; do
(cd /tmp && export TMPDIR=/tmp && BM_TRACE_VARIANT=12 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/x8_$sc -o k -- python3 $ROOT/tools/trace_once.py $sc 20 > $ROOT/gpurun_out/x8_$sc.log 2>&1) || exit $?
grep -h "k_cull\|k_trace_rays\|k_trace_quad" $ROOT/gpurun_out/x8_$sc/k_kernel_stats.csv | cut -c1-200
done
