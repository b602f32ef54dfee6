set -u
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$(pwd)
for lib in libbeam_hip.so libbeam_hip_nostore.so; do
(cd /tmp && export TMPDIR=/tmp && BEAM_HIP_LIB=$ROOT/raytracercuda_amd/$lib BM_TRACE_VARIANT=12 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/x12_$lib -o k -- python3 $ROOT/tools/trace_once.py bunny 20 > $ROOT/gpurun_out/x12_$lib.log 2>&1) || exit $?
echo $lib; grep -h "k_cull\|k_trace_rays" $ROOT/gpurun_out/x12_$lib/k_kernel_stats.csv | cut -c1-140
done
