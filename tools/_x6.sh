set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/x6
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > gpurun_out/x6/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/x6/$name.log | tail -15; [ $rc -lt 124 ] || exit $rc; }
run tests python -u -m pytest tests/test_gpu_variants.py -x -q --timeout 300
run ab python tools/variant_ab.py 10,12 bunny,armadillo_proxy,merged_proxy 50
ROOT=$(pwd)
(cd /tmp && export TMPDIR=/tmp && BM_TRACE_VARIANT=12 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/x8_bunny -o k -- python3 $ROOT/tools/trace_once.py bunny 20 > $ROOT/gpurun_out/x8_bunny.log 2>&1) || exit $?
grep -h "k_cull\|k_trace_rays" $ROOT/gpurun_out/x8_bunny/k_kernel_stats.csv | cut -c1-140
