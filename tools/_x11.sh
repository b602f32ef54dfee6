set -u
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for g in 256 512 1024; do
echo "== grid $g"
BM_TRACE_GRID=$g BM_TRACE_VARIANT=12 timeout -k 10 120 python tools/wave_timeline.py bunny 2>&1 | grep -v amdgpu.ids | head -6 || exit $?
done
for g in 256 512 1024 1280 1792; do
BM_TRACE_GRID=$g timeout -k 10 120 python tools/variant_ab.py 12 bunny 30 2>&1 | grep "v12" || exit $?
done
