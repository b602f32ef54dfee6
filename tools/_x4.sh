set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/x4
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1; shift; echo "== $name"; timeout -k 10 200 "$@" > gpurun_out/x4/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/x4/$name.log | tail -12; [ $rc -lt 124 ] || exit $rc; }
for pa in 8 16 40 1000000; do BM_TRACE_PRIO_AFTER=$pa run ab_prio$pa python tools/variant_ab.py 10 bunny,armadillo_proxy,merged_proxy 40; done
for pl in 1 3; do BM_TRACE_PRIO_LEVEL=$pl run ab_plevel$pl python tools/variant_ab.py 10 bunny,armadillo_proxy,merged_proxy 40; done
for g in 1024 1280 1536 1792; do BM_TRACE_GRID=$g run ab_grid$g python tools/variant_ab.py 10 bunny,armadillo_proxy,merged_proxy 40; done
