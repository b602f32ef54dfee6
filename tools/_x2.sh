set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/x2
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1; shift; echo "== $name"; timeout -k 10 200 "$@" > gpurun_out/x2/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/x2/$name.log | tail -12; [ $rc -lt 124 ] || exit $rc; }
run ab_default python tools/variant_ab.py 6,10,11 bunny,armadillo_proxy,merged_proxy 30
for rm in 1 4 12 16; do BM_TRACE_REFILL_MIN=$rm run ab_refill$rm python tools/variant_ab.py 6,11 bunny,armadillo_proxy 30; done
for g in 768 1024 1280 1536; do BM_TRACE_GRID=$g run ab_grid$g python tools/variant_ab.py 6,10,11 bunny,armadillo_proxy 30; done
