set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/x1
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1; shift; echo "== $name"; timeout -k 10 200 "$@" > gpurun_out/x1/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/x1/$name.log | tail -8; [ $rc -lt 124 ] || exit $rc; }
run ab_default python tools/variant_ab.py 6,10 bunny,armadillo_proxy 30
AB_SHADOW=1 run ab_shadow python tools/variant_ab.py 6,10 bunny,merged_proxy 30
BM_TRACE_GRID=1024 run ab_grid1024 python tools/variant_ab.py 6,10 bunny,armadillo_proxy 30
BM_TRACE_GRID=512 run ab_grid512 python tools/variant_ab.py 6,10 bunny,armadillo_proxy 30
BM_TRACE_PRIO_AFTER=8 run ab_prio8 python tools/variant_ab.py 6,10 bunny,armadillo_proxy 30
BM_TRACE_PRIO_AFTER=1000000 run ab_noprio python tools/variant_ab.py 6,10 bunny,armadillo_proxy 30
bash tools/pmc_compare.sh x1/pmc 6,10 bunny > gpurun_out/x1/pmc.log 2>&1; echo "pmc rc=$?"; tail -80 gpurun_out/x1/pmc.log
