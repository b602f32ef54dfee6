set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/x3
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1; shift; echo "== $name"; timeout -k 10 200 "$@" > gpurun_out/x3/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/x3/$name.log | tail -12; [ $rc -lt 124 ] || exit $rc; }
run ab_sched1 python tools/variant_ab.py 6,10 bunny,armadillo_proxy,merged_proxy 30
AB_SHADOW=1 run ab_sched1_shadow python tools/variant_ab.py 6,10 bunny,merged_proxy 30
BM_TRACE_SCHED=0 run ab_sched0 python tools/variant_ab.py 6,10 bunny,armadillo_proxy 30
for g in 1024 1280 1536; do BM_TRACE_GRID=$g run ab_grid$g python tools/variant_ab.py 6,10 bunny,armadillo_proxy 30; done
