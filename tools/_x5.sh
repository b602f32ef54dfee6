set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/x5
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > gpurun_out/x5/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/x5/$name.log | tail -12; [ $rc -lt 124 ] || exit $rc; }
run ab python tools/variant_ab.py 6,10 bunny,armadillo_proxy,merged_proxy 50
run tests python -u -m pytest tests/test_gpu_variants.py -x -q --timeout 300
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/x5/w -o w -- python3 $GRAFT_REPO_ROOT/tools/trace_once.py bunny 5 > $GRAFT_REPO_ROOT/gpurun_out/x5/w.log 2>&1; echo "pmc rc=$?"
grep k_trace_quad $GRAFT_REPO_ROOT/gpurun_out/x5/w/w_counter_collection.csv | head -3
