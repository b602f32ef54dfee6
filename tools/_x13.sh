set -u
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for pa in 24 0 8 48; do
echo "prio_after=$pa"; BM_TRACE_PRIO_AFTER=$pa timeout -k 10 120 python tools/variant_ab.py 12 bunny,armadillo_proxy 40 2>&1 | grep v12 || exit $?
done
for lvl in 1 3; do
echo "prio_level=$lvl"; BM_TRACE_PRIO_LEVEL=$lvl timeout -k 10 120 python tools/variant_ab.py 12 bunny,armadillo_proxy 40 2>&1 | grep v12 || exit $?
done
