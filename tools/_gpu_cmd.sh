set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD; OUT=$ROOT/gpurun_out/graph2; mkdir -p $OUT
for i in 1 2 3; do
BM_BUILD_GRAPH=0 timeout -k 10 120 python tools/build_bench.py bunny,merged_proxy >> $OUT/graph0.log 2>&1 || exit 3
BM_BUILD_GRAPH=1 timeout -k 10 120 python tools/build_bench.py bunny,merged_proxy >> $OUT/graph1.log 2>&1 || exit 4
done
echo ok
