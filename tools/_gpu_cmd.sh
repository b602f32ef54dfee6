set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD; OUT=$ROOT/gpurun_out/cq; mkdir -p $OUT
BM_TRACE_VARIANT=14 timeout -k 10 280 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_00_configs.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || exit 1
for i in 1 2; do
for cfg in c2 c3 filled; do
BM_TRACE_VARIANT=14 timeout -k 10 120 python bench.py --config $cfg --only single --no-extra --no-cpu-baseline --pmc off --steps 60 > $OUT/cq_${cfg}_$i.log 2>&1 || exit 3
timeout -k 10 120 python bench.py --config $cfg --only single --no-extra --no-cpu-baseline --pmc off --steps 60 > $OUT/q_${cfg}_$i.log 2>&1 || exit 4
done; done
echo ok
