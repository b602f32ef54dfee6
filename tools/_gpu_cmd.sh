set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v43; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_reference_mode.py > $OUT/tests.log 2>&1
rc=$?; tail -14 $OUT/tests.log; exit $rc
