set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hash
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_hash.py -x -v --timeout 300 --timeout-method thread > gpurun_out/hash/tests.log 2>&1; rc=$?
tail -25 gpurun_out/hash/tests.log
[ $rc -lt 124 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/hash/bench.log 2>&1; rc=$?
tail -1 gpurun_out/hash/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['hashed_grid'], d['reference_mode'])"
exit $rc
