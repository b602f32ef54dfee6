set -e
ROOT=$PWD
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 200 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy > gpurun_out/bb.log 2>&1
cd /tmp && export TMPDIR=/tmp
for sc in bunny merged_proxy; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/bprof_$sc -o b -- python3 $ROOT/tools/build_bench.py $sc > $ROOT/gpurun_out/bprof_$sc.log 2>&1
done
