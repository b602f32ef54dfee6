set -u
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$(pwd)
mkdir -p gpurun_out/pcs
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 60 rocprofv3 -L > $ROOT/gpurun_out/pcs/list.txt 2>&1; echo "list rc=$?")
(cd /tmp && export TMPDIR=/tmp && BM_TRACE_VARIANT=12 timeout -k 10 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 --output-format csv -d $ROOT/gpurun_out/pcs/s -o pcs -- python3 $ROOT/tools/trace_once.py bunny 20 > $ROOT/gpurun_out/pcs/run.log 2>&1; echo "pcs rc=$?")
ls -la gpurun_out/pcs/s 2>/dev/null | head
