set -u
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
BM_TRACE_VARIANT=10 PMC_GROUPS=tools/pmc_compact.txt bash tools/pmc_trace.sh pmc_v10 bunny || exit $?
BM_TRACE_VARIANT=12 PMC_GROUPS=tools/pmc_compact.txt bash tools/pmc_trace.sh pmc_v12 bunny || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_v10 > gpurun_out/pmc_v10/summary.txt
python3 tools/pmc_summary.py gpurun_out/pmc_v12 > gpurun_out/pmc_v12/summary.txt
