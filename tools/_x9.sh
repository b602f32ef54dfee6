set -u
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
BM_TRACE_VARIANT=12 PMC_GROUPS=tools/pmc_mem.txt bash tools/pmc_trace.sh pmc_mem12 bunny || exit $?
BM_TRACE_VARIANT=10 PMC_GROUPS=tools/pmc_mem.txt bash tools/pmc_trace.sh pmc_mem10 bunny || exit $?
sed -i 's/if "k_trace" not in k:/if "k_trace" not in k and "k_cull" not in k:/' tools/pmc_summary.py
python3 tools/pmc_summary.py gpurun_out/pmc_mem12 > gpurun_out/pmc_mem12/summary.txt
python3 tools/pmc_summary.py gpurun_out/pmc_mem10 > gpurun_out/pmc_mem10/summary.txt
